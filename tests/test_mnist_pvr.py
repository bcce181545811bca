"""MNIST-PVR task (reference tests/test_datasets.py + HL/corr/alignment/train smoke), offline synthetic digits."""
import numpy as np
import torch
from torch.utils.data import Dataset

from iit_amd.core.index import Ix
from iit_amd.tasks.mnist_pvr import MNIST_CLASS_MAP, ImagePVRDataset, MNIST_PVR_HL, MNIST_PVR_Leaky_HL
from iit_amd.tasks.mnist_pvr.digits import SyntheticMNIST


class SmallMNIST(Dataset):
    def __init__(self, images, labels):
        self.images, self.labels = images, labels

    def __len__(self):
        return len(self.images)

    def __getitem__(self, i):
        return self.images[i], self.labels[i]


def create_small_mnist():
    base = SyntheticMNIST(train=True, size=500)
    images, labels = [], []
    np.random.seed(0)
    while len(images) < 10:
        image, label = base[np.random.randint(0, len(base))]
        if label not in labels:
            images.append(image)
            labels.append(label)
    return SmallMNIST(images, labels)


def test_get_input_shape():
    ds = ImagePVRDataset(create_small_mnist(), length=1, pad_size=3, device="cpu")
    assert ds.get_input_shape() == (1, 3, (28 + 3 * 2) * 2, (28 + 3 * 2) * 2)
    assert ds[0][0].shape == (3, 68, 68)


def test_patch_quadrant():
    np.random.seed(1)
    ds = ImagePVRDataset(create_small_mnist(), length=1, pad_size=0, device="cpu")
    image, label, iv = ds[0]
    hl = MNIST_PVR_Leaky_HL()
    _, _, w, h = ds.get_input_shape()
    idx = {"tl": Ix[None, :w // 2, :h // 2].as_index, "tr": Ix[None, :w // 2, h // 2:h].as_index,
           "bl": Ix[None, w // 2:w, :h // 2].as_index, "br": Ix[None, w // 2:w, h // 2:h].as_index}
    for q in idx:
        new_imgs, new_labels, new_ivs = ds.patch_batch_at_hl([image], [iv], getattr(hl, f"hook_{q}"))
        for other in idx:
            same = torch.all(new_imgs[0][idx[other]] == image[idx[other]])
            assert bool(same) == (other != q), (q, other)
        k = "tl tr bl br".split().index(q)
        assert new_ivs[0][k] != iv[k]
        assert int(new_labels[0]) == int(new_ivs[0][MNIST_CLASS_MAP[int(new_ivs[0][0])]])


def test_gather_matches_items_and_hl_labels():
    base = SyntheticMNIST(train=False, size=300)
    ds = ImagePVRDataset(base, length=40, pad_size=7, device="cpu")
    x, y, iv = ds.gather(torch.arange(40))
    for i in (0, 7, 39):
        xi, yi, ivi = ds[i]
        assert torch.equal(x[i], xi) and int(y[i]) == int(yi) and torch.equal(iv[i], ivi)
    hl = MNIST_PVR_HL()
    assert torch.equal(hl((x, y, iv)), y)
    assert torch.equal(MNIST_PVR_Leaky_HL()((x, y, iv)), y)


def test_corr_modes_and_leaky_corr():
    from iit_amd.tasks.task_loader import get_alignment
    shape = (1, 3, 84, 84)
    ll, hl, corr = get_alignment("mnist_pvr", {"input_shape": shape, "device": "cpu", "mode": "c"})
    nodes = [next(iter(v)) for v in corr.values()]
    assert [n.index for n in nodes] == [Ix[None, 64 * i:64 * (i + 1), None, None] for i in range(4)]
    _, _, corr_q = get_alignment("mnist_pvr", {"input_shape": shape, "device": "cpu"})
    assert next(iter(corr_q[list(corr_q)[3]])).index == Ix[None, None, 3:6, 3:6]
    _, hl_leaky, corr_l = get_alignment("pvr_leaky", {"input_shape": shape, "device": "cpu"})
    assert len(corr_l) == 12 and len(hl_leaky.hook_dict) == 16
    assert "mod.layer3.mod.1.mod.conv2.hook_point" in ll.hook_dict
    names = [n for n, _ in ll.named_parameters()]
    assert "mod.layer1.mod.0.mod.conv1.mod.weight" in names and "mod.fc.mod.weight" in names


def test_pvr_behavior_pair_trains():
    from iit_amd.model_pairs import IITBehaviorModelPair
    from iit_amd.tasks.task_loader import get_alignment, get_dataset
    torch.manual_seed(0)
    tr, te = get_dataset("mnist_pvr", {"train_size": 32, "test_size": 16, "device": "cpu"})
    ll, hl, corr = get_alignment("mnist_pvr", {"input_shape": te.base_data.get_input_shape(), "device": "cpu"})
    pair = IITBehaviorModelPair(ll_model=ll, hl_model=hl, corr=corr,
                                training_args={"lr": 1e-3, "batch_size": 16, "early_stop": False,
                                               "lr_scheduler": None})
    pair.train(tr, te, epochs=1)
    d = pair.test_metrics.to_dict()
    assert set(d) >= {"val/iit_loss", "val/IIA", "val/accuracy"}
    assert np.isfinite(pair.train_metrics.to_dict()["train/iit_loss"])


def test_patch_batch_tensor_equals_per_sample_patching():
    """The device-side batch patch of the leakiness eval (eval_causality.py) makes the same rng draws in the same order
    as the reference's per-sample ``patch_batch_at_hl`` loop: identical images, labels and intermediate variables."""
    import copy

    from iit_amd.core.nodes import HLNode
    from iit_amd.tasks.task_loader import get_dataset
    _, te = get_dataset("pvr_leaky", dataset_config={"train_size": 1, "test_size": 64})
    ds = te.base_data
    b = ds.gather(torch.arange(0, 16))
    for name in ("hook_tl_leaked_to_tr", "hook_br_leaked_to_tl", "hook_bl_leaked_to_br"):
        node = HLNode(name, 10)
        d1, d2 = copy.deepcopy(ds), copy.deepcopy(ds)
        xs, ys, ivs = d1.patch_batch_at_hl(list(b[0]), list(b[2]), node)
        x2, y2, iv2 = d2.patch_batch_tensor(b[0], b[2], node)
        assert torch.equal(torch.stack(xs), x2), name
        assert torch.equal(torch.stack([torch.as_tensor(y) for y in ys]), y2), name
        assert torch.equal(torch.stack(ivs), iv2), name
