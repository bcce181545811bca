"""IOI task golden values (iit/tasks/ioi/test_ioi.py in the reference) + T2 engine semantics on CPU."""
import numpy as np
import pytest
import torch

from iit_amd.core.nodes import HLNode
from iit_amd.tasks.ioi import IOI_HL, make_ioi_corr, make_ioi_dataset_and_hl
from iit_amd.tasks.ioi.ioi_hl import DuplicateHead, NameMoverHead, PreviousHead, SInhibitionHead

NAMES = torch.tensor([10, 20, 30])


def nz(a):
    return torch.cat((a.nonzero(), a[a != 0][:, None]), dim=-1)


def test_duplicate_head():
    assert DuplicateHead()(torch.tensor([[3, 1, 4, 1, 5, 9, 2, 6, 5]])).equal(
        torch.tensor([[-1, -1, -1, 1, -1, -1, -1, -1, 4]]))


def test_previous_head():
    assert PreviousHead()(torch.tensor([[3, 1, 4, 1, 5, 9, 2, 6, 5]])).equal(
        torch.tensor([[-1, 3, 1, 4, 1, 5, 9, 2, 6]]))


def test_s_inhibition_head():
    a = SInhibitionHead()(torch.tensor([[3, 1, 4, 1, 5, 9, 2, 6, 5]]), torch.tensor([[-1, -1, -1, 1, -1, -1, -1, -1, 4]]))
    assert a.equal(torch.tensor([[-1, -1, -1, 1, -1, -1, -1, -1, 5]]))


def test_name_mover_head():
    a = NameMoverHead(NAMES, d_vocab=21)(torch.tensor([[1, 2, 10, 20]]), torch.tensor([[-1, 20, 10, -1]]))
    assert nz(a[0]).equal(torch.tensor([[1., 20., -15.], [2., 10., -5.], [2., 20., -15.], [3., 10., -5.],
                                        [3., 20., -5.]]))


def test_ioi_hl():
    a = IOI_HL(d_vocab=21, names=NAMES)((torch.tensor([[3, 10, 4, 10, 5, 9, 2, 6, 5]]), None, None))
    assert nz(a[0]).equal(torch.tensor([[1., 10., 10.], [2., 10., 10.], [3., 10., 5.], [4., 10., 5.], [5., 10., 5.],
                                        [6., 10., 5.], [7., 10., 5.], [8., 5., -15.], [8., 10., 5.]]))


def test_ioi_hl_last_only_matches_full():
    hl = IOI_HL(d_vocab=50, names=NAMES)
    tok = torch.randint(0, 50, (16, 12))
    tok[:, 3] = 10
    tok[:, 7] = 10
    full = hl((tok, None, None))
    last = hl((tok, None, None), last_only=True)
    assert torch.equal(full[:, -1], last)


def test_ioi_dataset_contract():
    # enough samples that every name appears as an IO (the HL name set is the IO set, as in the reference)
    ds, hl = make_ioi_dataset_and_hl(2000, None, device="cpu")
    x, y, iv = ds[0]
    assert x.shape == (16,) and y.shape == (16,) and iv.shape == (1,)
    assert torch.equal(x[1:], y[:-1])
    # the HL label at the last position equals the true next token (unpadded prompts)
    xb, yb, _ = ds.gather(torch.arange(64))
    out = hl((xb, yb, None), last_only=True)
    assert (out.argmax(-1) == yb[:, -1]).all()
    ds1h = make_ioi_dataset_and_hl(8, None, device="cpu", label_format="onehot")[0]
    assert ds1h[0][1].shape == (16, 50257)


def test_iit_dataset_pairs_and_loader_order():
    from iit_amd.data.iit_dataset import IITDataset, loader_epoch_permutation
    ds, _ = make_ioi_dataset_and_hl(10, None, device="cpu")
    iitd = IITDataset(ds, ds, seed=0, device="cpu")
    assert [iitd.pair_indices(i) for i in range(6)] == [(8, 6), (4, 5), (8, 2), (8, 0), (7, 9), (6, 8)]  # [OBS]
    torch.manual_seed(123)
    ref_order = [int(i) for b in torch.utils.data.DataLoader(list(range(10)), batch_size=4, shuffle=True) for i in b]
    torch.manual_seed(123)
    assert loader_epoch_permutation(10).tolist() == ref_order


def _pair(cls=None, n_layers=6, **args):
    from iit_amd.model_pairs import IOI_ModelPair
    from iit_amd.models.config import gpt2_config_dict
    from iit_amd.models.transformer import HookedTransformer
    cfg = gpt2_config_dict()
    cfg.update(n_layers=n_layers, d_model=32, n_heads=4, d_head=8, d_mlp=64, device="cpu")
    torch.manual_seed(0)
    ll = HookedTransformer(cfg)
    ds, hl = make_ioi_dataset_and_hl(256, ll, device="cpu")
    cls = cls or IOI_ModelPair
    pair = cls(hl, ll, make_ioi_corr(n_layers), training_args={"batch_size": 64, "lr": 1e-3, "lr_scheduler": None,
                                                                 **args})
    return pair, ds


def test_hl_node_sampling_sequence_matches_reference_generator():
    """Q19: same numpy Generator / call order as the reference (observed sequence at seed 0)."""
    pair, _ = _pair()
    pair.rng = np.random.default_rng(0)
    seq = [pair.sample_hl_name().name for _ in range(12)]
    keys = list(pair.corr.keys())
    rng = np.random.default_rng(0)
    assert seq == [rng.choice(keys).name for _ in range(12)]


def test_native_engine_equals_reference_engine():
    """The plan-driven engine gives the same losses as the reference hook/closure path (fp32)."""
    from iit_amd.data.iit_dataset import IITDataset
    pair, ds = _pair()
    train = IITDataset(ds, ds, seed=0, device="cpu")
    base, abl = next(iter(train.make_loader(64, 0)))
    for hl_node in pair.corr.keys():
        pair.training_args["engine"] = "native"
        l1 = pair.get_IIT_loss_over_batch(base, abl, hl_node, pair.loss_fn)
        pair.training_args["engine"] = "reference"
        l2 = pair.get_IIT_loss_over_batch(base, abl, hl_node, pair.loss_fn)
        assert torch.allclose(l1, l2, atol=1e-5), hl_node
    node = pair.nodes_not_in_circuit[2]
    pair.training_args["engine"] = "native"
    s1 = pair.get_strict_loss_over_batch(base, abl, node, pair.loss_fn)
    pair.training_args["engine"] = "reference"
    s2 = pair.get_strict_loss_over_batch(base, abl, node, pair.loss_fn)
    assert torch.allclose(s1, s2, atol=1e-5)


def test_gradients_native_vs_reference():
    from iit_amd.data.iit_dataset import IITDataset
    pair, ds = _pair()
    train = IITDataset(ds, ds, seed=0, device="cpu")
    base, abl = next(iter(train.make_loader(64, 0)))
    hl_node = list(pair.corr.keys())[2]
    grads = []
    for engine in ("native", "reference"):
        pair.training_args["engine"] = engine
        pair.ll_model.zero_grad(set_to_none=True)
        loss = pair.get_IIT_loss_over_batch(base, abl, hl_node, pair.loss_fn)
        pair.backward(loss)
        grads.append([p.grad.clone() for p in pair.ll_model.parameters()])
    for g1, g2 in zip(*grads):
        assert torch.allclose(g1, g2, atol=1e-5)


def test_do_intervention_verbose(capsys):
    """``verbose=True`` (reference base_model_pair.py:75-100) prints the HL and LL nodes."""
    from iit_amd.data.iit_dataset import IITDataset
    pair, ds = _pair()
    base, abl = next(iter(IITDataset(ds, ds, seed=0, device="cpu").make_loader(8, 0)))
    hl_node = list(pair.corr.keys())[0]
    hl_out, ll_out = pair.do_intervention(base, abl, hl_node, verbose=True)
    assert "ll_nodes=" in capsys.readouterr().out
    assert ll_out.shape[0] == 8


@pytest.mark.parametrize("single", [False, True])
def test_strict_train_step_counts(single):
    from iit_amd.data.iit_dataset import IITDataset
    pair, ds = _pair(use_single_loss=single)
    train = IITDataset(ds, ds, seed=0, device="cpu")
    opt = pair.make_optimizer(1e-3)
    calls = []
    orig = opt.step
    opt.step = lambda *a, **k: (calls.append(1), orig(*a, **k))[1]
    base, abl = next(iter(train.make_loader(64, 0)))
    out = pair.run_train_step(base, abl, pair.loss_fn, opt)
    assert set(out) == {"train/iit_loss", "train/behavior_loss", "train/strict_loss"}
    assert len(calls) == (1 if single else 3)


def test_all_pair_classes_train_one_epoch(tmp_path):
    from iit_amd.data.iit_dataset import IITDataset, train_test_split
    from iit_amd.model_pairs import (FreezedModelPair, IITBehaviorModelPair, IITModelPair, StopGradModelPair,
                                     StrictIITModelPair)
    for cls in (IITBehaviorModelPair, StrictIITModelPair, FreezedModelPair, StopGradModelPair):
        pair, ds = _pair()
        pair = cls(pair.hl_model, pair.ll_model, pair.corr, training_args={"batch_size": 64, "lr": 1e-3,
                                                                           "lr_scheduler": None})
        pair.loss_fn = lambda out, y: torch.nn.functional.cross_entropy(
            (out[:, -1] if out.dim() == 3 else out).float(),
            (y[:, -1] if y.dim() == 2 else y) if not y.dtype.is_floating_point else y.argmax(-1)[:, -1] if y.dim() == 3 else y.argmax(-1))
        tr, te = train_test_split(ds, 0.25, 42)
        pair.train(IITDataset(tr, tr, seed=0, device="cpu"), IITDataset(te, te, seed=0, device="cpu"), epochs=1)
        assert pair.train_metrics.metrics[0].get_value() > 0


def test_ioi_pair_trains_and_checkpoints(tmp_path):
    from iit_amd.data.iit_dataset import IITDataset, train_test_split
    pair, ds = _pair()
    tr, te = train_test_split(ds, 0.25, 42)
    pair.train(IITDataset(tr, tr, seed=0, device="cpu"), IITDataset(te, te, seed=0, device="cpu"), epochs=2)
    names = [m.get_name() for m in pair.test_metrics.metrics]
    assert names == ["val/iit_loss", "val/IIA", "val/accuracy", "val/per_token_accuracy"]
    assert pair.test_metrics.metrics[3].get_value().shape == (16,)


def test_oracle_train_step_under_detect_anomaly():
    """the fp32 oracle's full Strict-IIT step (5 forwards, 3 backwards incl. in-place splices, the
    fused-optimizer fallback) runs clean under ``torch.autograd.detect_anomaly`` (NaN / in-place-modification checks
    on every backward node)."""
    import torch

    from iit_amd.data.iit_dataset import IITDataset
    from iit_amd.model_pairs import IOI_ModelPair
    from iit_amd.models.config import gpt2_config_dict
    from iit_amd.models.transformer import HookedTransformer
    from iit_amd.tasks.ioi import make_ioi_corr, make_ioi_dataset_and_hl
    cfg = gpt2_config_dict()
    cfg.update(n_layers=6, d_model=32, n_heads=4, d_head=8, d_mlp=64, device="cpu")
    torch.manual_seed(0)
    ll = HookedTransformer(cfg)
    ds, hl = make_ioi_dataset_and_hl(128, ll, device="cpu")
    train = IITDataset(ds, ds, seed=0, device="cpu")
    pair = IOI_ModelPair(hl, ll, make_ioi_corr(6), training_args={"batch_size": 32, "lr": 1e-3, "lr_scheduler": None,
                                                                   "fused_optimizer": True})
    opt = pair.make_optimizer(1e-3)
    base, abl = next(iter(train.make_loader(32, 0)))
    with torch.autograd.detect_anomaly():
        for _ in range(2):
            out = pair.run_train_step(base, abl, pair.loss_fn, opt)
    assert all(torch.isfinite(torch.as_tensor(v)).all() for v in out.values())
