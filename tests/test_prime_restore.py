"""Graph priming before epoch 0 must not change the training run: the state snapshot of
:class:`iit_amd.engine.graphs._TrainState` puts weights, optimizer state and RNGs back exactly, in place."""
import numpy as np
import pytest
import torch

from iit_amd.data.iit_dataset import IITDataset
from iit_amd.engine.graphs import _TrainState
from iit_amd.tasks.ioi import make_ioi_corr, make_ioi_dataset_and_hl


def _pair(fused):
    from iit_amd.model_pairs import IOI_ModelPair
    from iit_amd.models.config import gpt2_config_dict
    from iit_amd.models.transformer import HookedTransformer
    cfg = gpt2_config_dict()
    cfg.update(n_layers=2, d_model=32, n_heads=4, d_head=8, d_mlp=64, device="cpu")
    torch.manual_seed(0)
    ll = HookedTransformer(cfg)
    ds, hl = make_ioi_dataset_and_hl(128, ll, device="cpu")
    pair = IOI_ModelPair(hl, ll, make_ioi_corr(2), training_args={"batch_size": 32, "lr": 1e-3, "lr_scheduler": None,
                                                                  "fused_optimizer": fused})
    return pair, IITDataset(ds, ds, seed=0, device="cpu")


@pytest.mark.parametrize("fused", [True, False])
def test_train_state_snapshot_restores_in_place(fused):
    pair, train = _pair(fused)
    opt = pair.make_optimizer(1e-3)
    batches = list(train.make_loader(32, 0))
    pair.run_train_step(*batches[0], pair.loss_fn, opt)  # optimizer state exists before the snapshot
    live = [p.data for p in pair.ll_model.parameters()]
    before = [t.clone() for t in live]
    snap = _TrainState(pair, opt)
    rng = pair.rng.bit_generator.state
    torch_rng = torch.get_rng_state()
    for b in batches[1:3]:  # "priming" steps
        pair.run_train_step(*b, pair.loss_fn, opt)
    torch.rand(3)
    assert any(not torch.equal(a, b) for a, b in zip(live, before))
    snap.restore()
    pair.rng.bit_generator.state = rng  # (prime() restores the node-sampling generator itself)
    assert all(torch.equal(a, b) for a, b in zip(live, before))  # same tensors, old values
    assert torch.equal(torch.get_rng_state(), torch_rng)
    # the continued run equals a run that never primed
    ref_pair, _ = _pair(fused)
    ref_opt = ref_pair.make_optimizer(1e-3)
    ref_pair.run_train_step(*batches[0], ref_pair.loss_fn, ref_opt)
    ref_pair.rng.bit_generator.state = rng
    out = pair.run_train_step(*batches[3], pair.loss_fn, opt)
    ref = ref_pair.run_train_step(*batches[3], ref_pair.loss_fn, ref_opt)
    for k in ref:
        assert np.isclose(float(out[k]), float(ref[k]), rtol=1e-6, atol=1e-7), k
    for a, b in zip(pair.ll_model.parameters(), ref_pair.ll_model.parameters()):
        assert torch.allclose(a, b, atol=1e-7, rtol=1e-6)


def test_train_state_restores_batchnorm_buffers():
    """the PVR ResNet LL is graphed and primed; the priming steps run in training mode and move every
    BatchNorm's running statistics and ``num_batches_tracked``.  The snapshot covers module buffers, so the
    restore puts them back exactly (eval metrics of a primed run equal an unprimed one's)."""
    from iit_amd.model_pairs import IITBehaviorModelPair
    from iit_amd.tasks.task_loader import get_alignment, get_dataset
    torch.manual_seed(0)
    tr, te = get_dataset("mnist_pvr", {"train_size": 32, "test_size": 16, "device": "cpu"})
    ll, hl, corr = get_alignment("mnist_pvr", {"input_shape": te.base_data.get_input_shape(), "device": "cpu"})
    pair = IITBehaviorModelPair(ll_model=ll, hl_model=hl, corr=corr,
                                training_args={"lr": 1e-3, "batch_size": 16, "early_stop": False,
                                               "lr_scheduler": None})
    opt = pair.make_optimizer(1e-3)
    module = pair._ll_module()
    bufs = [b for b in module.buffers()]
    assert any(b.dtype == torch.long for b in bufs)  # num_batches_tracked
    before = [b.clone() for b in bufs]
    snap = _TrainState(pair, opt)
    module.train()
    for b in list(tr.make_loader(16, 0))[:2]:
        pair.run_train_step(*b, pair.loss_fn, opt)
    assert any(not torch.equal(a, b) for a, b in zip(bufs, before))
    snap.restore()
    assert all(torch.equal(a, b) for a, b in zip(module.buffers(), before))


def test_graph_key_includes_module_mode():
    """a phase graph captured in eval mode must not be replayed in training mode -- the graph key carries
    the LL module's mode (and the optimizer's row-restriction version)."""
    from iit_amd.engine.graphs import GraphedTrainStep
    pair, _ = _pair(True)
    opt = pair.make_optimizer(1e-3)
    step = GraphedTrainStep(pair, opt, pair.loss_fn, enabled=False)
    step._sig = ("sig",)
    pair.ll_model.train()
    k_train = step._graph_key("iit", opt)
    pair.ll_model.eval()
    k_eval = step._graph_key("iit", opt)
    assert k_train != k_eval
    pair.ll_model.train()
    assert step._graph_key("iit", opt) == k_train
