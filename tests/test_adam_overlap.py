"""Overlapped optimizer update (iit_amd/ops/optim.py FusedAdam.enable_overlap / wait_stage).

A phase that another phase of the same train step follows launches only its clip-norm stage; its Adam runs as one
chunk per model stage on a side stream under the next phase's forward, each stage waiting for its own chunk.  CPU:
the model's stage gates and the arena ranges the chunks split at.  GPU: training with the overlapped update
reproduces the serial one, eager and graph-captured.
"""
import os

import pytest
import torch

from iit_amd.engine.flat import FlatParams
from iit_amd.models.transformer import HookedTransformer
from iit_amd.ops.optim import FusedAdam


def tiny(**kw):
    cfg = dict(n_layers=3, n_heads=3, d_model=12, d_head=4, d_mlp=24, n_ctx=16, act_fn="gelu_new", d_vocab=29,
               device="cpu", normalization_type="LN")
    cfg.update(kw)
    torch.manual_seed(0)
    return HookedTransformer(cfg)


@pytest.mark.parametrize("norm", ["LN", "LNPre"])
def test_stages_cover_the_arena_in_forward_order(norm):
    m = tiny(normalization_type=norm)
    flat = FlatParams(m)
    stages = m.param_stages()
    assert len(stages) == len(m.blocks) + 2
    assert sorted(id(p) for ps in stages for p in ps) == sorted(id(p) for p in m.parameters())
    hi = 0
    for ps in stages:
        lo = min(flat.offset_of(p) for p in ps)
        assert lo >= hi  # the chunk of a stage never holds a later stage's weights
        hi = max(flat.offset_of(p) + p.numel() for p in ps)


def test_forward_gates_each_stage_in_order():
    m = tiny()
    calls = []
    m.__dict__["_param_gate"] = calls.append
    m(torch.randint(0, 29, (2, 5)))
    assert calls == list(range(len(m.blocks) + 2))


def test_chunk_bounds_split_the_span_table(monkeypatch):
    m = tiny(d_model=64, d_head=16, n_heads=4, d_mlp=256, d_vocab=301)
    flat = FlatParams(m)
    opt = FusedAdam(flat, use_hip=False)
    opt._hip = object()  # (the bounds only; no launch on CPU)
    monkeypatch.setattr(torch.cuda, "Stream", lambda device=None: None)
    monkeypatch.setenv("IIT_ADAM_OVERLAP", "1")
    assert opt.enable_overlap(m.param_stages())
    flat.span_table(24, max_len4=16)
    idx = [0] + [flat.span_index(b) for b in opt._bounds[:-1]]
    assert idx == sorted(idx) and idx[-1] <= len(flat._span_starts)
    starts = flat._span_starts
    for k, b in enumerate(opt._bounds[:-1]):  # every span of chunk k starts below stage k's end
        assert all(s < b for s in starts[:idx[k + 1]]) and all(s >= b for s in starts[idx[k + 1]:])


def test_capture_guard_restores_a_pending_update():
    """a capture that launched the pending update and then failed must hand the record back, so the
    eager fallback still applies the previous phase's Adam (its norm stage already bumped the step)."""
    m = tiny()
    opt = FusedAdam(FlatParams(m), use_hip=False)
    rec = {"chunks": [(0, 1)]}
    opt._pending, opt._inflight = rec, None
    restore = opt.capture_guard()
    opt._pending, opt._inflight = None, ["event recorded inside the aborted capture"]  # the gate launched it
    restore()
    assert opt._pending is rec and opt._inflight is None


def test_overlap_disabled_by_env(monkeypatch):
    m = tiny()
    opt = FusedAdam(FlatParams(m), use_hip=False)
    opt._hip = object()
    monkeypatch.setenv("IIT_ADAM_OVERLAP", "0")
    assert not opt.enable_overlap(m.param_stages())


def _train(mode, overlap, monkeypatch, n_batches=8):
    # overlap: False, True (chunks inside the captured graphs) or "split" (per-stage graphs, chunks launched eagerly)
    monkeypatch.setenv("IIT_ADAM_OVERLAP", "2" if overlap == "split" else ("1" if overlap else "0"))
    from iit_amd.data.iit_dataset import IITDataset
    from iit_amd.engine.graphs import GraphedTrainStep
    from iit_amd.model_pairs import IOI_ModelPair
    from iit_amd.models.config import gpt2_config_dict
    from iit_amd.tasks.ioi import ioi_cfg, make_ioi_corr, make_ioi_dataset_and_hl
    import contextlib
    cfg = gpt2_config_dict()
    cfg.update(ioi_cfg)
    cfg.update(device="cuda", dtype=torch.bfloat16)
    torch.manual_seed(0)
    ll = HookedTransformer(cfg)
    ds, hl = make_ioi_dataset_and_hl(512, ll, device="cuda")
    train = IITDataset(ds, ds, seed=0, device="cuda")
    pair = IOI_ModelPair(hl, ll, make_ioi_corr(6), training_args={"batch_size": 64, "lr": 1e-3, "strict_weight": 0.4,
                                                                   "lr_scheduler": None})
    opt = pair.make_optimizer(1e-3)
    assert (opt._bounds is not None) == bool(overlap)
    torch.manual_seed(1)
    batches = [b for _, b in zip(range(n_batches), train.make_loader(64, 0))]
    step, ctx, g = pair.run_train_step, contextlib.nullcontext(), None
    if mode == "graphs":
        g = step = GraphedTrainStep(pair, opt, pair.loss_fn)
        ctx = g.stream_context()
    losses = []
    with ctx:
        for base, abl in batches * 2:
            out = step(base, abl, pair.loss_fn, opt)
            assert opt._pending is None and opt._inflight is None  # every step ends with its updates applied
            losses.append(torch.stack([out[k] for k in sorted(out)]))
    torch.cuda.synchronize()
    if g is not None:
        assert g.captures > 0 and g.replays > 0 and not g.failed, g.failed
    return torch.stack(losses).cpu(), opt.flat.data.clone(), int(opt._step_dev.item())


@pytest.mark.gpu
@pytest.mark.skipif(os.environ.get("IIT_TEST_ADAM_OVERLAP") != "1",
                    reason="opt-in path (IIT_ADAM_OVERLAP=1) not yet run on hardware: set IIT_TEST_ADAM_OVERLAP=1")
@pytest.mark.parametrize("mode,overlap", [("eager", True), ("graphs", True), ("graphs", "split")])
def test_overlapped_update_matches_serial(mode, overlap, monkeypatch):
    ls, ps, ss = _train(mode, False, monkeypatch)
    lo, po, so = _train(mode, overlap, monkeypatch)
    assert ss == so == 3 * 16  # three optimizer phases per step, every one counted once
    # same kernels, same order of every update: only fp32-atomic accumulation noise separates two runs
    # (tests/test_graphs.py); compare the early steps tightly and the weights loosely
    assert torch.allclose(ls[:12], lo[:12], rtol=2e-3, atol=2e-3), (ls[:12] - lo[:12]).abs().max()
    assert torch.isfinite(po).all() and (po - ps).abs().max() < 5e-2
