"""Tracing ranges, step timing and the race-debug switch (iit_amd/utils/tracing.py)."""
import os
import subprocess
import sys

import pytest
import torch

from iit_amd.data.iit_dataset import IITDataset, train_test_split
from iit_amd.tasks.ioi import make_ioi_corr, make_ioi_dataset_and_hl
from iit_amd.utils import tracing

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _pair():
    from iit_amd.model_pairs import IOI_ModelPair
    from iit_amd.models.config import gpt2_config_dict
    from iit_amd.models.transformer import HookedTransformer
    cfg = gpt2_config_dict()
    cfg.update(n_layers=2, d_model=16, n_heads=2, d_head=8, d_mlp=32, device="cpu")
    torch.manual_seed(0)
    ll = HookedTransformer(cfg)
    ds, hl = make_ioi_dataset_and_hl(96, ll, device="cpu")
    pair = IOI_ModelPair(hl, ll, make_ioi_corr(2), training_args={"batch_size": 16, "lr": 1e-3, "lr_scheduler": None,
                                                                   "early_stop": False, "strict_weight": 0.4})
    tr, te = train_test_split(ds, 0.25, 42)
    return pair, IITDataset(tr, tr, seed=0, device="cpu"), IITDataset(te, te, seed=0, device="cpu")


def test_phase_ranges_recorded_when_profiling(capsys):
    pair, tr, te = _pair()
    tracing.set_profiling(True)
    try:
        with torch.profiler.profile(activities=[torch.profiler.ProfilerActivity.CPU]) as prof:
            pair.train(tr, te, epochs=1)
    finally:
        tracing.set_profiling(False)
    names = {e.name for e in prof.events()}
    for want in ("train_step", "hl_source_cache", "ll_source_cache", "hl_intervened_fwd", "ll_spliced_fwd",
                 "backward", "clip_adam", "eval_epoch"):
        assert want in names, (want, sorted(n for n in names if not n.startswith("aten::"))[:40])
    assert "[perf] epoch 0:" in capsys.readouterr().out


def test_throughput_per_epoch_without_profiling():
    pair, tr, te = _pair()
    assert not tracing.PROFILE
    pair.train(tr, te, epochs=1)
    tp = pair.throughput
    n_batches = -(-len(tr) // 16)
    assert tp["steps"] == n_batches - 1  # the first (warm-up) step is left out
    assert tp["ms_per_step"] > 0 and tp["pairs_per_s"] > 0


def test_step_timer_math():
    t = tracing.StepTimer(world_size=4)
    t.cuda = False
    t._marks = [(0.0, 1.0, 8), (1.0, 1.5, 8), (1.5, 2.0, 4)]
    s = t.summary(skip_first=1)
    assert s["steps"] == 2 and abs(s["ms_per_step"] - 500.0) < 1e-9
    assert abs(s["pairs_per_s"] - (8 + 4) * 4 / 1.0) < 1e-9  # whole-job pairs over the timed steps
    assert t.summary() is None  # marks are consumed


def test_range_is_noop_when_off():
    assert not tracing.PROFILE
    assert tracing.trace_range("x") is tracing.trace_range("y")  # the shared null context: no allocation
    tracing.sync_point()  # no device: nothing to drain


def test_debug_sync_mode_serialises_hip_launches():
    env = {k: v for k, v in os.environ.items() if k not in ("HIP_LAUNCH_BLOCKING", "AMD_SERIALIZE_KERNEL")}
    env["IIT_DEBUG_SYNC"] = "1"
    code = ("import os, iit_amd.utils.tracing as t; "
            "print(os.environ['HIP_LAUNCH_BLOCKING'], os.environ['AMD_SERIALIZE_KERNEL'], t.DEBUG_SYNC)")
    out = subprocess.run([sys.executable, "-c", code], cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-2000:]
    assert out.stdout.split() == ["1", "3", "True"]


@pytest.mark.gpu
def test_debug_sync_and_ranges_keep_graph_capture_working():
    """Race-debug drains and roctx ranges around graph-captured phases: captures still succeed (no device sync
    inside a capture) and the ranges reach roctx without error."""
    from iit_amd.engine.graphs import GraphedTrainStep
    from iit_amd.model_pairs import IOI_ModelPair
    from iit_amd.models.config import gpt2_config_dict
    from iit_amd.models.transformer import HookedTransformer
    from iit_amd.ops import hip_kernels
    hip_kernels.lib()
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    cfg = gpt2_config_dict()
    cfg.update(n_layers=2, d_model=128, n_heads=4, d_head=32, d_mlp=512, device="cuda:0", dtype=torch.bfloat16)
    ll = HookedTransformer(cfg)
    ll.set_op_backend("hip")
    ds, hl = make_ioi_dataset_and_hl(256, ll, device=dev)
    train = IITDataset(ds, ds, seed=0, device=dev)
    pair = IOI_ModelPair(hl, ll, make_ioi_corr(2), training_args={"batch_size": 64, "lr": 1e-3, "lr_scheduler": None})
    opt = pair.make_optimizer(1e-3)
    runner = GraphedTrainStep(pair, opt, pair.loss_fn)
    tracing.set_profiling(True)
    tracing.set_debug_sync(True)
    try:
        for i, (base, abl) in enumerate(train.make_loader(64, 0)):
            out = runner(base, abl, pair.loss_fn, opt)
        torch.cuda.synchronize()
    finally:
        tracing.set_profiling(False)
        tracing.set_debug_sync(False)
    assert runner.captures > 0 and not runner.failed, runner.failed
    assert all(torch.isfinite(torch.as_tensor(v)).all() for v in out.values())
