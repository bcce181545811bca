"""The 1 -> N measurement path of ``bench.py`` (VERDICT r5 missing #4 / next #1), rehearsed on CPU with gloo.

* ``python bench.py --gpus 2`` with no launcher starts the two ranks itself and reports ``n_gpus: 2`` / ``dp2``;
* a launcher world that differs from ``--gpus`` exits non-zero instead of reporting another ``n_gpus``;
* ``--global-batch`` holds the job's batch (strong scaling);
* GEMM decisions agree across ranks after ``gemm_dispatch.sync_decisions`` even when the ranks timed different
  winners;
* ZeRO-1 deferred gathers are never consumed by a gate under stream capture.
"""
import json
import os
import socket
import subprocess
import sys

import pytest
import torch
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _bench_env(**extra):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(IIT_BENCH_TINY="1", OMP_NUM_THREADS="2", **extra)
    return env


def _json_line(stdout: str) -> dict:
    lines = [l for l in stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, stdout
    return json.loads(lines[0])


def test_bench_gpus2_self_launches(tmp_path):
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "1"]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=_bench_env(), cwd=str(tmp_path))
    assert out.returncode == 0, out.stderr[-3000:]
    rec = _json_line(out.stdout)
    assert rec["n_gpus"] == 2 and rec["config"]["parallelism"] == "dp2" and rec["scaling"] == "weak"
    assert rec["config"]["global_batch"] == 2 * 16  # tiny config: 16 pairs per rank
    assert "without a launcher" in out.stderr


def test_bench_strong_scaling_global_batch(tmp_path):
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "1",
           "--global-batch", "16"]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=_bench_env(), cwd=str(tmp_path))
    assert out.returncode == 0, out.stderr[-3000:]
    rec = _json_line(out.stdout)
    assert rec["n_gpus"] == 2 and rec["scaling"] == "strong" and rec["config"]["global_batch"] == 16


def test_bench_world_mismatch_fails(tmp_path):
    # a launcher environment of one rank while --gpus 2 is asked: exit 3, no JSON line
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1", "--warmup", "0"]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=_bench_env(WORLD_SIZE="1"),
                         cwd=str(tmp_path))
    assert out.returncode == 3, (out.returncode, out.stderr[-2000:])
    assert not [l for l in out.stdout.splitlines() if l.startswith("{")]
    # and under a real launcher with 2 ranks while --gpus 4 is asked
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", str(_free_port()), os.path.join(ROOT, "bench.py"), "--gpus", "4",
           "--steps", "1", "--warmup", "0"]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=_bench_env(), cwd=str(tmp_path))
    assert out.returncode != 0
    assert not [l for l in out.stdout.splitlines() if l.startswith("{")]


def _decision_worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    from iit_amd.ops import gemm_dispatch as gd
    from iit_amd.parallel import dist as pdist
    pdist.init_distributed("gloo")
    # perturbed timings: each rank "measured" a different winner for the shared keys, and one key only it met
    shared = [(4096, 768, 768, 0, 0, True, False, False), (768, 3072, 4096, 3, 2, False, True, False)]
    for i, k in enumerate(shared):
        times = {"hip": 10.0 + rank - i, "glds128": 10.5 - rank + i, "blas": 11.0}
        gd.DECISIONS[k] = (min(times, key=times.get), times)
    gd.DECISIONS[(rank + 1, 64, 64, 0, 0, False, False, False)] = (f"only{rank}", {f"only{rank}": 1.0})
    gd.DUAL_DECISIONS[("dual", 1, 2, 3, 0, False, 4, 5, 6, 2, True, False)] = (f"dual128.128r{2 ** rank}", {})
    gd.RAGGED[(1, 2, 3, 0, 0, False, False, False)] = (rank == 0, 1.0, [0.4, 0.5])
    before = {repr(k): v[0] for k, v in gd.DECISIONS.items()}
    changed = gd.sync_decisions()
    after = {"gemm": {repr(k): v[0] for k, v in gd.DECISIONS.items()},
             "dual": {repr(k): v[0] for k, v in gd.DUAL_DECISIONS.items()},
             "ragged": {repr(k): v[0] for k, v in gd.RAGGED.items()}}
    with open(os.path.join(out_dir, f"dec{rank}.json"), "w") as f:
        json.dump({"before": before, "after": after, "changed": changed}, f)
    pdist.destroy()


def test_gemm_decisions_rank_consistent(tmp_path):
    mp.spawn(_decision_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    r = [json.load(open(tmp_path / f"dec{i}.json")) for i in range(2)]
    assert r[0]["before"] != r[1]["before"]  # the ranks disagreed before the exchange
    assert r[0]["after"] == r[1]["after"]    # identical tables after it
    for k, v in r[0]["before"].items():      # rank 0's choices are the job's
        assert r[1]["after"]["gemm"][k] == v
    assert r[0]["changed"] == 1              # rank 0 only adopted the key rank 1 alone measured
    assert "only1" in r[0]["after"]["gemm"].values() and "only0" in r[1]["after"]["gemm"].values()
    assert list(r[1]["after"]["dual"].values()) == ["dual128.128r1"]
    assert list(r[1]["after"]["ragged"].values()) == [True]


def test_gemm_freeze_refuses_untabled_problem(monkeypatch):
    from iit_amd.ops import gemm_dispatch as gd
    monkeypatch.setattr(gd, "_FREEZE", True)
    with pytest.raises(RuntimeError, match="IIT_GEMM_FREEZE"):
        gd._frozen_miss((1, 2, 3))
    monkeypatch.setattr(gd, "_FREEZE", False)
    gd._frozen_miss((1, 2, 3))


class _Work:
    def __init__(self, fail=False):
        self.waits, self.fail = 0, fail

    def wait(self):
        self.waits += 1
        if self.fail:
            raise RuntimeError("collective failed")


def _bare_zero(nb=2):
    """A ShardedFusedAdam's gather bookkeeping without a process group (the methods under test only read these)."""
    from iit_amd.parallel.zero import ShardedFusedAdam, ShardPlan

    class _Flat:
        data = torch.zeros(256)
        shadow = None

    z = ShardedFusedAdam.__new__(ShardedFusedAdam)
    z.flat = _Flat()
    z.plan = ShardPlan([(0, 128), (128, 256)][:nb], 1, 0)
    z._pending = {}
    z._gather_bufs = {}
    z._hip = None
    return z


def test_zero_gate_is_a_noop_under_capture(monkeypatch):
    z = _bare_zero()
    w0, w1 = _Work(), _Work()
    z._pending = {0: (w0, False), 1: (w1, False)}
    monkeypatch.setattr(torch.cuda, "is_available", lambda: True)
    monkeypatch.setattr(torch.cuda, "is_current_stream_capturing", lambda: True)
    z._finish(0)
    z.wait_gathers()
    assert set(z._pending) == {0, 1} and w0.waits == w1.waits == 0  # nothing recorded-but-not-run, nothing dropped
    monkeypatch.setattr(torch.cuda, "is_current_stream_capturing", lambda: False)
    z.wait_gathers()
    assert not z._pending and w0.waits == w1.waits == 1


def test_zero_failed_wait_keeps_bucket_pending():
    z = _bare_zero(1)
    bad = _Work(fail=True)
    z._pending = {0: (bad, False)}
    with pytest.raises(RuntimeError):
        z._finish(0)
    assert 0 in z._pending  # a retry / join still sees it (never a silently stale mirror)
