"""T3: data parallelism without a cluster -- gloo, world_size 2, on CPU.

* DP(2) x (B/2) == 1 x B: same losses and the same weights after several Strict-IIT
  steps (3 optimizer steps each, global-norm clip after the bucketed all-reduce);
* every rank samples the same HL / strict node sequence (identically seeded RNG);
* epoch metrics are averaged across ranks;
* ``bench.py`` runs under ``torch.distributed.run`` with the driver's flags.
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


def _make(global_batch: int):
    from iit_amd.data.iit_dataset import IITDataset
    from iit_amd.model_pairs import IOI_ModelPair
    from iit_amd.models.config import gpt2_config_dict
    from iit_amd.models.transformer import HookedTransformer
    from iit_amd.tasks.ioi import make_ioi_corr, make_ioi_dataset_and_hl
    cfg = gpt2_config_dict()
    cfg.update(n_layers=2, d_model=16, n_heads=2, d_head=8, d_mlp=32, device="cpu")
    torch.manual_seed(0)
    ll = HookedTransformer(cfg)
    ds, hl = make_ioi_dataset_and_hl(256, ll, device="cpu")
    train = IITDataset(ds, ds, seed=0, device="cpu")
    pair = IOI_ModelPair(hl, ll, make_ioi_corr(2), training_args={
        "batch_size": global_batch, "lr": 1e-3, "lr_scheduler": None, "strict_weight": 0.4, "bucket_mb": 0.05})
    return pair, train


def _train(pair, train, per_rank_batch, steps=4):
    opt = pair.make_optimizer(1e-3)
    torch.manual_seed(5)
    loader = train.make_loader(per_rank_batch, 0)
    losses, nodes = [], []
    orig = pair.sample_hl_name
    pair.sample_hl_name = lambda: (lambda n: (nodes.append(n.name), n)[1])(orig())
    for i, (base, abl) in enumerate(loader):
        if i >= steps:
            break
        out = pair.run_train_step(base, abl, pair.loss_fn, opt)
        losses.append([float(out[k]) for k in sorted(out)])
    return losses, nodes


def _worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    from iit_amd.parallel import dist as pdist
    pdist.init_distributed("gloo")
    torch.set_num_threads(2)
    pair, train = _make(64)
    pdist.broadcast_module(pair.ll_model)
    losses, nodes = _train(pair, train, per_rank_batch=32)
    # metric all-reduce: each rank contributes its own value; the result is the mean
    from iit_amd.core.metric import MetricStore, MetricStoreCollection, MetricType
    mc = MetricStoreCollection([MetricStore("val/IIA", MetricType.ACCURACY)])
    mc.update({"val/IIA": float(rank)})
    pair._reduce_metrics(mc)
    torch.save({"losses": losses, "nodes": nodes, "metric": mc.metrics[0].get_value(),
                "params": {n: p.detach().clone() for n, p in pair.ll_model.named_parameters()}},
               os.path.join(out_dir, f"rank{rank}.pt"))
    pdist.destroy()


def test_dp2_equals_single_process(tmp_path):
    pair, train = _make(64)
    ref_losses, ref_nodes = _train(pair, train, per_rank_batch=64)
    ref_params = {n: p.detach().clone() for n, p in pair.ll_model.named_parameters()}
    mp.spawn(_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    r = [torch.load(tmp_path / f"rank{i}.pt", weights_only=True) for i in range(2)]
    assert r[0]["nodes"] == r[1]["nodes"] == ref_nodes
    for i in range(2):
        for n, p in ref_params.items():
            assert torch.allclose(r[i]["params"][n], p, atol=2e-5, rtol=1e-4), (i, n)
    # per-rank losses are shard means; their average is the global-batch loss
    avg = torch.tensor(r[0]["losses"]) / 2 + torch.tensor(r[1]["losses"]) / 2
    assert torch.allclose(avg, torch.tensor(ref_losses), atol=1e-4)
    assert r[0]["metric"] == pytest.approx(50.0) and r[1]["metric"] == pytest.approx(50.0)  # mean of 0, 100 (x100)


def test_bench_under_torchrun_gloo(tmp_path):
    """The driver's multi-GPU launch line, rehearsed on CPU with 2 gloo ranks and a tiny config."""
    env = dict(os.environ, IIT_BENCH_TINY="1", OMP_NUM_THREADS="2")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", str(_free_port()), os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps",
           "2", "--warmup", "1"]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=env, cwd=str(tmp_path))
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2 and rec["steps"] == 2 and rec["config"]["parallelism"] == "dp2"
    assert rec["value"] > 0 and rec["scaling"] == "weak"


def _worker_subset(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    from iit_amd.parallel import dist as pdist
    pdist.init_distributed("gloo")
    torch.set_num_threads(2)
    pair, train = _make(64)
    pdist.broadcast_module(pair.ll_model)
    opt = pair.make_optimizer(1e-3)
    pair.restrict_embedding_reduce(train)
    assert pair._reducer._subsets, "embedding row subset not installed"
    torch.manual_seed(5)
    for i, (base, abl) in enumerate(train.make_loader(32, 0)):
        if i >= 3:
            break
        pair.run_train_step(base, abl, pair.loss_fn, opt)
    torch.save({n: p.detach().clone() for n, p in pair.ll_model.named_parameters()},
               os.path.join(out_dir, f"subset{rank}.pt"))
    pdist.destroy()


def test_dp2_embedding_row_subset_reduce_is_exact(tmp_path):
    pair, train = _make(64)
    _train(pair, train, per_rank_batch=64, steps=3)
    ref = {n: p.detach().clone() for n, p in pair.ll_model.named_parameters()}
    mp.spawn(_worker_subset, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    for i in range(2):
        got = torch.load(tmp_path / f"subset{i}.pt", weights_only=True)
        for n, p in ref.items():
            assert torch.allclose(got[n], p, atol=2e-5, rtol=1e-4), (i, n)


def _worker_staged(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    from iit_amd.engine.graphs import GraphedTrainStep
    from iit_amd.parallel import dist as pdist
    pdist.init_distributed("gloo")
    torch.set_num_threads(2)
    pair, train = _make(64)
    pdist.broadcast_module(pair.ll_model)
    opt = pair.make_optimizer(1e-3)
    pair.restrict_sparse_rows(train)
    # the graph runner's DP schedule, kept eager (no GPU): staged backward + per-stage range all-reduce
    step = GraphedTrainStep(pair, opt, pair.loss_fn, warmup=10 ** 9, enabled=True)
    assert step.split and step.staged is not None and step.staged.cuts == [1]
    rng = step.staged.ranges()
    assert rng[0][1] == pair._reducer.flat.numel and rng[-1][0] == 0
    assert all(a[0] == b[1] for a, b in zip(rng, rng[1:]))  # contiguous, top to bottom
    edges = {e for b in pair._reducer.buckets for e in b}
    assert all(s in edges and e in edges for s, e in rng)
    torch.manual_seed(5)
    for i, (base, abl) in enumerate(train.make_loader(32, 0)):
        if i >= 3:
            break
        step(base, abl)
    assert not getattr(pair.ll_model, "_cut_log", [])
    torch.save({n: p.detach().clone() for n, p in pair.ll_model.named_parameters()},
               os.path.join(out_dir, f"staged{rank}.pt"))
    pdist.destroy()


def test_dp2_staged_backward_range_reduce_equals_single_process(tmp_path):
    pair, train = _make(64)
    _train(pair, train, per_rank_batch=64, steps=3)
    ref = {n: p.detach().clone() for n, p in pair.ll_model.named_parameters()}
    mp.spawn(_worker_staged, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    for i in range(2):
        got = torch.load(tmp_path / f"staged{i}.pt", weights_only=True)
        for n, p in ref.items():
            assert torch.allclose(got[n], p, atol=2e-5, rtol=1e-4), (i, n)


def test_grad_cut_backward_is_exact():
    """Cutting the residual stream and resuming the backward per stage gives plain autograd's gradients."""
    from iit_amd.engine.staged import StagedBackward
    from iit_amd.models.config import gpt2_config_dict
    from iit_amd.models.transformer import HookedTransformer
    cfg = gpt2_config_dict()
    cfg.update(n_layers=4, d_model=16, n_heads=2, d_head=8, d_mlp=32, d_vocab=50, n_ctx=16, device="cpu")
    torch.manual_seed(0)
    m = HookedTransformer(cfg)
    tok = torch.randint(0, 50, (3, 7))
    m(tok).pow(2).mean().backward()
    ref = {n: p.grad.clone() for n, p in m.named_parameters()}
    m.zero_grad()
    st = StagedBackward(m, 4)
    assert st.cuts == [1, 2, 3] and st.flat is None
    st.arm()
    loss = m(tok).pow(2).mean()
    st.disarm()
    loss.backward()
    assert m.blocks[0].attn.W_Q.grad is None or not m.blocks[0].attn.W_Q.grad.any()
    for k in st.stages():
        st.run_stage(k)
    st.release()
    for n, p in m.named_parameters():
        assert torch.allclose(p.grad, ref[n], atol=1e-6, rtol=1e-5), n


def test_rehearsal_device_mapping(monkeypatch):
    """IIT_REHEARSE_ONE_GPU maps every rank to cuda:0 (the one-GPU multi-rank rehearsal); otherwise LOCAL_RANK."""
    from iit_amd.parallel import dist as pdist
    monkeypatch.setenv("LOCAL_RANK", "3")
    monkeypatch.delenv("IIT_REHEARSE_ONE_GPU", raising=False)
    assert pdist.local_device_index() == 3
    monkeypatch.setenv("IIT_REHEARSE_ONE_GPU", "1")
    assert pdist.local_device_index() == 0


def _worker_bf16_wire(rank, world, port, out_dir):
    os.environ["IIT_DP_GRAD_DTYPE"] = "bf16"
    _worker(rank, world, port, out_dir)


def test_dp2_bf16_wire_gradients(tmp_path):
    """IIT_DP_GRAD_DTYPE=bf16: gradients travel as bf16 -- the ranks stay bit-identical to each other and close
    to the single-process (fp32) run."""
    pair, train = _make(64)
    ref_losses, _ = _train(pair, train, per_rank_batch=64)
    ref_params = {n: p.detach().clone() for n, p in pair.ll_model.named_parameters()}
    mp.spawn(_worker_bf16_wire, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    r = [torch.load(tmp_path / f"rank{i}.pt", weights_only=True) for i in range(2)]
    for n, p in ref_params.items():
        assert torch.equal(r[0]["params"][n], r[1]["params"][n]), n
        if n.endswith("b_K"):  # exactly-zero gradient in exact arithmetic: Adam turns rounding noise into +-lr steps
            continue
        err = float((r[0]["params"][n] - p).norm() / (p.norm() + 1e-12))
        assert err < 5e-2, (n, err)
    avg = torch.tensor(r[0]["losses"]) / 2 + torch.tensor(r[1]["losses"]) / 2
    assert torch.allclose(avg, torch.tensor(ref_losses), atol=2e-2, rtol=2e-2)


def _train_single_loss(pair, train, per_rank_batch, steps=3):
    pair.training_args["use_single_loss"] = True
    return _train(pair, train, per_rank_batch, steps=steps)


def _worker_single_loss(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    from iit_amd.parallel import dist as pdist
    pdist.init_distributed("gloo")
    torch.set_num_threads(2)
    pair, train = _make(64)
    pdist.broadcast_module(pair.ll_model)
    losses, nodes = _train_single_loss(pair, train, per_rank_batch=32)
    assert pair._reducer.overlap and not pair._reducer.deferred
    torch.save({"losses": losses, "nodes": nodes,
                "params": {n: p.detach().clone() for n, p in pair.ll_model.named_parameters()}},
               os.path.join(out_dir, f"single{rank}.pt"))
    pdist.destroy()


def test_dp2_single_loss_equals_single_process(tmp_path):
    """use_single_loss: one backward through the IIT, strict and behaviour forwards writes every weight gradient
    three times; the overlapped reducer must reduce only the final sums (launching a bucket at the first
    report raced the later accumulations and left the ranks with different weights)."""
    pair, train = _make(64)
    ref_losses, ref_nodes = _train_single_loss(pair, train, per_rank_batch=64)
    ref_params = {n: p.detach().clone() for n, p in pair.ll_model.named_parameters()}
    mp.spawn(_worker_single_loss, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    r = [torch.load(tmp_path / f"single{i}.pt", weights_only=True) for i in range(2)]
    assert r[0]["nodes"] == r[1]["nodes"] == ref_nodes
    for n, p in ref_params.items():
        assert torch.equal(r[0]["params"][n], r[1]["params"][n]), n
        assert torch.allclose(r[0]["params"][n], p, atol=2e-5, rtol=1e-4), n
    avg = torch.tensor(r[0]["losses"]) / 2 + torch.tensor(r[1]["losses"]) / 2
    assert torch.allclose(avg, torch.tensor(ref_losses), atol=1e-4)


def test_reducer_defers_launches_for_multi_forward_losses():
    """The forward counter: one grad-enabled forward keeps per-parameter launches; two defer them to finish()."""
    from iit_amd.engine.flat import FlatParams
    from iit_amd.parallel.ddp import GradReducer
    pair, train = _make(64)
    red = GradReducer(FlatParams(pair.ll_model), module=pair.ll_model)
    red.enabled = True  # no process group: only the bookkeeping is exercised (nothing is launched below)
    x = next(iter(train.make_loader(8, 0)))[0][0]
    pair.ll_model(x)
    red.start()
    assert not red.deferred
    pair.ll_model(x)
    pair.ll_model(x)
    red.start()
    assert red.deferred
    from iit_amd.engine import grad_hooks
    for p in pair.ll_model.parameters():  # the fused kernels' per-write reports launch nothing while deferred
        grad_hooks.notify(p)
    assert not any(red._launched)
    with torch.no_grad():
        pair.ll_model(x)
    red.start()
    assert red.deferred  # zero grad-enabled forwards: unknown producer count, stay conservative
    red.remove()


def _worker_zero(rank, world, port, out_dir, staged=False):
    """Optimizer-state sharding (iit_amd/parallel/zero.py): reduce-scatter -> sharded clip + Adam -> all-gather."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    from iit_amd.parallel import dist as pdist
    from iit_amd.parallel.zero import ShardedFusedAdam
    if world == 1:  # the one-rank rehearsal: the shard gradient aliases the arena, no reduce-scatter
        os.environ["IIT_DP_FORCE_REDUCER"] = "1"
    pdist.init_distributed("gloo")
    torch.set_num_threads(2)
    pair, train = _make(64)
    pair.training_args.update(zero=True, fused_optimizer=True)
    pdist.broadcast_module(pair.ll_model)
    per_rank = 64 // world
    if staged:
        from iit_amd.engine.graphs import GraphedTrainStep
        opt = pair.make_optimizer(1e-3)
        step = GraphedTrainStep(pair, opt, pair.loss_fn, warmup=10 ** 9, enabled=True)
        assert step.split and step.staged is not None
        torch.manual_seed(5)
        for i, (base, abl) in enumerate(train.make_loader(per_rank, 0)):
            if i >= 3:
                break
            step(base, abl)
    else:
        opt = pair.make_optimizer(1e-3)
        pair.restrict_sparse_rows(train)  # the shard span tables skip the unreachable embedding rows (exact)
        torch.manual_seed(5)
        for i, (base, abl) in enumerate(train.make_loader(per_rank, 0)):
            if i >= 3:
                break
            pair.run_train_step(base, abl, pair.loss_fn, opt)
        assert pair._ll_module()._flat_params.inactive_ranges(), "no rows restricted"
    assert isinstance(opt, ShardedFusedAdam) and pair._reducer.shard is opt
    assert opt.alias == (world == 1)
    # the all-gather of the last step is deferred to the next forward's gates: a direct read finishes it first
    assert opt._gate_groups is not None
    if world > 1:
        assert opt._pending  # issued, not waited for
        with torch.no_grad():
            pair.ll_model(base[0])  # the forward's gates finish every bucket, block by block
        assert not opt._pending
    pair.optimizer = opt
    pair.sync_params()
    assert not opt._pending
    flat = opt.flat
    assert opt.exp_avg.numel() <= flat.numel // world + 64 * len(opt.plan.buckets)  # moments are sharded
    torch.save({n: p.detach().clone() for n, p in pair.ll_model.named_parameters()},
               os.path.join(out_dir, f"zero{rank}.pt"))
    pdist.destroy()


def _worker_zero_staged(rank, world, port, out_dir):
    _worker_zero(rank, world, port, out_dir, staged=True)


@pytest.mark.parametrize("world,staged", [(1, False), (2, False), (4, False), (2, True)])
def test_zero1_sharded_optimizer_equals_single_process(tmp_path, world, staged, monkeypatch):
    # foreign pieces are NaN until their deferred gather is finished: a weight read that bypasses the forward's
    # gates would make the result NaN (and unequal to the single-process run)
    monkeypatch.setenv("IIT_ZERO_POISON", "1")
    """ZeRO-1 at world 2 and 4 (and under the staged DP schedule) reproduces the single-process run to fp32 tolerance
    -- every rank ends with identical weights."""
    pair, train = _make(64)
    _train(pair, train, per_rank_batch=64, steps=3)
    ref = {n: p.detach().clone() for n, p in pair.ll_model.named_parameters()}
    mp.spawn(_worker_zero_staged if staged else _worker_zero, args=(world, _free_port(), str(tmp_path)),
             nprocs=world, join=True)
    got = [torch.load(tmp_path / f"zero{i}.pt", weights_only=True) for i in range(world)]
    for n, p in ref.items():
        for i in range(world):
            assert torch.equal(got[i][n], got[0][n]), (i, n)
            assert torch.allclose(got[i][n], p, atol=3e-5, rtol=2e-4), (i, n, float((got[i][n] - p).abs().max()))


def _worker_zero_resume(rank, world, port, out_dir):
    """each rank saves and reloads ITS OWN moment shard; a shard offered to the wrong rank raises."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    from iit_amd.parallel import dist as pdist
    from iit_amd.utils import checkpoint as ck
    pdist.init_distributed("gloo")
    torch.set_num_threads(2)
    pair, train = _make(64)
    pair.training_args.update(zero=True, fused_optimizer=True)
    pdist.broadcast_module(pair.ll_model)
    opt = pair.make_optimizer(1e-3)
    torch.manual_seed(5)
    for i, (base, abl) in enumerate(train.make_loader(64 // world, 0)):
        if i >= 2:
            break
        pair.run_train_step(base, abl, pair.loss_fn, opt)
    ckdir = os.path.join(out_dir, "ck")
    ck.save_resume_state(ckdir, pair, opt, None, epoch=1)
    pdist.barrier()
    saved_m, saved_v = opt.exp_avg.clone(), opt.exp_avg_sq.clone()
    opt.exp_avg.zero_()
    opt.exp_avg_sq.zero_()
    assert ck.load_resume_state(ckdir, pair, opt, None) == 1
    assert torch.equal(opt.exp_avg, saved_m) and torch.equal(opt.exp_avg_sq, saved_v)
    other = torch.load(os.path.join(ckdir, f"resume_optim_rank{1 - rank}.pt"), weights_only=True)
    with pytest.raises(ValueError):
        opt.load_state_dict(other)
    torch.save({"m": saved_m}, os.path.join(out_dir, f"zr{rank}.pt"))
    pdist.destroy()


def test_zero1_resume_restores_each_ranks_own_shard(tmp_path):
    mp.spawn(_worker_zero_resume, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    m0 = torch.load(tmp_path / "zr0.pt", weights_only=True)["m"]
    m1 = torch.load(tmp_path / "zr1.pt", weights_only=True)["m"]
    assert not torch.equal(m0, m1)  # the shards differ, so loading rank 0's everywhere would have been wrong


def _worker_metrics(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    from iit_amd.core.metric import MetricStore, MetricStoreCollection, MetricType, PerTokenMetricStore
    from iit_amd.model_pairs.base_model_pair import BaseModelPair
    from iit_amd.parallel import dist as pdist
    pdist.init_distributed("gloo")
    mc = MetricStoreCollection([MetricStore("val/IIA", MetricType.ACCURACY), MetricStore("val/loss", MetricType.LOSS),
                                PerTokenMetricStore("val/per_token_accuracy")])
    # unequal batch counts per rank: rank 0 three batches, rank 1 one
    vals = [(1.0, 2.0), (1.0, 4.0), (0.0, 6.0)] if rank == 0 else [(0.0, 10.0)]
    for a, l in vals:
        mc.update({"val/IIA": a, "val/loss": l, "val/per_token_accuracy": torch.tensor([a, 1.0 - a]).numpy()})
    BaseModelPair._reduce_metrics(mc)
    torch.save({m.get_name(): torch.as_tensor(m.get_value()) for m in mc.metrics}, os.path.join(out_dir, f"m{rank}.pt"))
    pdist.destroy()


def test_metric_reduction_weights_by_batch_counts(tmp_path):
    """epoch metrics are all-reduced as sums and counts, so ranks with unequal numbers of
    batches give the single-process mean (4 batches in all), not a mean of per-rank means."""
    mp.spawn(_worker_metrics, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    for r in range(2):
        m = torch.load(tmp_path / f"m{r}.pt", weights_only=True)
        assert float(m["val/IIA"]) == pytest.approx(50.0)  # (1 + 1 + 0 + 0) / 4 x 100
        assert float(m["val/loss"]) == pytest.approx(5.5)  # (2 + 4 + 6 + 10) / 4
        assert torch.allclose(m["val/per_token_accuracy"].double(), torch.tensor([0.5, 0.5], dtype=torch.float64))


def _torchrun(tmp, fault, extra=()):
    env = dict(os.environ, OMP_NUM_THREADS="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--max-restarts", "1",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(ROOT, "tests", "dp_restart_worker.py"), str(tmp), str(fault), *extra]
    tmp.mkdir(parents=True, exist_ok=True)
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=900, env=env, cwd=str(tmp))
    assert out.returncode == 0, (out.stdout[-2000:], out.stderr[-4000:])
    return torch.load(tmp / "final.pt", weights_only=True)


@pytest.mark.parametrize("extra", [(), ("zero",)])
def test_dp2_rank_failure_restart_resumes(tmp_path, extra):
    """SURVEY §5.3 / VERDICT r4 missing #4: rank 1 dies hard (os._exit) after the epoch-0 checkpoint; torchrun
    (--max-restarts 1) restarts both ranks, which resume from their per-rank checkpoints (weights, optimizer state --
    each rank's own ZeRO-1 shard --, every RNG) and finish with exactly the weights of an uninterrupted run."""
    ref = _torchrun(tmp_path / "ref", 0, extra)
    got = _torchrun(tmp_path / "fault", 1, extra)
    assert ref["attempt"] == 0 and got["attempt"] == 1  # the fault run really restarted
    for n, p in ref["params"].items():
        assert torch.equal(got["params"][n], p), n
