"""Headline benchmark: IIT (base, source) intervened pairs/sec on IOI with a GPT-2-small LL model.

Config (BASELINE.json): IOI task, LL = GPT-2-small architecture (12L / 768d / 12H,
d_mlp 3072, V 50257, LNPre, gelu_new) with random init, bf16 compute (fp32
master weights / Adam), IOI_ModelPair strict IIT + behaviour multi-task step
exactly as ``train_ioi.py`` (batch 256 per GPU, Adam lr 1e-4, weights
iit/behaviour/strict = 1/1/0.4, clip 1.0): per step one IIT, one strict and one
behaviour optimizer update (3 backward passes, 5 LL forwards, 2 HL forwards).
Data: synthetic offline IOI prompts (BOS + 16 tokens), see iit_amd.tasks.ioi.

Weak scaling (default): every rank processes ``--batch`` pairs per step; the value is the
whole-job rate (global pairs / max-over-ranks step time).  Strong scaling: ``--global-batch B``
holds the job's batch at B (``train_ioi.py``'s 256) and splits it over the ranks.

    python bench.py --gpus 1 --steps 20 --warmup 5
    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 bench.py --gpus 8
    python bench.py --gpus 8          # no launcher: bench.py starts the 8 ranks itself (torch.distributed.run)

``--gpus N`` is binding: without a launcher environment and N > 1 the script launches N fresh rank
processes (the parent makes no GPU call first and only relays their output); under a launcher whose
world size differs from N it exits with status 3 instead of reporting another ``n_gpus``.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=256, help="pairs per GPU per step (weak scaling)")
    ap.add_argument("--global-batch", type=int, default=None,
                    help="strong scaling: pairs per step over the whole job, split over the ranks")
    ap.add_argument("--model", default="gpt2-small", choices=["gpt2-small", "ioi-6l"])
    ap.add_argument("--engine", default="native", choices=["native", "reference"],
                    help="reference = reference-semantics eager path (hook closures, full caches, full logits)")
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--graphs", type=int, default=int(os.environ.get("IIT_GRAPHS", "1")),
                    help="capture each train-step phase as a HIP graph (default on; 0 = eager)")
    ap.add_argument("--profile-dir", default=None)
    return ap.parse_args()


def setup(args, dev):
    """Model pair, optimizer and batch iterator of the headline config (shared with scripts/torch_profile.py)."""
    from iit_amd.data.iit_dataset import IITDataset, train_test_split
    from iit_amd.model_pairs import IOI_ModelPair
    from iit_amd.models.config import gpt2_config_dict
    from iit_amd.models.transformer import HookedTransformer
    from iit_amd.parallel import dist as pdist
    from iit_amd.tasks.ioi import ioi_cfg, make_ioi_corr, make_ioi_dataset_and_hl

    torch.manual_seed(0)
    np.random.seed(0)
    cfg = gpt2_config_dict()
    if args.model == "ioi-6l":
        cfg.update(ioi_cfg)
    tiny = os.environ.get("IIT_BENCH_TINY") == "1"  # CPU rehearsal of the launch path only (tests)
    if tiny:
        cfg.update(n_layers=2, d_model=16, n_heads=2, d_head=8, d_mlp=32)
        args.batch = min(args.batch, 16)
    cfg.update(device=str(dev), init_weights=True,
               dtype=torch.bfloat16 if args.dtype == "bf16" else torch.float32)
    ll = HookedTransformer(cfg)
    if args.engine == "reference" or args.dtype == "fp32":
        ll.set_op_backend("torch")
    ds, hl = make_ioi_dataset_and_hl(512 if tiny else 12000, ll, device=dev,
                                     label_format="onehot" if args.engine == "reference" else "index")
    train_ds, test_ds = train_test_split(ds, test_size=0.2, random_state=42)
    train_set = IITDataset(train_ds, train_ds, seed=0, device=dev)
    test_set = IITDataset(test_ds, test_ds, seed=0, device=dev)
    training_args = {"batch_size": args.batch, "lr": 1e-4, "iit_weight": 1.0, "behavior_weight": 1.0,
                     "strict_weight": 0.4, "next_token": False, "lr_scheduler": None, "clip_grad_norm": 1.0,
                     "early_stop": True, "use_single_loss": False, "engine": args.engine}
    pair = IOI_ModelPair(ll_model=ll, hl_model=hl, corr=make_ioi_corr(cfg["n_layers"]), training_args=training_args)
    pdist.broadcast_module(ll)
    opt = pair.make_optimizer(training_args["lr"])
    pair.restrict_sparse_rows(train_set)  # reduce / update only embedding rows the data can reach (exact)
    loss_fn = pair.loss_fn
    loader = train_set.make_loader(args.batch, 0)

    def batches():
        # full batches only: an epoch's short last batch would run eagerly (new shapes) inside the timed window
        # and carry fewer pairs than the rate counts
        while True:
            for b in loader:
                if b[0][0].shape[0] == args.batch:
                    yield b

    it = batches()
    step_fn = pair.run_train_step
    # graphs on the fused HIP backend (bf16); the fp32 torch-op backend runs eagerly (see train_step_fn)
    if args.graphs and dev.type == "cuda" and args.engine == "native" and args.dtype == "bf16":
        from iit_amd.engine.graphs import GraphedTrainStep
        g = GraphedTrainStep(pair, opt, loss_fn)
        if g.enabled:
            step_fn = g
    return pair, opt, loss_fn, it, step_fn, train_set, test_set


# the reference publishes no throughput; its semantics (fp32, eager hook closures, full-vocab
# logits, torch Adam) measured on one MI355X with ``--engine reference --dtype fp32 --graphs 0 --steps 20``
# (round 6 at HEAD, profiles/iia_6l_seeds_r6.txt: 153.9 ms/step; round 1's 5-step figure was 1,559.65)
REFERENCE_EAGER_PAIRS_PER_S = 1663.5


def _free_port() -> int:
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def self_launch(n: int) -> int:
    """``--gpus N`` without a launcher: run this script as N ranks under ``torch.distributed.run`` (one process per
    GPU, rendezvous on 127.0.0.1) as a CHILD process -- nothing here has touched the GPU, and the parent only waits
    and returns the launcher's exit status.  Rank 0's JSON line reaches stdout through the inherited descriptors."""
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__)] + sys.argv[1:]
    print(f"[bench] --gpus {n} without a launcher: starting {n} ranks ({' '.join(cmd[1:6])} ...)", file=sys.stderr,
          flush=True)
    return subprocess.call(cmd, env=dict(os.environ, IIT_BENCH_SELF_LAUNCHED="1"))


def main():
    args = parse()
    if args.gpus < 1:
        print(f"[bench] --gpus must be >= 1 (got {args.gpus})", file=sys.stderr)
        sys.exit(3)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(self_launch(args.gpus))
    from iit_amd.parallel import dist as pdist
    distributed = pdist.init_distributed()
    rank, world = pdist.rank(), pdist.world_size()
    if world != args.gpus:
        # never report another n_gpus than was asked for (VERDICT r5 missing #4)
        print(f"[bench] rank {rank}: the launcher started {world} rank(s) but --gpus {args.gpus} was requested",
              file=sys.stderr, flush=True)
        pdist.destroy()
        sys.exit(3)
    strong = args.global_batch is not None
    if strong:
        if args.global_batch % world:
            print(f"[bench] --global-batch {args.global_batch} does not split over {world} ranks", file=sys.stderr)
            pdist.destroy()
            sys.exit(3)
        args.batch = args.global_batch // world
    if torch.cuda.is_available():
        torch.cuda.set_device(pdist.local_device_index())
    dev = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu")

    pair, opt, loss_fn, it, step_fn, train_set, test_set = setup(args, dev)

    import contextlib
    # the whole loop runs on the graph runner's stream (batches included): no per-step stream handoff
    ctx = (step_fn.stream_context() if hasattr(step_fn, "stream_context") and os.environ.get("IIT_BENCH_STREAM_CTX") != "0"
           else contextlib.nullcontext())
    with ctx:
        for i in range(args.warmup):
            base, abl = next(it)
            if i == 0 and hasattr(step_fn, "prime"):
                step_fn.prime(base, abl, loss_fn, opt)  # capture every phase graph before timing
            step_fn(base, abl, loss_fn, opt)
        from iit_amd.ops.gemm_dispatch import sync_decisions
        sync_decisions()  # (collective) every rank times the same kernels: rank 0's GEMM choices
        pdist.barrier()
        if dev.type == "cuda":
            torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            base, abl = next(it)  # the device-side batch gather is part of the timed step
            out = step_fn(base, abl, loss_fn, opt)
        t_host = time.perf_counter() - t0  # (host enqueue time: close to the wall time = launch-bound)
        if dev.type == "cuda":
            torch.cuda.synchronize()
        pdist.barrier()
        dt = time.perf_counter() - t0
    executed = getattr(step_fn, "calls", None) or (args.warmup + args.steps)
    print(f"[bench] train steps executed in this process: {executed}; host enqueue {t_host / args.steps * 1e3:.3f} "
          f"ms/step of {dt / args.steps * 1e3:.3f} ms/step wall", file=sys.stderr)
    dt_t = torch.tensor([dt], dtype=torch.float64, device=dev if distributed and dev.type == "cuda" else "cpu")
    if distributed:
        torch.distributed.all_reduce(dt_t, op=torch.distributed.ReduceOp.MAX)
    dt = float(dt_t.item())
    ms = dt / args.steps * 1000.0
    global_batch = args.batch * world
    value = global_batch * args.steps / dt

    # IIA / accuracy on held-out pairs (outside the timed region)
    metrics = pair.make_test_metrics()
    with torch.no_grad():
        for i, (base, abl) in enumerate(test_set.make_loader(args.batch, 0)):
            metrics.update(pair.run_eval_step(base, abl, loss_fn))
            if i >= 3:
                break
    vals = metrics.to_dict()
    train_loss = {k: float(v) for k, v in out.items()} if isinstance(out, dict) else {}

    if rank == 0:
        rec = {
            "metric": "IIT (base,source) intervened pairs/sec, IOI GPT-2-small, IOI_ModelPair IIT+strict+behavior step",
            "value": round(value, 2),
            "unit": "pairs/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms, 3),
            "higher_is_better": True,
            "scaling": "strong" if strong else "weak",
            "vs_baseline": (round(value / REFERENCE_EAGER_PAIRS_PER_S, 3)
                            if args.model == "gpt2-small" and os.environ.get("IIT_BENCH_TINY") != "1" else None),
            "baseline": "reference-equivalent eager fp32 engine on 1x MI355X (BASELINE.md; the reference "
                        "publishes no number)",
            "dtype": args.dtype,
            "data": "synthetic (offline IOI prompts, random-init weights)",
            "config": {"model": ("tiny-test 2L/16d (launch rehearsal, not a measurement)"
                                 if os.environ.get("IIT_BENCH_TINY") == "1" else
                                 "gpt2-small 12L/768d/12H (TL GPT-2 cfg, LNPre, gelu_new, V=50257)"
                                 if args.model == "gpt2-small" else "ioi-6l 6L/64d/4H"),
                       "global_batch": global_batch, "seq_len": int(train_set.base_data.dataset.prompts.shape[1] - 1),
                       "parallelism": f"dp{world}", "engine": args.engine,
                       "graphs": bool(getattr(step_fn, "enabled", False))},
            "val_IIA": round(float(vals["val/IIA"]), 3),
            "val_accuracy": round(float(vals["val/accuracy"]), 3),
            "last_train_losses": {k: round(v, 4) for k, v in train_loss.items()},
        }
        print(json.dumps(rec))
        if os.environ.get("IIT_GEMM_REPORT"):
            from iit_amd.ops import gemm_dispatch
            with open(os.environ["IIT_GEMM_REPORT"], "w") as f:
                f.write(gemm_dispatch.report())
        if os.environ.get("IIT_GEMM_TABLE_EXPORT"):  # regenerate iit_amd/ops/tuned/gemm_decisions_gfx950.json
            from iit_amd.ops import gemm_dispatch
            gemm_dispatch.export_table(os.environ["IIT_GEMM_TABLE_EXPORT"])
    pdist.destroy()


if __name__ == "__main__":
    main()
