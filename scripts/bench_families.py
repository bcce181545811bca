"""Throughput of the other BASELINE.json configurations (the headline IOI GPT-2-small number is ``bench.py``).

* ``mqnli-bert-base``   -- MQNLI natural-logic causal model <-> BERT-base (12L/768d/12H, post-LN, GELU),
  ``IITBehaviorModelPair`` (IIT + behaviour: 2 optimizer steps per batch), 15-token sentence pairs;
* ``llama3-8b-causal``  -- 8-node arithmetic causal graph <-> Llama-3-8B (32L/4096d, 32 q / 8 kv heads, SwiGLU
  14336, RMSNorm, rotary, V=128256), ``CausalGraphModelPair`` (IIT + strict + behaviour: 3 optimizer steps),
  6-token prompts (``--seq 512``: a 506-token filler context before the operands, so the captured source
  activations -- ``attn.hook_z`` / ``mlp.hook_post`` over B x S tokens -- are GB-scale).  fp32 master weights + Adam
  moments + gradients = 128 GB, bf16 compute;
* ``pvr-resnet18``      -- MNIST-PVR pointer-value-retrieval HL <-> ResNet-18 (torchvision layout, fc 512->10),
  ``IITBehaviorModelPair`` exactly as ``train.py`` (lr 1e-3, batch 256), 84 x 84 RGB 2 x 2 digit tiles, spatial
  quadrant splice at ``mod.layer3.mod.1.mod.conv2.hook_point``; fp32 (the reference precision; MIOpen convolutions)
  or ``--dtype bf16`` (channels-last bf16 autocast).

Random-init weights of the named architectures, synthetic task data; same timing contract as ``bench.py``
(W untimed warmup steps, then K steps bracketed by barrier + synchronize, max over ranks; one JSON line)."""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--family", required=True, choices=["mqnli-bert-base", "llama3-8b-causal", "llama-tiny-causal",
                                                         "mqnli-bert-tiny", "pvr-resnet18"])
    ap.add_argument("--seq", type=int, default=6, help="causal-graph prompt length (>= 6; Llama families)")
    ap.add_argument("--zero", type=int, default=0, help="optimizer-state sharding (ZeRO-1) under data parallelism")
    ap.add_argument("--zero-overlap", type=int, default=1,
                    help="ZeRO-1: defer the all-gather of the updated pieces to the next forward's per-block gates")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--batch", type=int, default=None, help="pairs per GPU per step")
    ap.add_argument("--dtype", choices=["fp32", "bf16"], default="fp32",
                    help="pvr-resnet18 only: fp32 (the reference precision) or channels-last bf16 autocast")
    ap.add_argument("--channels-last", type=int, default=None,
                    help="pvr-resnet18: NHWC model and activations (default on)")
    ap.add_argument("--graphs", type=int, default=None,
                    help="HIP-graph phases (default: on for BERT; off for Llama, whose strict phase has one graph per "
                         "non-circuit node -- ~1000 at 32 layers x 32 heads -- and whose GEMMs are not launch-bound)")
    return ap.parse_args(argv)


def setup(args, dev):
    from iit_amd.data.iit_dataset import IITDataset, train_test_split
    torch.manual_seed(0)
    np.random.seed(0)
    if args.family.startswith("mqnli"):
        from iit_amd.model_pairs import IITBehaviorModelPair
        from iit_amd.models.bert import HookedEncoder, bert_config_dict
        from iit_amd.tasks.mqnli import VOCAB, make_mqnli_task
        size = "bert-base" if args.family == "mqnli-bert-base" else "bert-tiny"
        cfg = bert_config_dict(size, d_vocab=max(VOCAB, 64), device=str(dev), dtype=torch.bfloat16)
        ll = HookedEncoder(cfg, n_classes=3)
        ds, hl, corr = make_mqnli_task(ll, n_samples=20000, device=dev)
        args.batch = args.batch or 256
        pair = IITBehaviorModelPair(hl, ll, corr, training_args={"batch_size": args.batch, "lr": 1e-4,
                                                                  "lr_scheduler": None, "early_stop": False,
                                                                  "clip_grad_norm": 1.0})
        model_name = f"{size} + MQNLI natural-logic HL (10 nodes)"
        seq = 15
    elif args.family == "pvr-resnet18":
        from iit_amd.model_pairs import IITBehaviorModelPair
        # MIOpen find mode: the fastest measured convolution solution per shape (bf16 step 12.5 -> 9.0 ms,
        # profiles/pvr_step_r5.txt); IIT_CONV_BENCHMARK=0 keeps MIOpen's immediate-mode heuristic
        torch.backends.cudnn.benchmark = os.environ.get("IIT_CONV_BENCHMARK", "1") == "1"
        from iit_amd.tasks.task_loader import get_alignment, get_dataset
        n = 20000
        tr_set, te_set = get_dataset("mnist_pvr", {"train_size": n, "test_size": 2048, "device": dev})
        ll, hl, corr = get_alignment("mnist_pvr", {"input_shape": te_set.base_data.get_input_shape(), "device": dev})
        # NHWC for both dtypes: the fused NHWC BatchNorm / pool kernels take bf16 and fp32 (fp32 PVR step 18.9 ->
        # 14.6 ms, profiles/bn_fp32_r5.txt)
        cl = args.channels_last if args.channels_last is not None else 1
        if cl:  # NHWC activations for MIOpen's implicit-GEMM convolutions (and the fused NHWC BatchNorm)
            ll.to(memory_format=torch.channels_last)
        args.batch = args.batch or 256
        pair = IITBehaviorModelPair(hl, ll, corr, training_args={"batch_size": args.batch, "lr": 1e-3,
                                                                  "lr_scheduler": None, "early_stop": False,
                                                                  "zero": bool(args.zero)})
        model_name = "resnet18 (fc 512->10) + MNIST-PVR HL, quadrant splice at layer3.1.conv2"
        seq = 84
        ds = tr_set.base_data
    else:
        from iit_amd.models.convert import llama_config_dict
        from iit_amd.models.transformer import HookedTransformer
        from iit_amd.tasks.causal_graph import CausalGraphModelPair, make_causal_graph_task
        size = "llama-3-8b" if args.family == "llama3-8b-causal" else "llama-tiny"
        cfg = llama_config_dict(size, device=str(dev), dtype=torch.bfloat16)
        ll = HookedTransformer(cfg)
        ds, hl, corr = make_causal_graph_task(ll, n_samples=10000, device=dev, seq_len=args.seq)
        args.batch = args.batch or (64 if args.seq <= 16 else max(1, 8192 // args.seq))
        pair = CausalGraphModelPair(hl, ll, corr, training_args={"batch_size": args.batch, "lr": 1e-5,
                                                                  "lr_scheduler": None, "early_stop": False,
                                                                  "strict_weight": 0.4, "clip_grad_norm": 1.0})
        model_name = f"{size} + 8-node arithmetic causal graph"
        seq = args.seq
        pair.training_args["zero"] = bool(args.zero)
    pair.training_args["zero_overlap_gather"] = bool(args.zero_overlap)
    from iit_amd.parallel import dist as pdist
    pdist.broadcast_module(ll)
    if args.family == "pvr-resnet18":
        train_set, test_set = tr_set, te_set
    else:
        tr, te = train_test_split(ds, 0.1, 42)
        train_set = IITDataset(tr, tr, seed=0, device=dev)
        test_set = IITDataset(te, te, seed=0, device=dev)
    opt = pair.make_optimizer(pair.training_args["lr"])
    pair.restrict_sparse_rows(train_set)
    loader = train_set.make_loader(args.batch, 0)

    def batches():
        while True:
            for b in loader:
                yield b

    step_fn = pair.run_train_step
    if args.graphs is None:
        args.graphs = int(args.family.startswith("mqnli") or args.family.startswith("pvr"))
    if args.graphs and dev.type == "cuda":
        from iit_amd.engine.graphs import GraphedTrainStep
        g = GraphedTrainStep(pair, opt, pair.loss_fn)
        if g.enabled:
            step_fn = g
    return pair, opt, batches(), step_fn, test_set, model_name, seq


def main():
    args = parse()
    from iit_amd.parallel import dist as pdist
    distributed = pdist.init_distributed()
    rank, world = pdist.rank(), pdist.world_size()
    if torch.cuda.is_available():
        torch.cuda.set_device(pdist.local_device_index())  # (0 for every rank under IIT_REHEARSE_ONE_GPU=1)
    dev = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu")
    t_setup = time.perf_counter()
    pair, opt, it, step_fn, test_set, model_name, seq = setup(args, dev)
    t_setup = time.perf_counter() - t_setup
    if args.dtype == "bf16" and args.family.startswith("pvr"):
        import contextlib
        inner = step_fn
        # no autocast weight-cast cache: the casts must be re-done inside every captured / replayed graph
        amp = (lambda: torch.autocast("cuda", dtype=torch.bfloat16, cache_enabled=False)) if dev.type == "cuda" \
            else contextlib.nullcontext

        class _Amp:
            enabled = getattr(inner, "enabled", False)

            def prime(self, *a):
                if hasattr(inner, "prime"):
                    with amp():
                        inner.prime(*a)

            def __call__(self, *a):
                with amp():
                    return inner(*a)

        step_fn = _Amp()
    for i in range(args.warmup):
        base, abl = next(it)
        if i == 0 and hasattr(step_fn, "prime"):
            step_fn.prime(base, abl, pair.loss_fn, opt)
        step_fn(base, abl, pair.loss_fn, opt)
    timed = [next(it) for _ in range(args.steps)]
    pdist.barrier()
    if dev.type == "cuda":
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    for base, abl in timed:
        out = step_fn(base, abl, pair.loss_fn, opt)
    if dev.type == "cuda":
        torch.cuda.synchronize()
    pdist.barrier()
    dt = time.perf_counter() - t0
    dt_t = torch.tensor([dt], dtype=torch.float64, device=dev if distributed and dev.type == "cuda" else "cpu")
    if distributed:
        torch.distributed.all_reduce(dt_t, op=torch.distributed.ReduceOp.MAX)
    dt = float(dt_t.item())
    pair.optimizer = opt
    pair.sync_params()
    flat = getattr(pair._ll_module(), "_flat_params", None)
    wsum = float(flat.data.double().sum()) if flat is not None else None  # (bitwise-comparable weight checksum)
    metrics = pair.make_test_metrics()
    with torch.no_grad():
        for i, (base, abl) in enumerate(test_set.make_loader(args.batch, 0)):
            metrics.update(pair.run_eval_step(base, abl, pair.loss_fn))
            if i >= 1:
                break
    vals = metrics.to_dict()
    if rank == 0:
        n_params = sum(p.numel() for p in pair._ll_module().parameters())
        print(json.dumps({
            "metric": f"IIT (base,source) intervened pairs/sec, {args.family}", "value": round(
                args.batch * world * args.steps / dt, 2), "unit": "pairs/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(dt / args.steps * 1e3, 3), "higher_is_better": True,
            "scaling": "weak", "dtype": args.dtype if args.family.startswith("pvr") else "bf16",
            "data": "synthetic task data, random-init weights",
            "config": {"model": model_name, "params": n_params, "global_batch": args.batch * world, "seq_len": seq,
                       "parallelism": f"dp{world}", "graphs": bool(getattr(step_fn, "enabled", False))},
            "val_IIA": round(float(vals.get("val/IIA", float("nan"))), 3),
            "setup_s": round(t_setup, 1),
            "peak_mem_gb": round(torch.cuda.max_memory_allocated() / 2 ** 30, 1) if dev.type == "cuda" else None,
            "last_train_losses": {k: round(float(v), 4) for k, v in out.items()} if isinstance(out, dict) else {},
            "weight_checksum": wsum, "zero": bool(args.zero), "zero_overlap_gather": bool(args.zero_overlap),
            "optimizer_skipped_steps": int(getattr(opt, "_skipped_dev", torch.zeros(1)).sum()),
        }))
    if os.environ.get("IIT_CONV_REPORT") == "1" and rank == 0:  # the per-shape conv decisions (ops/conv.py)
        from iit_amd.ops import conv as hconv
        print(hconv.report(), file=sys.stderr)
    pdist.destroy()


if __name__ == "__main__":
    main()
