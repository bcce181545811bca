"""Executed matrix FLOPs of the headline training step (quote executed, not reference-semantics,
FLOPs).  Runs bench.py's configuration eagerly (graphs off) and counts 2*M*N*K of every GEMM the engine issues through
the dispatcher (``gemm_dispatch.gemm``: forward, input- and weight-gradient GEMMs, hipBLASLt or the repo's kernels)
plus the short-sequence attention products (QK^T and PV, forward; 2x that backward), averaged over ``--steps``
sampled steps (the IIT / strict nodes, hence the source-run depth, vary per step).

    python scripts/count_step_flops.py --steps 40
"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=40)
    a = ap.parse_args()
    import bench
    from iit_amd.ops import gemm_dispatch as gd
    from iit_amd.ops import hip_kernels as K

    counts = {"gemm": 0.0, "attn": 0.0, "calls": 0}
    orig_gemm = gd.gemm

    depth = [0]

    def counting_gemm(A, B, C, *, M, N, K, **kw):
        if not kw.get("_decide_only") and depth[0] == 0:  # outermost call only (ragged bulk / tail splits recurse)
            counts["gemm"] += 2.0 * M * N * K
            counts["calls"] += 1
        depth[0] += 1
        try:
            return orig_gemm(A, B, C, M=M, N=N, K=K, **kw)
        finally:
            depth[0] -= 1

    gd.gemm = counting_gemm
    import iit_amd.ops.hip_ops as ho
    ho.gemm = counting_gemm
    orig_fwd, orig_bwd, orig_pair = K.attn_small_fwd, K.attn_small_bwd, K.attn_pair_fwd

    def attn_flops(B, S, H, dh, mult):
        counts["attn"] += mult * 2.0 * 2 * B * H * S * S * dh  # QK^T and PV

    K.attn_small_fwd = lambda *x, **k: (attn_flops(x[5], x[6], x[7], x[8], 1), orig_fwd(*x, **k))[1]
    K.attn_small_bwd = lambda *x, **k: (attn_flops(x[5], x[6], x[7], x[8], 2), orig_bwd(*x, **k))[1]
    K.attn_pair_fwd = lambda *x, **k: (attn_flops(x[3], x[4], x[5], x[6], 1), orig_pair(*x, **k))[1]

    args = argparse.Namespace(gpus=1, steps=1, warmup=1, batch=256, model="gpt2-small", engine="native", dtype="bf16",
                              graphs=0, profile_dir=None)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    pair, opt, loss_fn, it, step_fn, _, _ = bench.setup(args, dev)
    base, abl = next(it)
    step_fn(base, abl, loss_fn, opt)  # GEMM autotuning happens here: not counted
    for k in counts:
        counts[k] = 0
    for _ in range(a.steps):
        base, abl = next(it)
        step_fn(base, abl, loss_fn, opt)
    torch.cuda.synchronize()
    per = {k: v / a.steps for k, v in counts.items()}
    print(json.dumps({"executed_tflop_per_step": round((per["gemm"] + per["attn"]) / 1e12, 3),
                      "gemm_tflop_per_step": round(per["gemm"] / 1e12, 3),
                      "attention_tflop_per_step": round(per["attn"] / 1e12, 4),
                      "gemm_calls_per_step": round(per["calls"], 1), "steps": a.steps,
                      "config": "bench.py: IOI GPT-2-small, B=256, S=16, IOI_ModelPair (IIT + strict + behaviour), "
                                "paired source+base forward, last-position logits"}))


if __name__ == "__main__":
    main()
