"""Where a GEMM launch's time goes, per workgroup: the LDS-DMA kernel's timeline probe (csrc/gemm_glds.hip
``G2Args::prof``) records the shader clock at kernel start, when the first K-tile has landed (prologue), after every
later K-tile, at the end of the main loop and after the epilogue's stores have drained, plus the 100 MHz wall clock
at start and end.  Run on L2-hot operands (back to back) and after a 1 GiB sweep evicts them (cold), for the
headline step's shapes on their shipped tiles.

    python scripts/gemm_timeline.py
"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from iit_amd.ops import hip_kernels as K  # noqa: E402

T = 4096
CASES = [  # name, M, N, K, mode, epi, tile
    ("fwd QKV 4096x2304x768 (t5 256x192)", T, 2304, 768, 2, K.EPI_BF16, 5),
    ("fwd W_in+gelu 4096x3072x768 (t5)", T, 3072, 768, 2, K.EPI_GELU, 5),
    ("fwd W_out+resid 4096x768x3072 (t9 128x96)", T, 768, 3072, 2, K.EPI_F32_RESID, 9),
    ("fwd W_out+resid 4096x768x3072 (t24 64x96 x2/CU)", T, 768, 3072, 2, K.EPI_F32_RESID, 24),
    ("dX W_in 4096x768x3072 (t9)", T, 768, 3072, 0, K.EPI_BF16, 9),
    ("dW W_in 768x3072x4096 (t8 96x96)", 768, 3072, T, 3, K.EPI_F32_STORE, 8),
]


def analyse(prof, nwg, nt):
    p = prof.view(nwg, 64).cpu().numpy().astype(np.float64)
    clk = p[:, :63]
    wall0, wall1 = p[:, 63], p[:, 60]
    # shader-clock ticks per microsecond, from each workgroup's own wall / shader spans
    span_clk = clk[:, 62] - clk[:, 0]
    span_us = (wall1 - wall0) / 100.0
    ok = span_us > 0
    tpu = float(np.median(span_clk[ok] / span_us[ok])) if ok.any() else float("nan")
    us = lambda x: x / tpu  # noqa: E731
    pro = us(clk[:, 1] - clk[:, 0])
    steps = us(np.diff(clk[:, 1:nt + 1], axis=1)) if nt > 1 else np.zeros((nwg, 0))
    loop = us(clk[:, 61] - clk[:, 1])
    epi = us(clk[:, 62] - clk[:, 61])
    start = (wall0 - wall0.min()) / 100.0
    end = (wall1 - wall0.min()) / 100.0
    return {"workgroups": nwg, "k_tiles": nt, "shader_ticks_per_us": round(tpu, 1),
            "launch_span_us": round(float(end.max()), 2),
            "start_skew_us (p50/p90/max)": [round(float(np.percentile(start, q)), 2) for q in (50, 90, 100)],
            "prologue_us (p50/p90)": [round(float(np.percentile(pro, q)), 2) for q in (50, 90)],
            "k_step_us (p50/p90)": [round(float(np.percentile(steps, q)), 3) for q in (50, 90)] if steps.size else None,
            "main_loop_us (p50/p90)": [round(float(np.percentile(loop, q)), 2) for q in (50, 90)],
            "epilogue_us (p50/p90)": [round(float(np.percentile(epi, q)), 2) for q in (50, 90)],
            "end_us (p50/max)": [round(float(np.percentile(end, 50)), 2), round(float(end.max()), 2)]}


def main():
    dev = "cuda"
    flush = torch.empty(256 << 20, dtype=torch.float32, device=dev)  # 1 GiB sweep: evicts L2 and the Infinity Cache
    for name, M, N, Kd, mode, epi, tile in CASES:
        torch.manual_seed(0)
        A = (torch.randn(Kd, M) if mode & 1 else torch.randn(M, Kd)).to(dev).bfloat16()
        B = (torch.randn(Kd, N) if mode & 2 else torch.randn(N, Kd)).to(dev).bfloat16() / 16
        lda = M if mode & 1 else Kd
        ldb = N if mode & 2 else Kd
        f32 = epi in (K.EPI_F32_STORE, K.EPI_F32_ACC, K.EPI_F32_RESID)
        C = torch.zeros(M, N, device=dev, dtype=torch.float32 if f32 else torch.bfloat16)
        ex = {}
        if epi == K.EPI_F32_RESID:
            ex = dict(resid=torch.randn(M, N, device=dev), ldr=N)
        if epi == K.EPI_GELU:
            ex = dict(C2=torch.empty(M, N, device=dev, dtype=torch.bfloat16), ldc2=N)
        bm, bn = K.GLDS_TILES[tile]
        nwg = (M // bm) * (N // bn)
        nt = Kd // 64
        prof = torch.zeros(nwg * 64, dtype=torch.int64, device=dev)
        run = lambda: K.gemm_glds(A, B, C, M=M, N=N, K=Kd, lda=lda, ldb=ldb, ldc=N, mode=mode, epi=epi,  # noqa
                                  tile=tile, **ex)
        out = {"gemm": name}
        for label in ("hot", "cold"):
            for _ in range(3):
                run()
            if label == "cold":
                flush.fill_(1.0)
            torch.cuda.synchronize()
            K.gemm_glds_set_prof(prof)
            run()
            torch.cuda.synchronize()
            out[label] = analyse(prof, nwg, nt)
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
