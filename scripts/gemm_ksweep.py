"""K-sweep of the LDS-DMA GEMM tiles: time(K) = fixed (launch + prologue + epilogue) + K * per-K cost.
Separates the main-loop rate (slope, TFLOP/s of the loop alone) from the fixed overhead (intercept) per tile."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from iit_amd.ops import gemm_dispatch as gd  # noqa: E402
from iit_amd.ops import hip_kernels as K  # noqa: E402

CASES = [  # (name, M, N, mode, epi, tile)
    ("fwd 256x192 bf16", 4096, 3072, 2, 0, 5),
    ("fwd 256x192 gelu", 4096, 3072, 2, 3, 5),
    ("fwd 128x128w8 bf16", 4096, 3072, 2, 0, 6),
    ("fwd 128x128s4 bf16", 4096, 3072, 2, 0, 4),
    ("dX 128x96 bf16", 4096, 768, 0, 0, 9),
    ("dW 96x96 acc", 768, 3072, 3, 5, 8),
    ("dW 128x128 acc", 768, 3072, 3, 5, 0),
]
KS = [256, 512, 768, 1536, 3072, 6144]


def main():
    dev = "cuda"
    for name, M, N, mode, epi, tile in CASES:
        ts, tb = [], []
        for Kd in KS:
            torch.manual_seed(0)
            A = (torch.randn(Kd, M) if mode & 1 else torch.randn(M, Kd)).to(dev).bfloat16()
            B = (torch.randn(Kd, N) if mode & 2 else torch.randn(N, Kd)).to(dev).bfloat16() / 16
            lda = M if mode & 1 else Kd
            ldb = N if mode & 2 else Kd
            C = torch.zeros(M, N, device=dev, dtype=torch.float32 if epi == 5 else torch.bfloat16)
            C2 = torch.zeros(M, N, device=dev, dtype=torch.bfloat16) if epi == 3 else None
            bias = torch.randn(N, device=dev) if epi == 3 else None
            kw = dict(M=M, N=N, K=Kd, lda=lda, ldb=ldb, ldc=N, mode=mode, epi=epi)
            ex = dict(C2=C2, ldc2=N, bias0=bias) if epi == 3 else {}
            assert K.gemm_glds_ok(A, B, C, C2=C2, ldc2=N if C2 is not None else 0, tile=tile, **kw)
            ts.append(min(gd._time(lambda: K.gemm_glds(A, B, C, tile=tile, **kw, **ex), reps=20) for _ in range(3)))
            a = A.t() if mode & 1 else A
            b = B if mode & 2 else B.t()
            tb.append(min(gd._time(lambda: torch.mm(a, b), reps=20) for _ in range(3)))
        slope, icpt = np.polyfit(KS, ts, 1)
        bslope, bicpt = np.polyfit(KS, tb, 1)
        loop_tf = 2 * M * N / (slope * 1e-6) / 1e12
        bl_tf = 2 * M * N / (bslope * 1e-6) / 1e12
        print(f"{name:22s} M={M} N={N}  glds us: " + " ".join(f"{t:7.1f}" for t in ts)
              + f" | fixed {icpt:6.1f} us, loop {loop_tf:6.0f} TF/s   blas us: " + " ".join(f"{t:7.1f}" for t in tb)
              + f" | fixed {bicpt:6.1f} us, loop {bl_tf:6.0f} TF/s", flush=True)


if __name__ == "__main__":
    main()
