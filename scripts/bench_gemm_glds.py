"""Graph-timed GEMM comparison on the GPT-2-small IIT step shapes: LDS-DMA kernel tiles vs the register-staged
kernel vs hipBLASLt (torch.mm).  Prints one line per shape (microseconds per call, TFLOP/s of the best)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from iit_amd.ops import gemm_dispatch as gd  # noqa: E402
from iit_amd.ops import hip_kernels as K  # noqa: E402

T = 4096
SHAPES = [  # (name, M, N, K, mode, epi)
    ("qkv fwd", T, 2304, 768, 2, 1), ("W_O fwd+resid", T, 768, 768, 2, 2), ("W_in fwd+gelu", T, 3072, 768, 2, 3),
    ("W_out fwd+resid", T, 768, 3072, 2, 2),
    ("dX qkv", T, 768, 2304, 0, 0), ("dX W_O", T, 768, 768, 0, 0), ("dX W_in", T, 768, 3072, 0, 0),
    ("dX W_out", T, 3072, 768, 0, 0),
    ("dW qkv", 768, 2304, T, 3, 5), ("dW W_O", 768, 768, T, 3, 5), ("dW W_in", 768, 3072, T, 3, 5),
    ("dW W_out", 3072, 768, T, 3, 5),
]


def run():
    dev = "cuda"
    print(f"{'shape':18s} {'M':>5s} {'N':>5s} {'K':>5s}  " + "  ".join(f"{c:>8s}" for c in
          ["128x128s3", "128x64s4", "64x128s4", "64x64s4", "128x128s4", "256x192w8", "128x128w8", "256x128w8", "96x96s4", "128x96s4", "hip_old", "blas"]) + "   best TF/s")
    for name, M, N, Kd, mode, epi in SHAPES:
        torch.manual_seed(0)
        A = (torch.randn(Kd, M) if mode & 1 else torch.randn(M, Kd)).to(dev).bfloat16()
        B = (torch.randn(Kd, N) if mode & 2 else torch.randn(N, Kd)).to(dev).bfloat16() / 16
        lda = M if mode & 1 else Kd
        ldb = N if mode & 2 else Kd
        out_bf16 = epi in (0, 1, 3)
        C = torch.zeros(M, N, device=dev, dtype=torch.bfloat16 if out_bf16 else torch.float32)
        C2 = torch.zeros(M, N, device=dev, dtype=torch.bfloat16) if epi == 3 else None
        R = torch.randn(M, N, device=dev) if epi == 2 else None
        bias = torch.randn(N, device=dev)
        b3 = [bias[i * (N // 3):(i + 1) * (N // 3)] for i in range(3)]
        kw = dict(M=M, N=N, K=Kd, lda=lda, ldb=ldb, ldc=N, mode=mode, epi=epi)
        extra = {}
        if epi == 1:
            extra = dict(bias0=b3[0], bias1=b3[1], bias2=b3[2], bias_cols=N // 3)
        elif epi == 2:
            extra = dict(bias0=bias, resid=R, ldr=N)
        elif epi == 3:
            extra = dict(bias0=bias, C2=C2, ldc2=N)
        res = []
        for tile in range(10):
            if K.gemm_glds_ok(A, B, C, C2=C2, resid=R, ldc2=N if C2 is not None else 0, ldr=N if R is not None else 0,
                              bias_cols=extra.get("bias_cols", 0), tile=tile, **{k: kw[k] for k in kw}):
                res.append(gd._time(lambda t=tile: K.gemm_glds(A, B, C, tile=t, **kw, **extra), reps=20))
            else:
                res.append(float("nan"))
        if epi == 5:  # split-K variants of the best tiles for the weight gradients
            for tile, sp in ((0, 2), (4, 2), (3, 2), (0, 4), (3, 4)):
                if K.gemm_glds_ok(A, B, C, tile=tile, splits=sp, **{k: kw[k] for k in kw}):
                    tt = gd._time(lambda t=tile, s_=sp: K.gemm_glds(A, B, C, tile=t, splits=s_, **kw), reps=20)
                    print(f"    split-K tile {tile} x{sp}: {tt:8.1f} us")
        old_extra = dict(extra)
        res.append(gd._time(lambda: K.gemm(A, B, C, **kw, **old_extra), reps=20))
        a = A.t() if mode & 1 else A
        b = B if mode & 2 else B.t()
        res.append(gd._time(lambda: torch.mm(a, b), reps=20))
        best = min(r for r in res if r == r)
        tf = 2 * M * N * Kd / best / 1e6
        print(f"{name:18s} {M:5d} {N:5d} {Kd:5d}  " + "  ".join(f"{r:8.1f}" for r in res) + f"   {tf:8.0f}")


if __name__ == "__main__":
    run()
