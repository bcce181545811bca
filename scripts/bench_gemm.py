"""GEMM microbenchmark on the GPT-2-small IIT step shapes: iit_amd MFMA kernel vs torch (hipBLASLt).

Interleaved rounds in one process (guide §5.4 rule 24), random operands (rule 25).
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from iit_amd.ops import hip_kernels as K

dev = "cuda"
T = 4096
d, dm, HD = 768, 3072, 768


def timeit(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record()
    for _ in range(reps):
        fn()
    ev1.record()
    torch.cuda.synchronize()
    return ev0.elapsed_time(ev1) / reps * 1000.0  # us


def case(name, M, N, Kd, mode, epi=K.EPI_BF16):
    torch.manual_seed(0)
    akm, bkm = bool(mode & K.MODE_AKM), bool(mode & K.MODE_BKM)
    A = (torch.randn(Kd, M, device=dev) if akm else torch.randn(M, Kd, device=dev)).to(torch.bfloat16)
    B = (torch.randn(Kd, N, device=dev) if bkm else torch.randn(N, Kd, device=dev)).to(torch.bfloat16)
    lda = M if akm else Kd
    ldb = N if bkm else Kd
    if epi in (K.EPI_F32_ACC, K.EPI_F32_STORE):
        C = torch.zeros(M, N, device=dev)
    else:
        C = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
    mine = lambda: K.gemm(A, B, C, M=M, N=N, K=Kd, lda=lda, ldb=ldb, ldc=N, mode=mode, epi=epi)  # noqa: E731
    At = A.t() if akm else A
    Bt = B if bkm else B.t()
    ref = lambda: torch.mm(At, Bt)  # noqa: E731
    t_m = min(timeit(mine) for _ in range(3))
    t_r = min(timeit(ref) for _ in range(3))
    fl = 2.0 * M * N * Kd
    print(f"{name:28s} M={M:5d} N={N:5d} K={Kd:5d} mode={mode:2d}  mine {t_m:8.1f}us {fl / t_m / 1e6:7.1f}TF   "
          f"torch {t_r:8.1f}us {fl / t_r / 1e6:7.1f}TF", flush=True)


if __name__ == "__main__":
    K.lib()
    for bkm in (0, K.MODE_BKM):
        case("qkv fwd", T, 3 * HD, d, bkm)
        case("o_proj fwd", T, d, HD, bkm)
        case("mlp_in fwd", T, dm, d, bkm)
        case("mlp_out fwd", T, d, dm, bkm)
        case("unembed last fwd", 256, 50257, d, bkm, K.EPI_F32_STORE)
    case("qkv dX", T, d, 3 * HD, 0)
    case("mlp_in dX", T, d, dm, 0)
    case("mlp_out dX", T, dm, d, 0)
    kk = K.MODE_AKM | K.MODE_BKM
    case("qkv dW", d, 3 * HD, T, kk, K.EPI_F32_ACC)
    case("o dW", HD, d, T, kk, K.EPI_F32_ACC)
    case("mlp_in dW", d, dm, T, kk, K.EPI_F32_ACC)
    case("mlp_out dW", dm, d, T, kk, K.EPI_F32_ACC)
    case("unembed dW", d, 50257, 256, kk, K.EPI_F32_ACC)
    case("square 4096", 4096, 4096, 4096, 0)
    case("square 4096 bkm", 4096, 4096, 4096, K.MODE_BKM)
