"""Stress the atomic split-K GEMM paths on the shapes the poison probe flagged (scripts/diag_uninit_poison.py: excluding
the ``s+hip`` candidate -- init C with bias / residual / zeros, then ``iit_gemm`` EPI_F32_ACC with split-K atomics --
made every configuration bit-stable).  Each case runs many times on fresh random operands against an fp32 reference
and reports the worst error and how many runs were off; variants: the s+hip candidate as the dispatcher builds it,
the raw ``iit_gemm`` split accumulate into a zeroed C, the same with a device sync between init and GEMM, and the
LDS-DMA kernel's atomic split-K tile.  Prints ``[split]`` lines."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

from iit_amd.ops import gemm_dispatch as D  # noqa: E402
from iit_amd.ops import hip_kernels as K  # noqa: E402

dev = "cuda"


def ref_mm(A, B, M, N, Kd, mode):
    a = A.float().view(Kd, M).t() if mode & K.MODE_AKM else A.float().view(M, Kd)
    b = B.float().view(Kd, N) if mode & K.MODE_BKM else B.float().view(N, Kd).t()
    return a @ b


def operands(M, N, Kd, mode, g):
    A = torch.randn((Kd, M) if mode & K.MODE_AKM else (M, Kd), device=dev, generator=g).bfloat16()
    B = torch.randn((Kd, N) if mode & K.MODE_BKM else (N, Kd), device=dev, generator=g).bfloat16()
    lda = M if mode & K.MODE_AKM else Kd
    ldb = N if mode & K.MODE_BKM else Kd
    return A, B, lda, ldb


def main():
    g = torch.Generator(device=dev).manual_seed(0)
    # (M, N, K, mode, epi): final-block last-position W_out residual, weight-gradient stores of the 4-layer test model
    cases = [(32, 128, 512, 0, K.EPI_F32_RESID), (128, 512, 512, 3, K.EPI_F32_STORE), (512, 128, 512, 3, K.EPI_F32_STORE),
             (128, 384, 512, 3, K.EPI_F32_STORE), (128, 128, 512, 3, K.EPI_F32_STORE), (256, 768, 3072, 0, K.EPI_F32_RESID),
             (768, 768, 256, 3, K.EPI_F32_STORE)]
    runs = int(os.environ.get("RUNS", "60"))
    for M, N, Kd, mode, epi in cases:
        sp = min(16, Kd // 64)
        for variant in ("s+hip", "raw", "raw+sync", "glds-k"):
            worst, bad = 0.0, 0
            for _ in range(runs):
                A, B, lda, ldb = operands(M, N, Kd, mode, g)
                resid = torch.randn(M, N, device=dev, generator=g) if epi == K.EPI_F32_RESID else None
                C = torch.full((M, N), float("nan"), device=dev)
                ref = ref_mm(A, B, M, N, Kd, mode) + (resid if resid is not None else 0)
                if variant == "s+hip":
                    calls = D._candidates_plain(A, B, C, None, M, N, Kd, lda, ldb, N, mode, epi, None, None, None,
                                                resid, N, None, 0, 0, (0, 0, 0), None, None, "auto", None)
                    if "s+hip" not in calls:
                        break
                    calls["s+hip"](C, None, None)
                elif variant.startswith("raw"):
                    C.copy_(resid) if resid is not None else C.zero_()
                    if variant == "raw+sync":
                        torch.cuda.synchronize()
                    K.gemm(A, B, C, M=M, N=N, K=Kd, lda=lda, ldb=ldb, ldc=N, mode=mode, epi=K.EPI_F32_ACC, splits=sp)
                else:
                    if epi != K.EPI_F32_STORE:
                        break
                    C.zero_()
                    tile = next((t for t in K.GLDS_DISPATCH_TILES if K.gemm_glds_ok(
                        A, B, C, M=M, N=N, K=Kd, lda=lda, ldb=ldb, ldc=N, mode=mode, epi=K.EPI_F32_ACC, tile=t,
                        splits=4)), None)
                    if tile is None:
                        break
                    K.gemm_glds(A, B, C, M=M, N=N, K=Kd, lda=lda, ldb=ldb, ldc=N, mode=mode, epi=K.EPI_F32_ACC,
                                tile=tile, splits=4)
                torch.cuda.synchronize()
                err = float(((C - ref).abs().max() / (ref.abs().max() + 1e-6)).nan_to_num(1e9))
                worst = max(worst, err)
                bad += err > 1e-2
            else:
                print(f"[split] M={M} N={N} K={Kd} mode={mode} epi={epi} {variant:9s} splits={sp}: worst rel err "
                      f"{worst:.3g}, {bad}/{runs} runs off", flush=True)


if __name__ == "__main__":
    main()
