"""Llama-3-8B GEMMs at B x S = 16 x 512: the repo's LDS-DMA MFMA kernel (every tile the dispatcher offers) against
hipBLASLt, per shape, through the dispatcher's own measurement (``gemm_dispatch.gemm(..., _decide_only=True)``,
graph-timed, isolated).  VERDICT r2 item 7: "run its GEMMs through the repo's own kernels or state why hipBLASLt
wins per shape, using the dispatcher table".

    IIT_GEMM_TABLE=0 python scripts/llama_gemm_study.py
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

PEAK_TFLOPS = 2500.0  # MI355X dense bf16


def main():
    from iit_amd.ops import gemm_dispatch as gd
    from iit_amd.ops import hip_kernels as K
    dev = "cuda"
    T, d, dkv, dm = 16 * 512, 4096, 1024, 14336
    bf = torch.bfloat16
    # (name, M, N, K, mode, epi): mode 2 = forward x @ W (TL [d_in, d_out] weights), 0 = dX = dY W^T,
    # 3 = dW = X^T dY (fp32 accumulate into the gradient)
    probs = [
        ("fwd qkv", T, d + 2 * dkv, d, K.MODE_BKM, K.EPI_BF16),
        ("fwd o", T, d, d, K.MODE_BKM, K.EPI_BF16),
        ("fwd gate/up", T, dm, d, K.MODE_BKM, K.EPI_BF16),
        ("fwd down", T, d, dm, K.MODE_BKM, K.EPI_BF16),
        ("dX qkv", T, d, d + 2 * dkv, 0, K.EPI_BF16),
        ("dX gate/up", T, d, dm, 0, K.EPI_BF16),
        ("dX down", T, dm, d, 0, K.EPI_BF16),
        ("dW qkv", d, d + 2 * dkv, T, K.MODE_AKM | K.MODE_BKM, K.EPI_F32_ACC),
        ("dW gate/up", d, dm, T, K.MODE_AKM | K.MODE_BKM, K.EPI_F32_ACC),
        ("dW down", dm, d, T, K.MODE_AKM | K.MODE_BKM, K.EPI_F32_ACC),
    ]
    rows = []
    for name, M, N, Kd, mode, epi in probs:
        torch.manual_seed(0)
        akm = bool(mode & K.MODE_AKM)
        bkm = bool(mode & K.MODE_BKM)
        A = (torch.randn(Kd, M, device=dev) if akm else torch.randn(M, Kd, device=dev)).to(bf) / 8
        B = (torch.randn(Kd, N, device=dev) if bkm else torch.randn(N, Kd, device=dev)).to(bf) / 8
        C = torch.zeros(M, N, device=dev, dtype=torch.float32 if epi == K.EPI_F32_ACC else bf)
        lda = M if akm else Kd
        ldb = N if bkm else Kd
        gd.gemm(A, B, C, M=M, N=N, K=Kd, lda=lda, ldb=ldb, ldc=N, mode=mode, epi=epi, _decide_only=True)
        key = next(k for k in gd.DECISIONS if k[:5] == (M, N, Kd, mode, epi))
        best, times = gd.DECISIONS[key]
        flop = 2.0 * M * N * Kd
        glds = {k: v for k, v in times.items() if k.startswith("glds") or k == "hip"}
        gbest = min(glds, key=glds.get) if glds else None
        blas = times.get("blas")
        row = {"gemm": name, "M": M, "N": N, "K": Kd, "winner": best,
               "blas_us": round(blas, 1) if blas else None,
               "blas_tflops": round(flop / blas / 1e6, 0) if blas else None,
               "own_best": gbest, "own_us": round(glds[gbest], 1) if gbest else None,
               "own_tflops": round(flop / glds[gbest] / 1e6, 0) if gbest else None}
        row["blas_pct_peak"] = round(100 * row["blas_tflops"] / PEAK_TFLOPS, 1) if blas else None
        row["own_pct_peak"] = round(100 * row["own_tflops"] / PEAK_TFLOPS, 1) if gbest else None
        rows.append(row)
        print(json.dumps(row), flush=True)
        del A, B, C
        torch.cuda.empty_cache()
    print(json.dumps({"llama3_8b_gemm_study": rows}))


if __name__ == "__main__":
    main()
