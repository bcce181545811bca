"""The 256 x 256 8-phase GEMM (csrc/gemm_8ph.hip, tile 40) against hipBLASLt and the best other LDS-DMA tile on
square shapes and the Llama-3-8B training GEMMs (B x S = 16 x 512 -> 8192 tokens), graph-timed in isolation on
uniform random operands (cdna_hip_programming.md §5.4 rule 25: never zero-filled).  Every time is the minimum over
interleaved rounds in one process (rule 24).

    python scripts/bench_gemm_8ph.py [--quick] [--others]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

PEAK_TFLOPS = 2500.0  # MI355X dense bf16


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--quick", action="store_true", help="square shapes only")
    ap.add_argument("--others", action="store_true", help="also time every other LDS-DMA tile (slow)")
    ap.add_argument("--rounds", type=int, default=3)
    args = ap.parse_args()
    from iit_amd.ops import gemm_dispatch as gd
    from iit_amd.ops import hip_kernels as K
    dev = "cuda"
    bf = torch.bfloat16
    import ctypes
    lib = K.lib()
    lib.iit_gemm_8ph_set_diag.argtypes = [ctypes.c_int]
    T, d, dkv, dm = 16 * 512, 4096, 1024, 14336
    probs = [("sq4096 fwd", 4096, 4096, 4096, K.MODE_BKM, K.EPI_BF16),
             ("sq8192 fwd", 8192, 8192, 8192, K.MODE_BKM, K.EPI_BF16),
             ("sq8192 dX", 8192, 8192, 8192, 0, K.EPI_BF16)]
    if not args.quick:
        probs += [
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
        akm, bkm = bool(mode & K.MODE_AKM), bool(mode & K.MODE_BKM)
        A = ((torch.rand(Kd, M, device=dev) if akm else torch.rand(M, Kd, device=dev)) * 2 - 1).to(bf)
        B = ((torch.rand(Kd, N, device=dev) if bkm else torch.rand(N, Kd, device=dev)) * 2 - 1).to(bf)
        C = torch.zeros(M, N, device=dev, dtype=torch.float32 if epi == K.EPI_F32_ACC else bf)
        lda = M if akm else Kd
        ldb = N if bkm else Kd
        a = A.t() if akm else A
        b = B if bkm else B.t()
        cands = {}
        kw = dict(M=M, N=N, K=Kd, lda=lda, ldb=ldb, ldc=N, mode=mode, epi=epi)
        tiles = [40] + ([t for t in K.GLDS_DISPATCH_TILES if t != 40] if args.others else [5, 7, 25, 27])
        for t in tiles:
            if K.gemm_glds_ok(A, B, C, tile=t, **kw):
                cands[f"glds{t}"] = lambda t=t: K.gemm_glds(A, B, C, tile=t, **kw)

        def one_phase():  # tile 40 with the two-B-register K-loop schedule (S = 1, diag 8) -- A/B in this process
            lib.iit_gemm_8ph_set_diag(8)
            K.gemm_glds(A, B, C, tile=40, **kw)
            lib.iit_gemm_8ph_set_diag(0)
        cands["glds40s0"] = one_phase
        for t in (41, 42):
            if K.gemm_glds_ok(A, B, C, tile=t, **kw):
                cands[f"glds{t}"] = lambda t=t: K.gemm_glds(A, B, C, tile=t, **kw)
        if epi == K.EPI_F32_ACC:
            cands["blas"] = lambda: torch.addmm(C, a, b, out_dtype=torch.float32, out=C)
        else:
            cands["blas"] = lambda: torch.mm(a, b, out=C)
        # correctness of tile 40 on this shape against hipBLASLt (bf16 outputs: relative Frobenius error)
        C.zero_()
        cands["glds42"]()
        got = C.float().clone()
        C.zero_()
        cands["blas"]()
        ref = C.float().clone()
        rel = ((got - ref).norm() / ref.norm()).item()
        times = {k: float("inf") for k in cands}
        for _ in range(args.rounds):
            for k, f in cands.items():
                times[k] = min(times[k], gd._time(f, reps=10))
        flop = 2.0 * M * N * Kd
        own = {k: v for k, v in times.items() if k not in ("glds40", "glds40s0", "glds41", "glds42", "blas")}
        best_other = min(own, key=own.get) if own else None
        row = {"gemm": name, "M": M, "N": N, "K": Kd, "rel_err_vs_blas": round(rel, 5),
               "t40_us": round(times["glds40"], 1), "t40_pct": round(100 * flop / times["glds40"] / 1e6 / PEAK_TFLOPS, 1),
               "t40s0_us": round(times["glds40s0"], 1),
               "t41_us": round(times["glds41"], 1), "t41_pct": round(100 * flop / times["glds41"] / 1e6 / PEAK_TFLOPS, 1),
               "t42_us": round(times["glds42"], 1), "t42_pct": round(100 * flop / times["glds42"] / 1e6 / PEAK_TFLOPS, 1),
               "t40s0_pct": round(100 * flop / times["glds40s0"] / 1e6 / PEAK_TFLOPS, 1),
               "blas_us": round(times["blas"], 1), "blas_pct": round(100 * flop / times["blas"] / 1e6 / PEAK_TFLOPS, 1),
               "other": best_other, "other_us": round(own[best_other], 1) if best_other else None,
               "other_pct": round(100 * flop / own[best_other] / 1e6 / PEAK_TFLOPS, 1) if best_other else None}
        rows.append(row)
        print(json.dumps(row), flush=True)
        del A, B, C, a, b, got, ref
        torch.cuda.empty_cache()
    print("%-12s %6s %6s %6s %8s %5s %8s %5s %8s %5s %8s %5s %8s %5s %7s %8s %5s" % (
        "gemm", "M", "N", "K", "4w32 us", "%pk", "4w64 us", "%pk", "8ph us", "%pk", "8phS1", "%pk", "blas us", "%pk",
        "other", "us", "%pk"))
    for r in rows:
        print("%-12s %6d %6d %6d %8.1f %5.1f %8.1f %5.1f %8.1f %5.1f %8.1f %5.1f %8.1f %5.1f %7s %8s %5s" % (
            r["gemm"], r["M"], r["N"], r["K"], r["t42_us"], r["t42_pct"], r["t41_us"], r["t41_pct"], r["t40_us"],
            r["t40_pct"], r["t40s0_us"], r["t40s0_pct"], r["blas_us"], r["blas_pct"], r["other"], r["other_us"],
            r["other_pct"]))


if __name__ == "__main__":
    main()
