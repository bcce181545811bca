"""The headline step's GEMM shapes (IOI GPT-2-small, B = 256 pairs x 16 tokens: 8192-row paired forwards, 4096-row
backwards) in isolation: the dispatcher's shipped choice, every LDS-DMA tile that covers the shape (``--all``), the
256 x 256 four-wave kernel (tile 41), the persistent stream-K kernel (``sk``) and hipBLASLt -- graph-timed on uniform
random operands, the minimum over interleaved rounds in one process (cdna_hip_programming.md §5.4 rules 24-25).

    python scripts/bench_headline_gemms.py [--all] [--rounds 3] [--only NAME]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

PEAK_TFLOPS = 2500.0


def problems():
    from iit_amd.ops import hip_kernels as K
    T2, T, d, dm, d3 = 8192, 4096, 768, 3072, 2304
    B2, MD = K.MODE_BKM, K.MODE_AKM | K.MODE_BKM
    return [
        # name, M, N, K, mode, epi
        ("fwd qkv", T2, d3, d, B2, K.EPI_BF16_BIAS3),
        ("fwd o+res", T2, d, d, B2, K.EPI_F32_RESID),
        ("fwd mlp-in gelu", T2, dm, d, B2, K.EPI_GELU),
        ("fwd mlp-out+res", T2, d, dm, B2, K.EPI_F32_RESID),
        ("dX mlp-out dgelu", T, dm, d, 0, K.EPI_DGELU),
        ("dX mlp-in", T, d, dm, 0, K.EPI_BF16),
        ("dX qkv", T, d, d3, 0, K.EPI_BF16),
        ("dX o", T, d, d, 0, K.EPI_BF16),
        ("dW mlp-out", dm, d, T, MD, K.EPI_F32_STORE),
        ("dW mlp-in", d, dm, T, MD, K.EPI_F32_STORE),
        ("dW qkv", d, d3, T, MD, K.EPI_F32_STORE),
        ("dW o", d, d, T, MD, K.EPI_F32_STORE),
    ]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--all", action="store_true", help="time every LDS-DMA tile that covers each shape")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--only", default="")
    args = ap.parse_args()
    from iit_amd.ops import gemm_dispatch as gd
    from iit_amd.ops import hip_kernels as K
    dev = "cuda"
    bf, f32 = torch.bfloat16, torch.float32
    rows = []
    for name, M, N, Kd, mode, epi in problems():
        if args.only and args.only not in name:
            continue
        torch.manual_seed(0)
        akm, bkm = bool(mode & K.MODE_AKM), bool(mode & K.MODE_BKM)
        A = ((torch.rand(Kd, M, device=dev) if akm else torch.rand(M, Kd, device=dev)) * 2 - 1).to(bf)
        B = ((torch.rand(Kd, N, device=dev) if bkm else torch.rand(N, Kd, device=dev)) * 2 - 1).to(bf)
        f32_out = epi in (K.EPI_F32_RESID, K.EPI_F32_STORE, K.EPI_F32_ACC)
        C = torch.zeros(M, N, device=dev, dtype=f32 if f32_out else bf)
        C2 = (torch.rand(M, N, device=dev) * 2 - 1).to(bf) if epi in (K.EPI_GELU, K.EPI_DGELU) else None
        resid = torch.rand(M, N, device=dev) if epi == K.EPI_F32_RESID else None
        bias = torch.rand(N, device=dev) if epi in (K.EPI_GELU, K.EPI_F32_RESID) else None
        b3 = [torch.rand(N // 3, device=dev) for _ in range(3)] if epi == K.EPI_BF16_BIAS3 else [None] * 3
        lda = M if akm else Kd
        ldb = N if bkm else Kd
        kw = dict(M=M, N=N, K=Kd, lda=lda, ldb=ldb, ldc=N, mode=mode, epi=epi)
        ekw = dict(C2=C2, ldc2=N if C2 is not None else 0, resid=resid, ldr=N if resid is not None else 0)
        if epi == K.EPI_BF16_BIAS3:
            ekw.update(bias0=b3[0], bias1=b3[1], bias2=b3[2], bias_cols=N // 3)
        elif bias is not None:
            ekw.update(bias0=bias)
        cands = {}

        def disp():
            gd.gemm(A, B, C, aux=C2 if epi == K.EPI_DGELU else None, **{k: v for k, v in ekw.items()
                                                                         if not (epi == K.EPI_DGELU and k == "C2")},
                    **kw)
        cands["dispatch"] = disp
        tiles = list(K.GLDS_DISPATCH_TILES) if args.all else [41]
        for t in tiles:
            if K.gemm_glds_ok(A, B, C, tile=t, **kw, **{k: v for k, v in ekw.items()
                                                         if k in ("C2", "resid", "ldc2", "ldr", "bias_cols")}):
                cands[f"glds{t}"] = lambda t=t: K.gemm_glds(A, B, C, tile=t, **kw, **ekw)
        if hasattr(K, "gemm_sk") and K.gemm_sk_ok(A, B, C, **kw, **{k: v for k, v in ekw.items()
                                                                     if k in ("C2", "resid", "ldc2", "ldr",
                                                                              "bias_cols")}):
            cands["sk"] = lambda: K.gemm_sk(A, B, C, **kw, **ekw)
        a = A.t() if akm else A
        b = B if bkm else B.t()
        if f32_out:
            cands["blas"] = lambda: torch.mm(a, b, out_dtype=f32, out=C)
        else:
            cands["blas"] = lambda: torch.mm(a, b, out=C)
        disp()  # decide (shipped table or in-process timing) before the timed rounds
        times = {k: float("inf") for k in cands}
        for _ in range(args.rounds):
            for k, f in cands.items():
                times[k] = min(times[k], gd._time(f, reps=20))
        flop = 2.0 * M * N * Kd
        choice = None
        for key, (c, _t) in gd.DECISIONS.items():
            if key[:5] == (M, N, Kd, mode, epi):
                choice = c
        best = min(times, key=times.get)
        row = {"gemm": name, "M": M, "N": N, "K": Kd, "dispatch_choice": choice,
               "us": {k: round(v, 1) for k, v in sorted(times.items(), key=lambda kv: kv[1])},
               "best": best, "best_pct_peak": round(100 * flop / times[best] / 1e6 / PEAK_TFLOPS, 1),
               "dispatch_pct_peak": round(100 * flop / times["dispatch"] / 1e6 / PEAK_TFLOPS, 1)}
        rows.append(row)
        print(json.dumps(row), flush=True)
        del A, B, C, C2, resid
        torch.cuda.empty_cache()
    tot_d = sum(r["us"]["dispatch"] for r in rows)
    tot_b = sum(min(r["us"].values()) for r in rows)
    print(f"sum dispatch {tot_d:.1f} us, sum best {tot_b:.1f} us")


if __name__ == "__main__":
    main()
