"""The packed-QKV forward GEMM ([T][768] x [768][2304] + packed bias, bf16 out) at the headline step's two row counts
(T = 8192 paired source+base, 4096 base only): every LDS-DMA tile that covers it vs hipBLASLt, graph-timed, with a
max-error check of each against an fp32 torch reference.  One line per (T, candidate)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from iit_amd.ops import gemm_dispatch as gd  # noqa: E402
from iit_amd.ops import hip_kernels as K  # noqa: E402


def main():
    dev = "cuda"
    d, N = 768, 2304
    for T in (8192, 4096):
        torch.manual_seed(0)
        A = torch.randn(T, d, device=dev).bfloat16()
        B = (torch.randn(d, N, device=dev) / 16).bfloat16()
        bias = torch.randn(N, device=dev)
        b3 = [bias[i * 768:(i + 1) * 768] for i in range(3)]
        C = torch.empty(T, N, device=dev, dtype=torch.bfloat16)
        ref = A.float() @ B.float() + bias
        kw = dict(M=T, N=N, K=d, lda=d, ldb=N, ldc=N, mode=K.MODE_BKM, epi=K.EPI_BF16_BIAS3)
        extra = dict(bias0=b3[0], bias1=b3[1], bias2=b3[2], bias_cols=768)
        flops = 2.0 * T * N * d
        rows = []
        for tile in K.GLDS_TILES:
            if not K.gemm_glds_ok(A, B, C, bias_cols=768, tile=tile, **kw):
                continue
            fn = lambda t=tile: K.gemm_glds(A, B, C, tile=t, **kw, **extra)  # noqa: E731
            C.zero_()
            fn()
            err = float((C.float() - ref).abs().max())
            us = gd._time(fn, reps=20)
            rows.append((us, f"glds{tile} {K.GLDS_TILES[tile]}", err))
        bb = torch.cat(b3).bfloat16()
        fn = lambda: gd._blas(A, B, C, T, N, d, d, N, N, K.MODE_BKM, K.EPI_BF16_BIAS3, None, None, b3[0], b3[1],  # noqa
                              b3[2], None, 0, None, 0, 768, (0, 0, 0), bb)
        try:
            C.zero_()
            fn()
            err = float((C.float() - ref).abs().max())
            rows.append((gd._time(fn, reps=20), "blas", err))
        except Exception as e:  # noqa: BLE001
            print("blas failed", e)
        for us, name, err in sorted(rows):
            print(f"T={T:5d} {name:22s} {us:8.1f} us  {flops / us / 1e6:7.1f} TF/s  max|err| {err:.3g}", flush=True)


if __name__ == "__main__":
    main()
