"""A handful of the headline step's GEMMs on their dispatcher-chosen LDS-DMA tiles (5 calls each, no graphs) for
hardware-counter passes: ``rocprofv3 --pmc ... -- python3 scripts/pmc_gemm.py`` (scripts/gpu_pmc.sh)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from iit_amd.ops import hip_kernels as K  # noqa: E402

T = 4096
CASES = [  # name, M, N, K, mode, epi, tile[, splits, reduce]
    ("W_in fwd+gelu", T, 3072, 768, 2, K.EPI_GELU, 5),
    ("qkv fwd", T, 2304, 768, 2, K.EPI_BF16_BIAS3, 5),
    ("dX W_out + dgelu", T, 3072, 768, 0, K.EPI_DGELU, 5),
    ("dW W_in (X^T dY)", 768, 3072, T, 3, K.EPI_F32_STORE, 8),
    # the deterministic reduction split-K the dispatcher now picks for the weight gradients
    ("dW W_in 96x192 r2", 768, 3072, T, 3, K.EPI_F32_STORE, 10, 2, True),
    ("dW W_O 64x64 r2", 768, 768, T, 3, K.EPI_F32_STORE, 3, 2, True),
]


def main():
    dev = "cuda"
    for name, M, N, Kd, mode, epi, tile, *sk in CASES:
        splits, reduce = (sk + [1, False])[:2] if sk else (1, False)
        A = (torch.randn(Kd, M) if mode & 1 else torch.randn(M, Kd)).to(dev).bfloat16()
        B = (torch.randn(Kd, N) if mode & 2 else torch.randn(N, Kd)).to(dev).bfloat16() / 16
        lda = M if mode & 1 else Kd
        ldb = N if mode & 2 else Kd
        f32 = epi in (K.EPI_F32_STORE, K.EPI_F32_ACC)
        C = torch.zeros(M, N, device=dev, dtype=torch.float32 if f32 else torch.bfloat16)
        C2 = torch.randn(M, N, device=dev).bfloat16() if epi in (K.EPI_GELU, K.EPI_DGELU) else None
        bias = torch.randn(N, device=dev)
        extra = {}
        if epi == K.EPI_BF16_BIAS3:
            extra = dict(bias0=bias[:N // 3], bias1=bias[N // 3:2 * N // 3], bias2=bias[2 * N // 3:], bias_cols=N // 3)
        elif epi == K.EPI_GELU:
            extra = dict(bias0=bias)
        for _ in range(5):
            K.gemm_glds(A, B, C, M=M, N=N, K=Kd, lda=lda, ldb=ldb, ldc=N, mode=mode, epi=epi, C2=C2,
                        ldc2=N if C2 is not None else 0, tile=tile, splits=splits, reduce=reduce, **extra)
        torch.cuda.synchronize()
        print(name, "ok", flush=True)


if __name__ == "__main__":
    main()
