"""MLP backward dpre GEMM variants on the GPT-2-small step shape (M=4096 tokens, N=3072, K=768, mode 0):
plain bf16 GEMM + dgelu + column-sum passes vs the fused DGELU epilogue (with / without fused column sums)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from iit_amd.ops import gemm_dispatch as gd  # noqa: E402
from iit_amd.ops import hip_kernels as K  # noqa: E402


def main():
    M, N, Kd = 4096, 3072, 768
    dev = "cuda"
    A = torch.randn(M, Kd, device=dev).bfloat16()
    B = (torch.randn(N, Kd, device=dev) / 16).bfloat16()
    pre = torch.randn(M, N, device=dev).bfloat16()
    C = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    T = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    cs = torch.zeros(N, device=dev)
    kw = dict(M=M, N=N, K=Kd, lda=Kd, ldb=Kd, ldc=N, mode=0)
    rows = []
    for tile in (0, 5, 6, 7):
        if not K.gemm_glds_ok(A, B, C, epi=K.EPI_BF16, tile=tile, **kw):
            continue
        plain = gd._time(lambda t=tile: K.gemm_glds(A, B, T, epi=K.EPI_BF16, tile=t, **kw), reps=20)
        unf = gd._time(lambda t=tile: (K.gemm_glds(A, B, T, epi=K.EPI_BF16, tile=t, **kw), K.dgelu(T, pre, C),
                                       K.colsum_accum(C, N, cs, M, N)), reps=20)
        dg = gd._time(lambda t=tile: K.gemm_glds(A, B, C, epi=K.EPI_DGELU, C2=pre, ldc2=N, tile=t, **kw), reps=20)
        dgc = gd._time(lambda t=tile: K.gemm_glds(A, B, C, epi=K.EPI_DGELU, C2=pre, ldc2=N, tile=t, csum=cs, **kw),
                       reps=20)
        rows.append(f"glds tile {tile}: gemm {plain:6.1f}  gemm+dgelu+colsum {unf:6.1f}  fused dgelu {dg:6.1f}  "
                    f"fused dgelu+colsum {dgc:6.1f} us")
    hip = gd._time(lambda: K.gemm(A, B, C, epi=K.EPI_DGELU, aux=pre, ldc2=N, **kw), reps=20)
    dgelu = gd._time(lambda: K.dgelu(T, pre, C), reps=20)
    col = gd._time(lambda: K.colsum_accum(C, N, cs, M, N), reps=20)
    rows.append(f"hip DGELU {hip:6.1f} us; dgelu pass {dgelu:6.1f} us; colsum pass {col:6.1f} us")
    print("\n".join(rows))


if __name__ == "__main__":
    main()
