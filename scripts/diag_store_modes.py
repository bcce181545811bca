"""Does a GEMM's output store flavour change what the NEXT kernel pays at the boundary?

Chains of two dependent GEMMs from the step -- MLP-in (bias + gelu_new: writes pre and post, 2 x 25 MB) followed by
MLP-out (+ fp32 residual, reads post) and QKV (writes 19 MB) followed by its consumer shape -- are graph-timed with the
producer's epilogue stores plain, non-temporal, or write-through (sc1), against each GEMM alone."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from iit_amd.ops import gemm_dispatch as gd
    from iit_amd.ops import hip_kernels as K
    dev = "cuda"
    torch.manual_seed(0)
    T, d, dm = 4096, 768, 3072
    bf = torch.bfloat16
    x = torch.randn(T, d, device=dev, dtype=bf)
    W_in = (torch.randn(d, dm, device=dev) / 30).to(bf)
    b_in = torch.zeros(dm, device=dev)
    W_out = (torch.randn(dm, d, device=dev) / 60).to(bf)
    b_out = torch.zeros(d, device=dev)
    pre = torch.empty(T, dm, device=dev, dtype=bf)
    post = torch.empty(T, dm, device=dev, dtype=bf)
    resid = torch.randn(T, d, device=dev)
    out = torch.empty(T, d, device=dev)

    def mlp_in(sm):
        K.gemm_glds(x, W_in, post, M=T, N=dm, K=d, lda=d, ldb=dm, ldc=dm, mode=2, epi=K.EPI_GELU, C2=pre, ldc2=dm,
                    bias0=b_in, tile=5, store_mode=sm)

    def mlp_out(sm):
        K.gemm_glds(post, W_out, out, M=T, N=d, K=dm, lda=dm, ldb=d, ldc=d, mode=2, epi=K.EPI_F32_RESID,
                    bias0=b_out, resid=resid, ldr=d, tile=9, store_mode=sm)

    def time_it(fn, reps=20):
        return min(gd._time(fn, reps=reps) for _ in range(3))

    for sm in (0, 1, 2):
        a = time_it(lambda: mlp_in(sm))
        b = time_it(lambda: mlp_out(0))
        ab = time_it(lambda: (mlp_in(sm), mlp_out(0)))
        print(f"store {sm}: mlp_in {a:6.1f} us  mlp_out {b:6.1f} us  chain {ab:6.1f} us  (chain - parts {ab - a - b:+5.1f})",
              flush=True)
    for sm in (0, 1, 2):
        b = time_it(lambda: mlp_out(sm))
        ab = time_it(lambda: (mlp_out(sm), mlp_in(0)))
        a = time_it(lambda: mlp_in(0))
        print(f"resid store {sm}: mlp_out {b:6.1f} us  then mlp_in: chain {ab:6.1f} us  (chain - parts {ab - a - b:+5.1f})",
              flush=True)


if __name__ == "__main__":
    main()
