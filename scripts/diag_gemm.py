"""Diagnostics for the GEMM k-major (transpose-read) path."""
import ctypes, sys, os, math
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from iit_amd.ops import hip_kernels as K
L = K.lib()
L.iit_probe_tr16.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
out = torch.zeros(64 * 4, dtype=torch.int16, device="cuda")
L.iit_probe_tr16(out.data_ptr(), torch.cuda.current_stream().cuda_stream)
torch.cuda.synchronize()
o = out.view(64, 4).cpu()
for l in range(0, 64):
    print(l, o[l].tolist())
bf = lambda x: x.to(torch.bfloat16)
for (M, N, T, splits) in [(64, 64, 64, 1), (64, 200, 96, 1), (768, 768, 4096, 1), (768, 768, 4096, 4), (256, 256, 128, 1)]:
    torch.manual_seed(1)
    X = torch.randn(T, M, device="cuda"); G = torch.randn(T, N, device="cuda")
    out = torch.zeros(M, N, device="cuda")
    K.gemm(bf(X), bf(G), out, M=M, N=N, K=T, lda=M, ldb=N, ldc=N, mode=K.MODE_AKM | K.MODE_BKM, epi=K.EPI_F32_ACC, splits=splits)
    ref = bf(X).float().T @ bf(G).float()
    err = ((out - ref).norm() / ref.norm()).item()
    # also A-kmajor only / B-kmajor only vs nn
    print("kmaj", M, N, T, splits, "rel", err)
    outa = torch.zeros(M, N, device="cuda")
    K.gemm(bf(X), bf(G.T.contiguous()), outa, M=M, N=N, K=T, lda=M, ldb=T, ldc=N, mode=K.MODE_AKM, epi=K.EPI_F32_ACC, splits=splits)
    print("  A-kmaj only rel", ((outa - ref).norm() / ref.norm()).item())
    outb = torch.zeros(M, N, device="cuda")
    K.gemm(bf(X.T.contiguous()), bf(G), outb, M=M, N=N, K=T, lda=T, ldb=N, ldc=N, mode=K.MODE_BKM, epi=K.EPI_F32_ACC, splits=splits)
    print("  B-kmaj only rel", ((outb - ref).norm() / ref.norm()).item())
