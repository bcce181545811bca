import ctypes, sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from iit_amd.ops import hip_kernels as K
L = K.lib()
L.iit_probe_tr16b.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
out = torch.zeros(256, dtype=torch.int16, device="cuda")
L.iit_probe_tr16b(out.data_ptr(), torch.cuda.current_stream().cuda_stream)
torch.cuda.synchronize()
o = out.view(64, 4).cpu()
for l in [0, 1, 5, 15, 16, 17, 31, 32, 47, 48, 63]:
    print("lane", l, o[l].tolist())
bf = lambda x: x.to(torch.bfloat16)
# structured: out[m][n] = sum_t X[t][m] G[t][n]; X = I (T=M=64)  -> out = G
T = M = N = 64
X = torch.eye(64, device="cuda")
G = torch.arange(64 * 64, device="cuda", dtype=torch.float32).view(64, 64) % 251
out = torch.zeros(M, N, device="cuda")
K.gemm(bf(X), bf(G), out, M=M, N=N, K=T, lda=M, ldb=N, ldc=N, mode=K.MODE_AKM | K.MODE_BKM, epi=K.EPI_F32_ACC, splits=1)
ref = bf(G).float()
bad = (out != ref).nonzero()
print("mismatches", bad.shape[0])
for r, c in bad[:20].tolist():
    v = out[r, c].item()
    loc = (ref == v).nonzero()[:3].tolist()
    print((r, c), "got", v, "want", ref[r, c].item(), "value lives at", loc)
outa = torch.zeros(M, N, device="cuda")
K.gemm(bf(X), bf(G.T.contiguous()), outa, M=M, N=N, K=T, lda=M, ldb=T, ldc=N, mode=K.MODE_AKM, epi=K.EPI_F32_ACC, splits=1)
print("A-only mismatches", (outa != ref).sum().item())
outb = torch.zeros(M, N, device="cuda")
K.gemm(bf(X.T.contiguous()), bf(G), outb, M=M, N=N, K=T, lda=T, ldb=N, ldc=N, mode=K.MODE_BKM, epi=K.EPI_F32_ACC, splits=1)
print("B-only mismatches", (outb != ref).sum().item())
bad = (outb != ref).nonzero()
for r, c in bad[:10].tolist():
    v = outb[r, c].item()
    print("B", (r, c), "got", v, "want", ref[r, c].item(), "lives at", (ref == v).nonzero()[:2].tolist())
