"""The library-GEMM side of ``iit_amd.ops.gemm_dispatch`` against fp32 references.

The dispatcher picks, per (shape, layout, epilogue), between the hand-written
MFMA kernel and hipBLASLt (``torch.mm``); both must implement the same operand
layouts and epilogues.  The library side is plain torch, so it is checked on CPU
here; the HIP side is checked by ``test_hip_kernels.py`` on the GPU.
"""
import torch

from iit_amd.ops import gemm_dispatch as gd
from iit_amd.ops import hip_kernels as K
from iit_amd.ops.torch_ops import gelu_new

BF = torch.bfloat16


def _ref_ops(A, B, M, N, Kd, mode):
    a = A.float().view(-1)
    b = B.float().view(-1)
    if mode & K.MODE_AKM:
        am = a[: Kd * M].view(Kd, M).t()
    else:
        am = a[: M * Kd].view(M, Kd)
    if mode & K.MODE_BKM:
        bm = b[: Kd * N].view(Kd, N)
    else:
        bm = b[: N * Kd].view(N, Kd).t()
    return am.to(BF).float() @ bm.to(BF).float()


def _call(A, B, C, M, N, Kd, mode, epi, **kw):
    defaults = dict(C2=None, C3=None, bias0=None, bias1=None, bias2=None, resid=None, ldr=0, aux=None, ldc2=0,
                    bias_cols=0, qkv=(0, 0, 0))
    defaults.update(kw)
    lda = M if mode & K.MODE_AKM else Kd
    ldb = N if mode & K.MODE_BKM else Kd
    gd._blas(A, B, C, M, N, Kd, lda, ldb, N, mode, epi, **{k: defaults[k] for k in
             ("C2", "C3", "bias0", "bias1", "bias2", "resid", "ldr", "aux", "ldc2", "bias_cols", "qkv")})


def test_blas_layouts_and_bias3():
    torch.manual_seed(0)
    M, H, dh, Kd = 24, 3, 8, 16
    N = 3 * H * dh
    for mode in (K.MODE_NN, K.MODE_BKM, K.MODE_AKM | K.MODE_BKM):
        A = torch.randn(M * Kd).to(BF)
        B = torch.randn(N * Kd).to(BF)
        bq, bk, bv = (torch.randn(H, dh) for _ in range(3))  # TL per-head bias shapes
        C = torch.empty(M, N, dtype=BF)
        _call(A, B, C, M, N, Kd, mode, K.EPI_BF16_BIAS3, bias0=bq, bias1=bk, bias2=bv, bias_cols=H * dh)
        ref = _ref_ops(A, B, M, N, Kd, mode) + torch.cat([bq.reshape(-1), bk.reshape(-1), bv.reshape(-1)])
        assert torch.allclose(C.float(), ref, atol=0.1, rtol=0.02), mode


def test_blas_residual_gelu_acc_store():
    torch.manual_seed(1)
    M, N, Kd = 20, 12, 32
    A = torch.randn(M, Kd).to(BF)
    B = torch.randn(N, Kd).to(BF)
    bias = torch.randn(N)
    base = _ref_ops(A, B, M, N, Kd, K.MODE_NN)
    R = torch.randn(M, N)
    C = torch.empty(M, N)
    _call(A, B, C, M, N, Kd, K.MODE_NN, K.EPI_F32_RESID, bias0=bias, resid=R, ldr=N)
    assert torch.allclose(C, R + base + bias, atol=0.05, rtol=0.02)
    post = torch.empty(M, N, dtype=BF)
    pre = torch.empty(M, N, dtype=BF)
    _call(A, B, post, M, N, Kd, K.MODE_NN, K.EPI_GELU, bias0=bias, C2=pre, ldc2=N)
    assert torch.allclose(pre.float(), base + bias, atol=0.1, rtol=0.02)
    assert torch.allclose(post.float(), gelu_new(pre.float()), atol=0.05, rtol=0.02)
    acc = torch.randn(M, N)
    exp = acc + base
    _call(A, B, acc, M, N, Kd, K.MODE_NN, K.EPI_F32_ACC)
    assert torch.allclose(acc, exp, atol=0.05, rtol=0.02)
    st = torch.empty(M, N)
    _call(A, B, st, M, N, Kd, K.MODE_NN, K.EPI_F32_STORE, bias0=bias)
    assert torch.allclose(st, base + bias, atol=0.05, rtol=0.02)


def test_gemm_entry_point_forced_blas_on_cpu(monkeypatch):
    """The public entry point (policy plumbing, candidate table) runs on CPU with the library path forced."""
    monkeypatch.setattr(gd, "POLICY", "blas")
    torch.manual_seed(2)
    M, N, Kd = 8, 12, 16
    A = torch.randn(M, Kd).to(BF)
    B = torch.randn(N, Kd).to(BF)
    C = torch.empty(M, N, dtype=BF)
    gd.gemm(A, B, C, M=M, N=N, K=Kd, lda=Kd, ldb=Kd, ldc=N, mode=K.MODE_NN, epi=K.EPI_BF16)
    assert torch.allclose(C.float(), A.float() @ B.float().T, atol=0.1, rtol=0.02)
    assert isinstance(gd.DECISIONS, dict) and "library fast paths" in gd.report()


def test_ragged_split_pieces_cover_the_problem():
    """_ragged_split: an N-ragged problem becomes a 128-aligned bulk + tail over disjoint columns (operand / output
    offsets per layout); a K-ragged accumulate becomes a 1024-aligned bulk + tail over disjoint reduction steps."""
    V, d, T = 50257, 768, 256
    A = torch.zeros(T, d, dtype=BF)
    B = torch.zeros(d, 50264, dtype=BF)
    C = torch.zeros(T, 50264)
    bias = torch.zeros(V)
    parts = gd._ragged_split(A, B, C, M=T, N=V, K=d, lda=d, ldb=50264, mode=K.MODE_BKM, epi=K.EPI_F32_STORE,
                             C2=None, bias0=bias, resid=None, aux=None)
    bulk, tail = parts
    assert bulk["N"] == 50176 and tail["N"] == V - 50176
    assert tail["B"].data_ptr() == B.data_ptr() + 50176 * 2  # k-major B: column offset
    assert tail["C"].data_ptr() == C.data_ptr() + 50176 * 4 and tail["bias0"].data_ptr() == bias.data_ptr() + 50176 * 4
    # K-ragged fp32 accumulate (the unembed input gradient, K = vocab)
    G = torch.zeros(T, 50264, dtype=BF)
    U = torch.zeros(d, 50264, dtype=BF)
    X = torch.zeros(T, d)
    bulk, tail = gd._ragged_split(G, U, X, M=T, N=d, K=V, lda=50264, ldb=50264, mode=K.MODE_NN, epi=K.EPI_F32_ACC,
                                  C2=None, bias0=None, resid=None, aux=None)
    assert bulk["K"] == 50176 and tail["K"] == V - 50176 and tail["C"] is X
    assert tail["A"].data_ptr() == G.data_ptr() + 50176 * 2 and tail["B"].data_ptr() == U.data_ptr() + 50176 * 2
    # aligned or small problems are left whole
    assert gd._ragged_split(A, B, C, M=T, N=4096, K=d, lda=d, ldb=50264, mode=K.MODE_BKM, epi=K.EPI_F32_STORE,
                            C2=None, bias0=None, resid=None, aux=None) is None


def test_dual_name_parsing_and_families():
    """Dual-launch candidate names round-trip to (dW tile, dX tile, splits, reduce); the tile families pair up."""
    assert gd._parse_dual("dual1.3") == (1, 3, 1, False)
    assert gd._parse_dual("dual0.3r2") == (0, 3, 2, True)
    assert gd._parse_dual("dual4.3k2") == (4, 3, 2, False)
    assert gd._parse_dual("serial") is None and gd._parse_dual("glds5") is None
    assert K.dual_family_ok(0, 3) and K.dual_family_ok(5, 4) and K.dual_family_ok(7, 8)
    assert not K.dual_family_ok(0, 4) and not K.dual_family_ok(5, 7) and not K.dual_family_ok(7, 0)


def test_gemm_pair_falls_back_to_serial_off_gpu(monkeypatch):
    """On the CPU (or for a pair the dual kernel does not cover) gemm_pair runs both GEMMs one after the other."""
    torch.manual_seed(0)
    xs0 = dict(A=torch.zeros(1), mode=0, epi=K.EPI_BF16)
    ws0 = dict(mode=K.MODE_AKM | K.MODE_BKM, epi=K.EPI_F32_STORE)
    assert not gd._dual_eligible(xs0, ws0)  # CPU tensors
    monkeypatch.setattr(gd, "POLICY", "blas")  # no device timing on the CPU
    T, kin, n = 32, 16, 24
    x = torch.randn(T, kin).bfloat16()
    dy = torch.randn(T, n).bfloat16()
    w = torch.randn(kin, n).bfloat16()
    dX = torch.empty(T, kin, dtype=torch.bfloat16)
    gW = torch.empty(kin, n)
    xs = dict(A=dy, B=w, C=dX, M=T, N=kin, K=n, lda=n, ldb=n, ldc=kin, epi=K.EPI_BF16)
    ws = dict(A=x, B=dy, C=gW, M=kin, N=n, K=T, lda=kin, ldb=n, ldc=n, mode=K.MODE_AKM | K.MODE_BKM,
              epi=K.EPI_F32_STORE, fresh=True)
    gd.gemm_pair(xs, ws)
    torch.testing.assert_close(gW, x.float().t() @ dy.float(), rtol=1e-2, atol=1e-2)
    torch.testing.assert_close(dX.float(), (dy.float() @ w.float().t()), rtol=2e-2, atol=5e-2)
