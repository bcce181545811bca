"""The 256 x 256 big-problem GEMMs against fp32 PyTorch -- the 8-phase 8-wave kernel (csrc/gemm_8ph.hip, LDS-DMA tile
40, both K-loop schedules) and the four-wave 32x32x16 kernel (csrc/gemm_4w.hip, tile 41): every layout x epilogue
they cover, K-loops of 1, 2, 3 and many K-tiles (the prologue / tail branches of the prefetch schedules), fused
column sums / sums of squares, and an exact small-integer race screen over a multi-tile grid."""
import pytest
import torch

from test_gemm_glds import CASES, _ops

pytestmark = pytest.mark.gpu
dev = "cuda"


@pytest.fixture(scope="module", params=[(40, 0), (40, 8), (41, 0), (42, 0)],
                ids=["8ph-onephase", "8ph-deep", "4w-bk64", "4w-bk32"])
def K(request):
    """Tile 40 with both K-loop schedules (the shipped one-phase S = 0 and S = 1, diag bit 8) and the four-wave
    kernel with 64- and 32-deep K-tiles (tiles 41 / 42)."""
    import ctypes
    from iit_amd.ops import hip_kernels
    lib = hip_kernels.lib()
    lib.iit_gemm_8ph_set_diag.argtypes = [ctypes.c_int]
    lib.iit_gemm_8ph_set_diag(request.param[1])
    global TILE
    TILE = request.param[0]
    yield hip_kernels
    lib.iit_gemm_8ph_set_diag(0)


TILE = 40

@pytest.mark.parametrize("kd", [64, 128, 192, 640])
@pytest.mark.parametrize("mode,epi", CASES)
def test_8ph_matches_fp32(K, mode, epi, kd):
    from iit_amd.ops.torch_ops import gelu_new
    M, N, pad = 512, 768, 8
    A, B, lda, ldb, a, b = _ops(K, mode, M, N, kd, pad)
    ref = a @ b
    ldc = N + 8
    bias = torch.randn(N, device=dev)
    kw = dict(M=M, N=N, K=kd, lda=lda, ldb=ldb, ldc=ldc, mode=mode, epi=epi, tile=TILE)
    if epi in (K.EPI_BF16, K.EPI_BF16_BIAS3, K.EPI_GELU, K.EPI_GELU_ERF):
        C = torch.zeros(M, ldc, device=dev, dtype=torch.bfloat16)
    else:
        C = torch.randn(M, ldc, device=dev)
    C0 = C.clone()
    extra = {}
    if epi == K.EPI_BF16:
        extra = dict(bias0=bias)
        exp = ref + bias
    elif epi == K.EPI_BF16_BIAS3:
        b3 = [torch.randn(N // 3, device=dev) for _ in range(3)]
        extra = dict(bias0=b3[0], bias1=b3[1], bias2=b3[2], bias_cols=N // 3)
        exp = ref + torch.cat(b3)
    elif epi == K.EPI_F32_RESID:
        R = torch.randn(M, N + 16, device=dev)
        extra = dict(bias0=bias, resid=R, ldr=N + 16)
        exp = ref + bias + R[:, :N]
    elif epi in (K.EPI_GELU, K.EPI_GELU_ERF):
        C2 = torch.zeros(M, ldc, device=dev, dtype=torch.bfloat16)
        extra = dict(bias0=bias, C2=C2, ldc2=ldc)
        exp = gelu_new(ref + bias) if epi == K.EPI_GELU else torch.nn.functional.gelu(ref + bias)
    elif epi == K.EPI_F32_ACC:
        exp = C0[:, :N] + ref
    else:
        extra = dict(bias0=bias) if mode != 3 else {}
        exp = ref + (bias if mode != 3 else 0)
    assert K.gemm_glds_ok(A, B, C, C2=extra.get("C2"), resid=extra.get("resid"), ldc2=extra.get("ldc2", 0),
                          ldr=extra.get("ldr", 0), bias_cols=extra.get("bias_cols", 0), **kw)
    K.gemm_glds(A, B, C, **kw, **extra)
    torch.cuda.synchronize()
    got = C[:, :N].float()
    err = ((got - exp).norm() / exp.norm()).item()
    assert err < 1e-2, err
    assert torch.equal(C[:, N:], C0[:, N:])  # padding columns untouched


def test_8ph_dgelu_colsum(K):
    from iit_amd.ops.torch_ops import gelu_new
    M, N, kd = 512, 512, 384
    A, B, lda, ldb, a, b = _ops(K, 0, M, N, kd, 0)
    pre = torch.randn(M, N, device=dev).bfloat16()
    C = torch.zeros(M, N, device=dev, dtype=torch.bfloat16)
    cs = torch.zeros(N, device=dev)
    x = pre.float().requires_grad_(True)
    gelu_new(x).backward(a @ b)
    K.gemm_glds(A, B, C, M=M, N=N, K=kd, lda=lda, ldb=ldb, ldc=N, mode=0, epi=K.EPI_DGELU, C2=pre, ldc2=N,
                tile=TILE, csum=cs)
    torch.cuda.synchronize()
    exp = x.grad
    assert ((C.float() - exp).norm() / exp.norm()).item() < 1e-2
    assert torch.allclose(cs, C.float().sum(0), rtol=2e-3, atol=2e-2)


@pytest.mark.parametrize("epi", [5, 7])
def test_8ph_weight_gradient_bsum_gsq(K, epi):
    """mode 3 (X^T dY) with the fused column sums of dY (the bias gradient) and, for stores, the sum of squares."""
    M, N, kd = 512, 768, 1024
    A, B, lda, ldb, a, b = _ops(K, 3, M, N, kd, 8)
    C = torch.randn(M, N, device=dev)
    exp = a @ b + (C if epi == K.EPI_F32_ACC else 0)
    bsum = torch.zeros(N, device=dev)
    gsq = torch.zeros(64, device=dev) if epi == K.EPI_F32_STORE else None
    K.gemm_glds(A, B, C, M=M, N=N, K=kd, lda=lda, ldb=ldb, ldc=N, mode=3, epi=epi, tile=TILE, bsum=bsum, gsq=gsq)
    torch.cuda.synchronize()
    assert ((C - exp).norm() / exp.norm()).item() < 1e-2
    assert torch.allclose(bsum, b.sum(0), rtol=1e-3, atol=1e-2)
    if gsq is not None:
        assert torch.allclose(gsq.sum(), (C * C).sum(), rtol=1e-3)


@pytest.mark.parametrize("mode", [0, 2, 3])
def test_8ph_exact_integer_race_screen(K, mode):
    """Small-integer operands (exact in bf16, sums exact in fp32): every element of a 16-tile grid must equal the
    reference exactly, over repeated launches -- an early LDS read (RAW) or an early restage (WAR) of the prefetch
    schedule would show up as wrong tiles."""
    M, N, kd = 1024, 1024, 2048
    g = torch.Generator(device=dev).manual_seed(mode)
    a = torch.randint(-3, 4, (M, kd), device=dev, generator=g).float()
    b = torch.randint(-2, 3, (kd, N), device=dev, generator=g).float()
    b[:, ::7] *= 0.5  # asymmetric columns
    A = (a.t().contiguous() if mode == 3 else a).bfloat16()
    B = (b if mode in (2, 3) else b.t().contiguous()).bfloat16()
    lda = M if mode == 3 else kd
    ldb = N if mode in (2, 3) else kd
    ref = a @ b
    epi = K.EPI_F32_STORE
    for _ in range(4):
        C = torch.full((M, N), float("nan"), device=dev)
        K.gemm_glds(A, B, C, M=M, N=N, K=kd, lda=lda, ldb=ldb, ldc=N, mode=mode, epi=epi, tile=TILE)
        torch.cuda.synchronize()
        bad = (C != ref).sum().item()
        assert bad == 0, f"{bad} wrong elements"


def test_8ph_rejects(K):
    A = torch.zeros(256, 64, device=dev, dtype=torch.bfloat16)
    B = torch.zeros(64, 384, device=dev, dtype=torch.bfloat16)
    C = torch.zeros(256, 384, device=dev, dtype=torch.bfloat16)
    assert not K.gemm_glds_ok(A, B, C, M=256, N=384, K=64, lda=64, ldb=384, ldc=384, mode=2, epi=0, tile=TILE)
    assert not K.gemm_glds_ok(A, B, C, M=256, N=256, K=64, lda=64, ldb=384, ldc=384, mode=2, epi=0, tile=TILE,
                              splits=2)
