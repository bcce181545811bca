"""Dual GEMM launch (csrc/gemm_dual.hip): a layer's dW = X^T dY and dX = dY W^T in one launch vs fp32 PyTorch,
for every (dW tile, dX tile) pair, both epilogues of each side, and the dW K-splits (reduction / atomic)."""
import pytest
import torch

pytestmark = pytest.mark.gpu
dev = "cuda"
T, KIN, NOUT = 512, 384, 384


@pytest.fixture(scope="module")
def K():
    from iit_amd.ops import hip_kernels
    hip_kernels.lib()
    return hip_kernels


def _problem(seed, kin=KIN, nout=NOUT):
    torch.manual_seed(seed)
    x = torch.randn(T, kin, device=dev).bfloat16()
    dy = (torch.randn(T, nout, device=dev) / 4).bfloat16()
    w = (torch.randn(kin, nout, device=dev) / 8).bfloat16()
    pre = torch.randn(T, kin, device=dev).bfloat16()
    return x, dy, w, pre


# (dW tile, dX tile) pairs: every pair of the 4-wave family, every pair of the 8-wave family
PAIRS = ([(wt, xt) for wt in range(5) for xt in range(4)] + [(wt, xt) for wt in (5, 6) for xt in (4, 5, 6)]
         + [(wt, xt) for wt in (7, 8) for xt in (7, 8)])


VARIANTS = [  # (dW epilogue, dX epilogue, splits, reduce)
    ("store", "bf16", 1, False),
    ("store", "dgelu", 2, True),
    ("acc", "bf16", 4, True),
    ("acc", "dgelu", 2, False),
]


@pytest.mark.parametrize("wt,xt", PAIRS)
@pytest.mark.parametrize("variant", VARIANTS, ids=lambda v: f"{v[0]}-{v[1]}-{'r' if v[3] else 'k'}{v[2]}")
def test_dual_matches_fp32(K, wt, xt, variant):
    from iit_amd.ops.torch_ops import gelu_new
    wepi_s, xepi_s, splits, reduce = variant
    KIN, NOUT = (768, 768) if wt >= 5 else (384, 384)  # the 8-wave tiles need 256-row / 192-column multiples
    x, dy, w, pre = _problem(wt * 10 + xt, KIN, NOUT)
    wepi = K.EPI_F32_STORE if wepi_s == "store" else K.EPI_F32_ACC
    xepi = K.EPI_BF16 if xepi_s == "bf16" else K.EPI_DGELU
    gW0 = torch.randn(KIN, NOUT, device=dev)
    gW = gW0.clone()
    dX = torch.zeros(T, KIN, device=dev, dtype=torch.bfloat16)
    csum = torch.randn(KIN, device=dev) if xepi == K.EPI_DGELU else None
    csum0 = csum.clone() if csum is not None else None
    bsum0 = torch.randn(NOUT, device=dev)
    bsum = bsum0.clone()
    gsq = torch.zeros(64, device=dev)
    ws = dict(A=x, B=dy, C=gW, M=KIN, N=NOUT, K=T, lda=KIN, ldb=NOUT, ldc=NOUT, epi=wepi, bsum=bsum, gsq=gsq)
    xs = dict(A=dy, B=w, C=dX, C2=pre if xepi == K.EPI_DGELU else None, M=T, N=KIN, K=NOUT, lda=NOUT, ldb=NOUT,
              ldc=KIN, ldc2=KIN, epi=xepi, csum=csum)
    assert K.gemm_dual_ok(ws, xs, wt, xt, splits, reduce)
    for rep in range(2):  # a second launch reuses the reduction tickets the first one re-armed
        gW.copy_(gW0)
        bsum.copy_(bsum0)
        gsq.zero_()
        if csum is not None:
            csum.copy_(csum0)
        K.gemm_dual(ws, xs, wt, xt, splits, reduce)
        torch.cuda.synchronize()
        ref_w = x.float().t() @ dy.float() + (gW0 if wepi == K.EPI_F32_ACC else 0)
        torch.testing.assert_close(gW, ref_w, rtol=1e-4, atol=2e-3)
        torch.testing.assert_close(bsum, bsum0 + dy.float().sum(0), rtol=1e-4, atol=2e-3)  # fused bias gradient
        if wepi == K.EPI_F32_STORE:  # fused sum of squares of the stored gradient (the clip's norm share)
            torch.testing.assert_close(gsq.sum(), gW.double().pow(2).sum().float(), rtol=1e-4, atol=1e-3)
        else:
            assert float(gsq.abs().sum()) == 0.0
        ref_x = dy.float() @ w.float().t()
        if xepi == K.EPI_DGELU:
            p = pre.float().requires_grad_(True)
            gp, = torch.autograd.grad(gelu_new(p).sum(), p)
            ref_x = (ref_x * gp).bfloat16().float()
            torch.testing.assert_close(csum, csum0 + dX.float().sum(0), rtol=1e-4, atol=1e-2)
        torch.testing.assert_close(dX.float(), ref_x, rtol=2e-2, atol=2e-2)


def test_dual_rejects_misfit(K):
    x, dy, w, pre = _problem(0)
    gW = torch.zeros(KIN, NOUT, device=dev)
    dX = torch.zeros(T, KIN, device=dev, dtype=torch.bfloat16)
    ws = dict(A=x, B=dy, C=gW, M=KIN, N=NOUT, K=T, lda=KIN, ldb=NOUT, ldc=NOUT, epi=K.EPI_F32_STORE)
    xs = dict(A=dy, B=w, C=dX, M=T, N=KIN - 8, K=NOUT, lda=NOUT, ldb=NOUT, ldc=KIN, epi=K.EPI_BF16)
    assert not K.gemm_dual_ok(ws, xs, 0, 0)  # N not a multiple of the dX tile
    xs["N"] = KIN
    assert not K.gemm_dual_ok(ws, xs, 0, 0, 2, False)  # atomic split of a store epilogue
    assert K.gemm_dual_ok(ws, xs, 0, 0, 2, True)


def test_gemm_pair_dispatch_matches_serial(K):
    """The dispatcher's pair path (whatever it picks) gives the serial results, and both layer backwards agree."""
    from iit_amd.ops import gemm_dispatch as gd
    x, dy, w, pre = _problem(7)
    outs = []
    for dual in (False, True):
        gd.DUAL = dual
        gW = torch.empty(KIN, NOUT, device=dev)
        dX = torch.empty(T, KIN, device=dev, dtype=torch.bfloat16)
        xs = dict(A=dy, B=w, C=dX, M=T, N=KIN, K=NOUT, lda=NOUT, ldb=NOUT, ldc=KIN, epi=K.EPI_BF16)
        wspec = dict(A=x, B=dy, C=gW, M=KIN, N=NOUT, K=T, lda=KIN, ldb=NOUT, ldc=NOUT, mode=K.MODE_AKM | K.MODE_BKM,
                     epi=K.EPI_F32_STORE, fresh=True)
        gd.gemm_pair(xs, wspec)
        torch.cuda.synchronize()
        outs.append((gW.clone(), dX.clone()))
    gd.DUAL = True
    torch.testing.assert_close(outs[0][0], outs[1][0], rtol=1e-4, atol=2e-3)
    torch.testing.assert_close(outs[0][1].float(), outs[1][1].float(), rtol=1e-2, atol=1e-2)


@pytest.mark.parametrize("tile", [0, 3, 5, 8, 9, 20, 23, 25, 26, 30])
@pytest.mark.parametrize("epi,splits,reduce", [(7, 1, False), (5, 2, False), (7, 2, True), (5, 4, True)])
def test_glds_weight_grad_bias_sums(K, tile, epi, splits, reduce):
    """Single-launch LDS-DMA weight gradient (mode 3) with the fused column sums of dY (``bsum``)."""
    bm, bn = K.GLDS_TILES[tile]
    M, N, Tk = bm * 2, bn * 2, 512
    torch.manual_seed(tile)
    x = torch.randn(Tk, M, device=dev).bfloat16()
    dy = torch.randn(Tk, N, device=dev).bfloat16()
    C0 = torch.randn(M, N, device=dev)
    C = C0.clone()
    bs0 = torch.randn(N, device=dev)
    bs = bs0.clone()
    kw = dict(M=M, N=N, K=Tk, lda=M, ldb=N, ldc=N, mode=K.MODE_AKM | K.MODE_BKM, epi=epi, tile=tile, splits=splits,
              reduce=reduce)
    if not K.gemm_glds_ok(x, dy, C, **{k: v for k, v in kw.items()}):
        pytest.skip("tile does not cover this case")
    sq = torch.zeros(64, device=dev)
    K.gemm_glds(x, dy, C, bsum=bs, gsq=sq, **kw)
    torch.cuda.synchronize()
    ref = x.float().t() @ dy.float() + (C0 if epi == K.EPI_F32_ACC else 0)
    torch.testing.assert_close(C, ref, rtol=1e-4, atol=2e-3)
    torch.testing.assert_close(bs, bs0 + dy.float().sum(0), rtol=1e-4, atol=2e-3)
    if epi == K.EPI_F32_STORE:
        torch.testing.assert_close(sq.sum(), C.double().pow(2).sum().float(), rtol=1e-4, atol=1e-2)


@pytest.mark.parametrize("tile", [5, 7, 9, 23, 25])
@pytest.mark.parametrize("splits", [2, 4])
def test_glds_residual_reduction_split(K, tile, splits):
    """Forward fp32 residual GEMM (mode 2, ``resid + x W + b``) with the deterministic reduction split-K: the
    last-arriving split adds bias and residual once; bit-identical across launches."""
    bm, bn = K.GLDS_TILES[tile]
    M, N, Kd = bm * 2, bn * 2, 1024
    torch.manual_seed(tile + splits)
    x = torch.randn(M, Kd, device=dev).bfloat16()
    w = (torch.randn(Kd, N, device=dev) / 16).bfloat16()
    resid = torch.randn(M, N, device=dev)
    bias = torch.randn(N, device=dev)
    kw = dict(M=M, N=N, K=Kd, lda=Kd, ldb=N, ldc=N, mode=K.MODE_BKM, epi=K.EPI_F32_RESID, resid=resid, ldr=N,
              tile=tile, splits=splits, reduce=True)
    C = torch.empty(M, N, device=dev)
    assert K.gemm_glds_ok(x, w, C, **kw)
    outs = []
    for _ in range(2):
        C.fill_(float("nan"))
        K.gemm_glds(x, w, C, bias0=bias, **kw)
        torch.cuda.synchronize()
        outs.append(C.clone())
    ref = resid + x.float() @ w.float() + bias
    torch.testing.assert_close(outs[0], ref, rtol=1e-4, atol=2e-3)
    assert torch.equal(outs[0], outs[1])
