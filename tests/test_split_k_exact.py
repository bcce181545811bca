"""Split-K publication audit: every in-step split-K path, run right after kernels that dirty the L2
of every XCD with garbage over the output and the partial-tile workspace, must equal the non-split result BITWISE.

Operands are small integers (exact in bf16; every partial sum below 2^24, exact in fp32), so the result does not
depend on the order the partials are added in: a lost, duplicated or stale partial tile -- an atomic add that did
not land, a reduction that read a slab line another XCD had not yet written back, a ticket that was not re-armed --
shows up as a wrong element, never as rounding.  The paths:

* atomic split-K (fp32 ``global_atomic_add`` into C) of the LDS-DMA kernel (``glds*k*``) and of the older hip
  kernel (``csrc/gemm.hip``);
* the deterministic reduction split-K (``glds*r*``): write-through (``sc1``) slab stores, ``s_waitcnt vmcnt(0)``,
  a workgroup barrier, one relaxed agent-scope ticket per tile; the last arriver reads the other slabs with ``sc1``
  loads (cdna_hip_programming.md "Projection GEMM at M = 256" item 2, MI355X_MICROARCH.md hand-off table row 1);
* the dual dX + dW launch with atomic and reduction splits of its dW problem.

The root cause of the round-4 run-to-run gradient variation is recorded in profiles/split_store_rootcause_r5.txt:
fp32 summation ORDER of >= 2 atomic adders per element (a last-bit difference in the residual stream that a later
bf16 rounding can turn into a whole bf16 ulp), not a publication hazard -- this test is the publication half.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu
dev = "cuda"


@pytest.fixture(scope="module")
def K():
    from iit_amd.ops import hip_kernels
    hip_kernels.lib()
    return hip_kernels


def _ints(shape, lo, hi, seed):
    g = torch.Generator(device=dev).manual_seed(seed)
    return torch.randint(lo, hi, shape, device=dev, generator=g).float()


def _dirty(*bufs):
    """Plain-store garbage over each buffer from every CU (dirty lines in every XCD's L2), then a second kernel that
    reads it all back (clean copies of the garbage in the L2s / L1s)."""
    for b in bufs:
        if b is not None:
            b.fill_(float("nan") if b.dtype.is_floating_point else -7)
    s = sum(float(b.float().nan_to_num(1.0).sum()) for b in bufs if b is not None)
    return s


def _operands(K, mode, M, N, Kd, seed):
    a = _ints((M, Kd), -3, 4, seed)
    b = _ints((Kd, N), -2, 3, seed + 1)
    A = (a.t().contiguous() if mode & K.MODE_AKM else a).bfloat16()
    B = (b if mode & K.MODE_BKM else b.t().contiguous()).bfloat16()
    lda = M if mode & K.MODE_AKM else Kd
    ldb = N if mode & K.MODE_BKM else Kd
    return A, B, lda, ldb, a @ b


GLDS_SPLITS = [  # (tile, splits, reduce, mode, epi)
    (0, 2, False, 3, 5), (3, 4, False, 3, 5), (30, 8, False, 3, 5), (25, 16, False, 3, 5),
    (8, 2, True, 3, 5), (8, 4, True, 3, 7), (26, 2, True, 3, 7), (30, 4, True, 3, 7), (20, 4, True, 3, 7),
    (23, 2, True, 2, 2), (24, 4, True, 2, 2), (29, 2, True, 2, 2),
]


@pytest.mark.parametrize("tile,splits,reduce,mode,epi", GLDS_SPLITS)
def test_glds_split_k_exact_after_dirty_l2(K, tile, splits, reduce, mode, epi):
    bm, bn = K.GLDS_TILES[tile]
    M, N, Kd = bm * 4, bn * 3, 64 * 4 * splits * 2
    A, B, lda, ldb, ref = _operands(K, mode, M, N, Kd, tile * 31 + splits)
    C0 = _ints((M, N), -50, 50, 7)
    R = _ints((M, N), -50, 50, 8) if epi == K.EPI_F32_RESID else None
    bias = _ints((N,), -5, 5, 9) if epi in (K.EPI_F32_RESID, K.EPI_F32_STORE) and mode != 3 else None
    exp = ref + (C0 if epi == K.EPI_F32_ACC else 0) + (R if R is not None else 0) + (bias if bias is not None else 0)
    kw = dict(M=M, N=N, K=Kd, lda=lda, ldb=ldb, ldc=N, mode=mode, epi=epi, tile=tile)
    assert K.gemm_glds_ok(A, B, C0, resid=R, ldr=N if R is not None else 0, splits=splits, reduce=reduce, **kw)
    ws = cnt = None
    if reduce:
        ws, cnt = K.split_workspace(M, N, tile, splits, A.device)
        ws = ws[: splits * M * N]  # the partial tiles this launch writes
    for rep in range(4):
        C = torch.empty_like(C0)
        _dirty(C, ws)
        C.copy_(C0)  # (an accumulate reads C: written by a kernel right before, its lines dirty in the L2s)
        K.gemm_glds(A, B, C, resid=R, ldr=N if R is not None else 0, bias0=bias, splits=splits, reduce=reduce, **kw)
        torch.cuda.synchronize()
        bad = int((C != exp).sum())
        assert bad == 0, f"rep {rep}: {bad} of {C.numel()} elements differ from the exact result"
    if reduce:
        assert int(cnt.abs().sum()) == 0  # every ticket re-armed


@pytest.mark.parametrize("splits", [2, 4, 8])
def test_hip_kernel_atomic_split_k_exact_after_dirty_l2(K, splits):
    """The older hip kernel's atomic split-K (csrc/gemm.hip), incl. a partial M tile (32 rows: the round-4
    last-position residual shape) -- the removed split-store candidate's accumulate launch."""
    for M, N, Kd in ((32, 128, 512), (200, 384, 1024)):
        A, B, lda, ldb, ref = _operands(K, K.MODE_BKM, M, N, Kd, splits + M)
        C0 = _ints((M, N), -50, 50, 3)
        for rep in range(4):
            C = torch.empty_like(C0)
            _dirty(C)
            C.copy_(C0)
            K.gemm(A, B, C, M=M, N=N, K=Kd, lda=lda, ldb=ldb, ldc=N, mode=K.MODE_BKM, epi=K.EPI_F32_ACC,
                   splits=splits)
            torch.cuda.synchronize()
            assert int((C != C0 + ref).sum()) == 0, (M, rep)


@pytest.mark.parametrize("wtile,xtile,splits,reduce", [(1, 3, 2, True), (0, 1, 4, True), (2, 3, 2, False),
                                                        (5, 5, 2, True), (7, 7, 4, True), (8, 8, 2, False)])
def test_dual_split_k_exact_after_dirty_l2(K, wtile, xtile, splits, reduce):
    wbm, wbn = K.DUAL_W_TILES[wtile]
    xbm, xbn = K.DUAL_X_TILES[xtile]
    T = 64 * 4 * splits * 2  # tokens: the dW reduction
    Mw, Nw = wbm * 3, wbn * 2
    X = _ints((T, Mw), -3, 4, 11)
    dY = _ints((T, Nw), -2, 3, 12)
    Wm = _ints((xbn * 2, 256), -2, 3, 13)  # dX = dY' W^T with dY' [xbm * 2][256], W [xbn * 2][256]
    dYx = _ints((xbm * 2, 256), -3, 4, 14)
    w = dict(A=X.bfloat16(), B=dY.bfloat16(), M=Mw, N=Nw, K=T, lda=Mw, ldb=Nw, ldc=Nw, epi=K.EPI_F32_ACC)
    x = dict(A=dYx.bfloat16(), B=Wm.bfloat16(), M=xbm * 2, N=xbn * 2, K=256, lda=256, ldb=256, ldc=xbn * 2,
             epi=K.EPI_BF16)
    C0 = _ints((Mw, Nw), -50, 50, 15)
    expw = C0 + X.t() @ dY
    expx = (dYx @ Wm.t()).bfloat16().float()  # the exact sum rounded once to the bf16 output
    ws = None
    for rep in range(4):
        w["C"] = torch.empty_like(C0)
        x["C"] = torch.empty(x["M"], x["N"], device=dev, dtype=torch.bfloat16)
        if rep == 0:
            if not K.gemm_dual_ok(w, x, wtile, xtile, splits, reduce):
                pytest.skip("pair not covered by this dual tile family")
            if reduce:
                ws, _ = K.split_workspace(Mw, Nw, K.DUAL_W_TILES[wtile], splits, X.device)
                ws = ws[: splits * Mw * Nw]  # the partial tiles this launch writes
        _dirty(w["C"], x["C"], ws)
        w["C"].copy_(C0)
        K.gemm_dual(w, x, wtile, xtile, splits, reduce)
        torch.cuda.synchronize()
        assert int((w["C"] != expw).sum()) == 0, rep
        assert int((x["C"].float() != expx).sum()) == 0, rep
