"""The implicit-GEMM NHWC 3x3 convolution (csrc/conv_nhwc.hip, iit_amd/ops/conv.py) against an fp32 PyTorch
convolution of the same bf16 inputs: forward on every kernel tile, the input gradient (negated taps on the re-laid
weight), with and without the reduction split-K, the weight-gradient kernel and the autograd op."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
dev = "cuda"
CL = torch.channels_last


def rel(a, b):
    return float((a.float() - b.float()).norm() / (b.float().norm() + 1e-12))


@pytest.mark.parametrize("N,Cin,Cout,hw", [(128, 64, 64, 21), (128, 128, 128, 11), (128, 256, 256, 6),
                                           (128, 512, 512, 3), (16, 64, 128, 8)])
def test_conv3x3_matches_fp32(N, Cin, Cout, hw):
    from iit_amd.ops import hip_kernels as K
    torch.manual_seed(Cin + hw)
    x = torch.randn(N, Cin, hw, hw, device=dev).to(torch.bfloat16).contiguous(memory_format=CL)
    w = (torch.randn(Cout, Cin, 3, 3, device=dev) / (3 * Cin ** 0.5)).to(torch.bfloat16).contiguous(memory_format=CL)
    ref = F.conv2d(x.float(), w.float(), None, 1, 1)
    dy = torch.randn_like(ref).to(torch.bfloat16).contiguous(memory_format=CL)
    dx_ref = torch.nn.grad.conv2d_input(x.shape, w.float(), dy.float(), 1, 1)
    ran = split = 0
    for t in range(K.conv3x3_tiles()):
        for sp in (1, 2, 3, 4, 8):  # unsplit and the reduction split-K (fixed-order sum of fp32 partial tiles)
            if not K.conv3x3_ok(N, hw, hw, Cin, Cout, t, sp):
                continue
            ran += 1
            split += sp > 1
            y = torch.full((N, Cout, hw, hw), float("nan"), device=dev, dtype=torch.bfloat16).contiguous(
                memory_format=CL)
            K.conv3x3(x, w, y, N, hw, hw, Cin, Cout, False, t, sp)
            assert rel(y, ref) < 8e-3, (t, sp)
            if sp > 1:  # twice: the tickets were re-armed by the first launch
                y2 = torch.full_like(y, float("nan"))
                K.conv3x3(x, w, y2, N, hw, hw, Cin, Cout, False, t, sp)
                assert torch.equal(y, y2), (t, sp)
            if K.conv3x3_ok(N, hw, hw, Cout, Cin, t, sp):
                dx = torch.full_like(x, float("nan"))
                K.conv3x3(dy, w, dx, N, hw, hw, Cout, Cin, True, t, sp)
                assert rel(dx, dx_ref) < 8e-3, (t, sp)
    assert ran > 0 and split > 0


@pytest.mark.parametrize("N,Cin,Cout,hw", [(64, 64, 64, 21), (64, 128, 128, 11), (64, 256, 256, 6),
                                           (128, 512, 512, 3)])
def test_conv3x3_wgrad_matches_fp32(N, Cin, Cout, hw):
    """The weight-gradient kernel (k-major im2col columns gathered by the DMA) on every tile and K-split against the
    fp32 weight gradient of the same bf16 operands; store and accumulate epilogues."""
    from iit_amd.ops import hip_kernels as K
    torch.manual_seed(Cout + hw)
    x = torch.randn(N, Cin, hw, hw, device=dev).to(torch.bfloat16).contiguous(memory_format=CL)
    dy = torch.randn(N, Cout, hw, hw, device=dev).to(torch.bfloat16).contiguous(memory_format=CL)
    ref = torch.nn.grad.conv2d_weight(x.float(), (Cout, Cin, 3, 3), dy.float(), 1, 1)
    ran = 0
    for t in K.CONV_WG_TILES:
        for sp in K.conv3x3_wgrad_splits(N * hw * hw)[:4]:
            if not K.conv3x3_wgrad_ok(N, hw, hw, Cin, Cout, t, sp):
                continue
            ran += 1
            dw = torch.full((Cout, Cin, 3, 3), float("nan"), device=dev).contiguous(memory_format=CL)
            K.conv3x3_wgrad(dy, x, dw, N, hw, hw, Cin, Cout, False, t, sp)
            assert rel(dw, ref) < 1e-4, (t, sp)
            K.conv3x3_wgrad(dy, x, dw, N, hw, hw, Cin, Cout, True, t, sp)  # accumulate: 2 x
            assert rel(dw, 2 * ref) < 1e-4, (t, sp)
    assert ran > 0


def test_conv3x3_autograd_arena_weight(monkeypatch):
    """The autograd op on an arena weight (fp32 master, bf16 mirror): output, input gradient and the fp32 weight
    gradient written into the arena slot, against fp32 torch -- with every pass forced onto the repo's kernels."""
    from iit_amd.engine.flat import FlatParams
    from iit_amd.ops import conv as hconv
    monkeypatch.setattr(hconv, "POLICY", "1")
    hconv.DECISIONS.clear()
    torch.manual_seed(0)
    conv = torch.nn.Conv2d(64, 128, 3, padding=1, bias=False).to(dev).to(memory_format=CL)
    flat = FlatParams(conv, with_bf16_shadow=True)
    W = conv.weight
    x = torch.randn(64, 64, 21, 21, device=dev).to(torch.bfloat16).contiguous(memory_format=CL).requires_grad_()
    assert hconv.covered(x, conv)
    y = hconv.conv3x3(x, W, flat)
    g = torch.randn_like(y)
    y.backward(g)
    assert all(ch is not None for ch, _ in hconv.DECISIONS.values()) and len(hconv.DECISIONS) == 3
    xr = x.detach().float().requires_grad_()
    wr = flat.shadow_view(W).detach().float().requires_grad_()
    yr = F.conv2d(xr, wr, None, 1, 1)
    yr.backward(g.float())
    assert rel(y, yr) < 8e-3
    assert rel(x.grad, xr.grad) < 1e-2 and rel(W.grad, wr.grad) < 1e-3


@pytest.mark.parametrize("N,C,hw,tile,splits,offset", [(128, 64, 21, 0, 1, 0.0), (64, 128, 11, 3, 2, 0.0),
                                                       (128, 256, 6, 4, 1, 40.0), (128, 512, 3, 2, 4, 0.0)])
def test_conv_epilogue_bn_statistics(N, C, hw, tile, splits, offset):
    """BatchNorm statistics from the conv epilogue (per-tile column records, gemm_glds_body.h E_BF16_CS, combined
    around the batch's first row by bn_tile_finalize_kernel) against the BatchNorm's own statistics pass on the same
    bf16 output: same normalised output, running statistics and num_batches_tracked; ``offset`` puts the channel means
    far from zero (the pivot keeps the variance from cancelling), checked against float64."""
    from iit_amd.ops import hip_kernels as K
    torch.manual_seed(C + hw)
    if not K.conv3x3_ok(N, hw, hw, C, C, tile, splits):
        pytest.skip("tile does not cover the shape")
    x = torch.randn(N, C, hw, hw, device=dev).to(torch.bfloat16).contiguous(memory_format=CL)
    w = (torch.randn(C, C, 3, 3, device=dev) / (3 * C ** 0.5)).to(torch.bfloat16).contiguous(memory_format=CL)
    y = torch.empty(N, C, hw, hw, device=dev, dtype=torch.bfloat16).contiguous(memory_format=CL)
    T = N * hw * hw // K.conv3x3_rows(tile)
    cstat = torch.full((3 * C * T,), float("nan"), device=dev)
    K.conv3x3(x, w, y, N, hw, hw, C, C, False, tile, splits, cstat=cstat)
    y0 = torch.empty_like(y)
    K.conv3x3(x, w, y0, N, hw, hw, C, C, False, tile, splits)
    assert torch.equal(y, y0)  # the statistics do not change the output
    if offset:
        y = (y.float() + offset).to(torch.bfloat16).contiguous(memory_format=CL)
        cstat2 = torch.full_like(cstat, float("nan"))  # re-derive the records of the shifted output from its rows
        v = y.permute(0, 2, 3, 1).reshape(T, -1, C).float()
        piv = v[:, 0, :]
        d = v - piv[:, None, :]
        cstat2.view(3, C, T)[0] = piv.t()
        cstat2.view(3, C, T)[1] = d.sum(1).t()
        cstat2.view(3, C, T)[2] = (d * d).sum(1).t()
        cstat = cstat2
    M = N * hw * hw
    gw = torch.rand(C, device=dev) + 0.5
    gb = torch.randn(C, device=dev)
    outs = []
    for use_tiles in (True, False):
        rm, rv = torch.zeros(C, device=dev), torch.ones(C, device=dev)
        nbt = torch.zeros((), dtype=torch.long, device=dev)
        out = torch.empty_like(y)
        save = torch.empty(2 * C, device=dev)
        if use_tiles:
            K.bn_fwd_tiles(y, None, out, cstat, T, M // T, rm, rv, gw, gb, M, C, 1e-5, True, save, 0.1, nbt)
        else:
            ws = torch.zeros(K.bn_ws_floats(C), device=dev)
            K.bn_fwd(y, None, out, ws, rm, rv, gw, gb, M, C, 1e-5, True, True, save, 0.1, nbt)
        outs.append((out, rm, rv, nbt, save))
    (o1, rm1, rv1, n1, s1), (o2, rm2, rv2, n2, s2) = outs
    assert int(n1) == int(n2) == 1
    assert rel(o1, o2) < 4e-3
    yd = y.double().permute(0, 2, 3, 1).reshape(-1, C)
    mean, var = yd.mean(0), yd.var(0, unbiased=False)
    assert float(((s1[:C].double() - mean).abs() / (var.sqrt() + 1e-6)).max()) < 1e-3
    assert float(((s1[C:].double() - (var + 1e-5).rsqrt()).abs() / (var + 1e-5).rsqrt()).max()) < 2e-3
    assert rel(rm1, rm2) < 1e-3 and rel(rv1, rv2) < 1e-3


@pytest.mark.parametrize("N,Cin,Cout,hw,k,s", [(64, 64, 128, 21, 3, 2), (64, 128, 256, 11, 3, 2),
                                              (64, 256, 512, 6, 3, 2), (64, 64, 128, 21, 1, 2),
                                              (64, 256, 512, 6, 1, 2), (32, 64, 64, 8, 1, 1)])
def test_conv2d_strided_and_pointwise_match_fp32(N, Cin, Cout, hw, k, s):
    """The general implicit-GEMM entry points on the ResNet's other body convolutions -- the 3 x 3 stride-2 first
    convolution of layers 2-4 and the 1 x 1 (stride-2) downsample: forward, the transposed input gradient (stride 2:
    the taps that do not divide read the zero page) and the weight gradient, every covering tile / split, against
    fp32 torch on the same bf16 operands."""
    from iit_amd.ops import hip_kernels as K
    from iit_amd.ops.conv import _out_hw, _relaid
    torch.manual_seed(Cin + hw + k + s)
    pad = k // 2
    x = torch.randn(N, Cin, hw, hw, device=dev).to(torch.bfloat16).contiguous(memory_format=CL)
    w = (torch.randn(Cout, Cin, k, k, device=dev) / (k * Cin ** 0.5)).to(torch.bfloat16).contiguous(memory_format=CL)
    ref = F.conv2d(x.float(), w.float(), None, s, pad)
    OH, OW = _out_hw(hw, hw, k, s, pad)
    assert ref.shape[2:] == (OH, OW)
    dy = torch.randn_like(ref).to(torch.bfloat16).contiguous(memory_format=CL)
    dx_ref = torch.nn.grad.conv2d_input(x.shape, w.float(), dy.float(), s, pad)
    dw_ref = torch.nn.grad.conv2d_weight(x.float(), w.shape, dy.float(), s, pad)
    wf = w  # the transposed kernel reads the forward weight in place
    fwd = dgr = wgr = 0
    for t in range(K.conv3x3_tiles()):
        for sp in (1, 2, 3):
            if K.conv2d_ok(N, hw, hw, Cin, OH, OW, Cout, k, s, pad, False, t, sp):
                fwd += 1
                y = torch.full((N, Cout, OH, OW), float("nan"), device=dev, dtype=torch.bfloat16).contiguous(
                    memory_format=CL)
                K.conv2d(x, w, y, N, hw, hw, Cin, OH, OW, Cout, k, s, pad, False, t, sp)
                assert rel(y, ref) < 8e-3, ("fwd", t, sp)
            if K.conv2d_ok(N, OH, OW, Cout, hw, hw, Cin, k, s, pad, True, t, sp):
                dgr += 1
                dx = torch.full_like(x, float("nan"))
                K.conv2d(dy, wf, dx, N, OH, OW, Cout, hw, hw, Cin, k, s, pad, True, t, sp)
                assert rel(dx, dx_ref) < 8e-3, ("dgrad", t, sp)
                dx2 = torch.full_like(x, float("nan"))  # mode 2: the re-laid k-contiguous weight copy
                K.conv2d(dy, _relaid(w), dx2, N, OH, OW, Cout, hw, hw, Cin, k, s, pad, 2, t, sp)
                assert rel(dx2, dx_ref) < 8e-3, ("dgrad relaid", t, sp)
    for t in K.CONV_WG_TILES:
        for sp in K.conv3x3_wgrad_splits(N * OH * OW)[:3]:
            if K.conv2d_wgrad_ok(N, hw, hw, Cin, OH, OW, Cout, k, s, pad, t, sp):
                wgr += 1
                dw = torch.full((Cout, Cin, k, k), float("nan"), device=dev).contiguous(memory_format=CL)
                K.conv2d_wgrad(dy, x, dw, N, hw, hw, Cin, OH, OW, Cout, k, s, pad, False, t, sp)
                assert rel(dw, dw_ref) < 1e-4, ("wgrad", t, sp)
    assert fwd > 0 and dgr > 0 and wgr > 0, (fwd, dgr, wgr)


def test_resnet_block_convs_on_repo_kernels(monkeypatch):
    """A stride-2 BasicBlock with its 1 x 1 downsample under bf16 autocast, every convolution forced onto the repo's
    kernels (IIT_CONV_HIP=1 policy): output and every parameter gradient against the same block in fp32 within the
    library bf16 path's own error."""
    from iit_amd.engine.flat import FlatParams
    from iit_amd.models.resnet import BasicBlock, conv1x1
    from iit_amd.ops import conv as hconv
    monkeypatch.setattr(hconv, "POLICY", "1")
    monkeypatch.setattr(hconv, "GEOMS", {"k3s1", "k3s2", "k1s1", "k1s2"})  # (k3s2 is opt-in by default)
    hconv.DECISIONS.clear()
    torch.manual_seed(1)
    blocks = []
    for _ in range(3):
        ds = torch.nn.Sequential(conv1x1(64, 128, 2), torch.nn.BatchNorm2d(128))
        blocks.append(BasicBlock(64, 128, 2, ds).to(dev).to(memory_format=CL))
    for b in blocks[1:]:
        b.load_state_dict(blocks[0].state_dict())
    FlatParams(blocks[0], with_bf16_shadow=True)
    x = torch.randn(64, 64, 21, 21, device=dev).contiguous(memory_format=CL)
    outs = []
    for b, env, amp in ((blocks[0], "1", True), (blocks[1], "0", True), (blocks[2], "0", False)):
        monkeypatch.setenv("IIT_CONV_MIRROR", env)
        xi = x.clone().requires_grad_()
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=amp):
            y = b(xi)
        y.float().square().mean().backward()
        outs.append((y.float().detach(), xi.grad.float()))
    kinds = {key[0] + str(key[6]) + str(key[7]) for key in hconv.DECISIONS}
    assert {"fwd32", "fwd12", "dgrad32", "dgrad12", "wgrad32", "wgrad12"} <= kinds, kinds
    assert all(ch is not None for ch, _ in hconv.DECISIONS.values())
    (ym, gm), (yc, gc), (yr, gr) = outs
    assert rel(ym, yr) <= 1.5 * rel(yc, yr) + 1e-2
    assert rel(gm, gr) <= 1.5 * rel(gc, gr) + 2e-2
    for (n, pm), (_, pc), (_, pr) in zip(*(b.named_parameters() for b in blocks)):
        assert pm.grad is not None, n
        em, ec = rel(pm.grad, pr.grad), rel(pc.grad, pr.grad)
        assert em <= 1.5 * ec + 2e-2, (n, em, ec)
