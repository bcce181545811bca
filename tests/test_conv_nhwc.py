"""The implicit-GEMM NHWC 3x3 convolution (csrc/conv_nhwc.hip, iit_amd/ops/conv.py) against an fp32 PyTorch
convolution of the same bf16 inputs: forward on every kernel tile, the input gradient (negated taps on the re-laid
weight) and the autograd op (library weight gradient)."""
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
    from iit_amd.ops.conv import _flip_weight
    torch.manual_seed(Cin + hw)
    x = torch.randn(N, Cin, hw, hw, device=dev).to(torch.bfloat16).contiguous(memory_format=CL)
    w = (torch.randn(Cout, Cin, 3, 3, device=dev) / (3 * Cin ** 0.5)).to(torch.bfloat16).contiguous(memory_format=CL)
    ref = F.conv2d(x.float(), w.float(), None, 1, 1)
    dy = torch.randn_like(ref).to(torch.bfloat16).contiguous(memory_format=CL)
    dx_ref = torch.nn.grad.conv2d_input(x.shape, w.float(), dy.float(), 1, 1)
    ran = 0
    for t in range(K.conv3x3_tiles()):
        if not K.conv3x3_ok(N, hw, hw, Cin, Cout, t):
            continue
        ran += 1
        y = torch.full((N, Cout, hw, hw), float("nan"), device=dev, dtype=torch.bfloat16).contiguous(memory_format=CL)
        K.conv3x3(x, w, y, N, hw, hw, Cin, Cout, False, t)
        assert rel(y, ref) < 8e-3, t
        if K.conv3x3_ok(N, hw, hw, Cout, Cin, t):
            dx = torch.full_like(x, float("nan"))
            K.conv3x3(dy, _flip_weight(w), dx, N, hw, hw, Cout, Cin, True, t)
            assert rel(dx, dx_ref) < 8e-3, t
    assert ran > 0


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
