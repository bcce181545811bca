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


@pytest.mark.parametrize("N,Cin,Cout,hw", [(8, 64, 64, 21), (16, 128, 128, 11), (32, 256, 256, 6), (64, 512, 512, 3),
                                           (16, 64, 128, 8)])
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


@pytest.mark.parametrize("policy", ["1"])
def test_conv3x3_autograd(monkeypatch, policy):
    from iit_amd.ops import conv as hconv
    monkeypatch.setattr(hconv, "POLICY", policy)
    hconv.DECISIONS.clear()
    torch.manual_seed(0)
    x = torch.randn(16, 64, 21, 21, device=dev).to(torch.bfloat16).contiguous(memory_format=CL).requires_grad_()
    w = (torch.randn(64, 64, 3, 3, device=dev) / 24).to(torch.bfloat16).contiguous(memory_format=CL).requires_grad_()
    y = hconv.conv3x3(x, w)
    assert any(t is not None for t, _ in hconv.DECISIONS.values())  # the repo's kernel ran
    g = torch.randn_like(y)
    y.backward(g)
    xr = x.detach().float().requires_grad_()
    wr = w.detach().float().requires_grad_()
    yr = F.conv2d(xr, wr, None, 1, 1)
    yr.backward(g.float())
    assert rel(y, yr) < 8e-3
    assert rel(x.grad, xr.grad) < 1e-2 and rel(w.grad, wr.grad) < 1e-2
