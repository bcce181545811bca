"""Fused BatchNorm (+ residual) (+ ReLU) on channels-last bf16 (csrc/bn_nhwc.hip, iit_amd/ops/bn.py) against a
plain fp32 PyTorch reference of the same op on the same bf16 inputs, and the fused ResNet-18 against its module
path (IIT_FUSED_BN=0)."""
import os

import pytest
import torch

pytestmark = pytest.mark.gpu
dev = "cuda"


def rel(a, b):
    return float((a.float() - b.float()).norm() / (b.float().norm() + 1e-12))


def _ref(x, w, b, res, relu, training, rm, rv, eps, mom):
    xf = x.float()
    if training:
        mean = xf.mean((0, 2, 3))
        var = xf.var((0, 2, 3), unbiased=False)
        n = xf.numel() // xf.shape[1]
        rm = (1 - mom) * rm + mom * mean
        rv = (1 - mom) * rv + mom * var * n / (n - 1)
    else:
        mean, var = rm, rv
    y = (xf - mean[None, :, None, None]) * torch.rsqrt(var + eps)[None, :, None, None] * w[None, :, None, None] \
        + b[None, :, None, None]
    if res is not None:
        y = y + res.float()
    return (y.relu() if relu else y), rm, rv


@pytest.mark.parametrize("C,hw", [(64, 21), (128, 11), (256, 6), (512, 3)])
@pytest.mark.parametrize("res", [False, True])
@pytest.mark.parametrize("training", [True, False])
def test_bn_act_matches_fp32(C, hw, res, training):
    from iit_amd.ops import bn as fbn
    torch.manual_seed(C + hw)
    N = 64
    bn = torch.nn.BatchNorm2d(C).to(dev)
    with torch.no_grad():
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.uniform_(-0.5, 0.5)
        bn.running_mean.uniform_(-0.2, 0.2)
        bn.running_var.uniform_(0.5, 2.0)
    bn.train(training)
    x = (torch.randn(N, C, hw, hw, device=dev) * 1.5 + 0.3).bfloat16().contiguous(memory_format=torch.channels_last)
    r = torch.randn_like(x, memory_format=torch.channels_last) if res else None
    x.requires_grad_()
    if r is not None:
        r.requires_grad_()
    assert fbn.covered(x, bn, r)
    rm0, rv0, nbt0 = bn.running_mean.clone(), bn.running_var.clone(), int(bn.num_batches_tracked)
    y = fbn.bn_act(x, bn, r, relu=True)
    assert y.dtype == torch.bfloat16 and y.is_contiguous(memory_format=torch.channels_last)
    xr = x.detach().float().requires_grad_()
    rr = r.detach().float().requires_grad_() if r is not None else None
    wr, br = bn.weight.detach().clone().requires_grad_(), bn.bias.detach().clone().requires_grad_()
    yr, rm, rv = _ref(xr, wr, br, rr, True, training, rm0, rv0, bn.eps, bn.momentum)
    assert rel(y, yr) < 1e-2
    assert torch.allclose(bn.running_mean, rm, rtol=1e-4, atol=1e-5)
    assert torch.allclose(bn.running_var, rv, rtol=1e-4, atol=1e-5)
    assert int(bn.num_batches_tracked) == nbt0 + (1 if training else 0)
    g = torch.randn_like(yr)
    y.backward(g.bfloat16())
    yr.backward(g)
    assert rel(x.grad, xr.grad) < 2e-2
    assert rel(bn.weight.grad, wr.grad) < 1e-2 and rel(bn.bias.grad, br.grad) < 1e-2
    if r is not None:
        assert rel(r.grad, rr.grad) < 1e-2


def test_fused_resnet_matches_module_path():
    """ResNet-18 (84 x 84, channels-last, bf16 autocast, training mode) with the fused BN ops vs IIT_FUSED_BN=0, both
    against the fp32 model (no autocast): the fused path's error on the logits, the loss and every parameter gradient
    is within the module path's own bf16 error (plus a small floor); running statistics and num_batches_tracked
    after the step agree."""
    from iit_amd.models.resnet import resnet18
    torch.manual_seed(0)
    ms = [resnet18(num_classes=10).to(dev).to(memory_format=torch.channels_last) for _ in range(3)]
    for m in ms[1:]:
        m.load_state_dict(ms[0].state_dict())
    x = torch.rand(64, 3, 84, 84, device=dev).contiguous(memory_format=torch.channels_last)
    t = torch.randint(0, 10, (64,), device=dev)
    outs = []
    for m, env, amp in ((ms[0], "1", True), (ms[1], "0", True), (ms[2], "0", False)):
        os.environ["IIT_FUSED_BN"] = env
        try:
            with torch.autocast("cuda", dtype=torch.bfloat16, enabled=amp):
                y = m(x)
                loss = torch.nn.functional.cross_entropy(y.float(), t)
            loss.backward()
        finally:
            os.environ.pop("IIT_FUSED_BN", None)
        outs.append((y.float().detach(), float(loss)))
    (yf, lf), (ym, lm), (yr, lr) = outs
    print("logits err fused / module:", rel(yf, yr), rel(ym, yr), "loss", lf, lm, lr)
    assert rel(yf, yr) <= 1.5 * rel(ym, yr) + 1e-2
    assert abs(lf - lr) <= 1.5 * abs(lm - lr) + 1e-2 * abs(lr)
    worst = []
    for (n, pf), (_, pm), (_, pr) in zip(*(m.named_parameters() for m in ms)):
        ef, em = rel(pf.grad, pr.grad), rel(pm.grad, pr.grad)
        worst.append((ef - em, n, ef, em))
        assert ef <= 1.5 * em + 2e-2, (n, ef, em)
    worst.sort(reverse=True)
    print("gradient error fused vs module (worst 5):", worst[:5])
    for (n, bf), (_, bm) in zip(ms[0].named_buffers(), ms[1].named_buffers()):
        if bf.dtype == torch.long:
            assert torch.equal(bf, bm), n
        else:
            assert rel(bf, bm) < 1e-2, n
