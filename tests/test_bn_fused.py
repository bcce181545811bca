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
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_bn_act_matches_fp32(C, hw, res, training, dtype):
    """The fused NHWC BatchNorm(+residual)+ReLU op on bf16 or fp32 activations against the fp32 torch reference
    (fp32 activations: tolerances 1e-4, the kernels' fp32 statistics against torch's)."""
    from iit_amd.ops import bn as fbn
    torch.manual_seed(C + hw)
    tol = 1.0 if dtype == torch.bfloat16 else 1e-2  # scales the bf16 tolerances down for fp32
    N = 64
    bn = torch.nn.BatchNorm2d(C).to(dev)
    with torch.no_grad():
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.uniform_(-0.5, 0.5)
        bn.running_mean.uniform_(-0.2, 0.2)
        bn.running_var.uniform_(0.5, 2.0)
    bn.train(training)
    x = (torch.randn(N, C, hw, hw, device=dev) * 1.5 + 0.3).to(dtype).contiguous(memory_format=torch.channels_last)
    r = torch.randn_like(x, memory_format=torch.channels_last) if res else None
    x.requires_grad_()
    if r is not None:
        r.requires_grad_()
    assert fbn.covered(x, bn, r)
    rm0, rv0, nbt0 = bn.running_mean.clone(), bn.running_var.clone(), int(bn.num_batches_tracked)
    y = fbn.bn_act(x, bn, r, relu=True)
    assert y.dtype == dtype and y.is_contiguous(memory_format=torch.channels_last)
    xr = x.detach().float().requires_grad_()
    rr = r.detach().float().requires_grad_() if r is not None else None
    wr, br = bn.weight.detach().clone().requires_grad_(), bn.bias.detach().clone().requires_grad_()
    yr, rm, rv = _ref(xr, wr, br, rr, True, training, rm0, rv0, bn.eps, bn.momentum)
    assert rel(y, yr) < 1e-2 * tol
    assert torch.allclose(bn.running_mean, rm, rtol=1e-4, atol=1e-5)
    assert torch.allclose(bn.running_var, rv, rtol=1e-4, atol=1e-5)
    assert int(bn.num_batches_tracked) == nbt0 + (1 if training else 0)
    g = torch.randn_like(yr)
    y.backward(g.to(dtype))
    yr.backward(g)
    assert rel(x.grad, xr.grad) < 2e-2 * tol
    assert rel(bn.weight.grad, wr.grad) < 1e-2 * tol and rel(bn.bias.grad, br.grad) < 1e-2 * tol
    if r is not None:
        assert rel(r.grad, rr.grad) < 1e-2 * tol


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


@pytest.mark.parametrize("hook", ["mod.layer3.mod.1.mod.conv2.hook_point", "mod.layer1.mod.0.mod.conv1.hook_point",
                                  "mod.conv1.hook_point"])
def test_conv_hook_splice_read_by_fused_bn(hook):
    """A plan splice at a conv hook of the wrapped PVR ResNet (the IIT intervention of train.py) is applied by the
    fused BatchNorm's reads (no splice_kernel launch) and equals the separate splice pass bitwise: logits, input
    gradient and every parameter gradient (IIT_BN_SPLICE=0 is the separate pass)."""
    from iit_amd.core.index import Ix
    from iit_amd.engine.plan import RunPlan
    from iit_amd.ops import hip_kernels as K
    from iit_amd.tasks.task_loader import get_alignment
    torch.manual_seed(0)
    ll, _, _ = get_alignment("mnist_pvr", config={"input_shape": (1, 3, 84, 84), "device": dev})
    ll.to(memory_format=torch.channels_last)
    xs = torch.rand(32, 3, 84, 84, device=dev)
    xb = torch.rand(32, 3, 84, 84, device=dev)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        src = ll.run_capture(xs.contiguous(memory_format=torch.channels_last), [hook])[hook]
    hw = src.shape[-1] // 2
    outs = []
    for env in ("1", "0"):
        os.environ["IIT_BN_SPLICE"] = env
        calls = []
        orig = K.splice
        K.splice = lambda *a, **kw: (calls.append(1), orig(*a, **kw))[1]
        try:
            ll.zero_grad(set_to_none=True)
            x = xb.clone().requires_grad_()
            plan = RunPlan.with_splices([(hook, Ix[None, None, :hw, hw:2 * hw], src)])
            with torch.autocast("cuda", dtype=torch.bfloat16):
                y = ll(x, plan=plan)
            y.float().logsumexp(-1).sum().backward()
        finally:
            K.splice = orig
            os.environ.pop("IIT_BN_SPLICE", None)
        outs.append((y.detach().float(), x.grad.clone(), {n: p.grad.clone() for n, p in ll.named_parameters()},
                     len(calls)))
    (y1, gx1, g1, c1), (y0, gx0, g0, c0) = outs
    assert c1 == 0 and c0 >= 2
    # the separate pass keeps the activation channels-last, so the same fused BatchNorm reads the spliced copy; the
    # per-channel statistics are fp32 atomic sums (order varies run to run, as MIOpen's), so the runs agree to bf16
    # rounding, not bitwise -- the gradient semantics are pinned by test_bn_splice_on_read_exact
    assert rel(y1, y0) < 2e-2


@pytest.mark.parametrize("res", [False, True])
@pytest.mark.parametrize("training", [True, False])
def test_bn_splice_on_read_exact(res, training):
    """bn_act with splice=(index, src) equals bn_act on the pre-spliced channels-last input bitwise (forward, running
    statistics, residual / weight / bias gradients); its input gradient equals the pre-spliced run's with the spliced
    elements zeroed."""
    from iit_amd.core.index import Ix
    from iit_amd.ops import bn as fbn
    torch.manual_seed(3)
    N, C, H = 16, 128, 11
    idx = Ix[None, 32:96, 3:9, :5]
    x0 = torch.randn(N, C, H, H, device=dev).bfloat16().contiguous(memory_format=torch.channels_last)
    src = torch.randn(N, C, H, H, device=dev).bfloat16()  # NCHW source: strided reads in the kernel
    r0 = torch.randn_like(x0, memory_format=torch.channels_last) if res else None
    g0 = torch.randn(N, C, H, H, device=dev).bfloat16().contiguous(memory_format=torch.channels_last)
    outs = []
    for pre in (False, True):
        bn = torch.nn.BatchNorm2d(C).to(dev).train(training)
        x = x0.clone()
        r = r0.clone() if res else None
        if pre:
            x = x.clone()
            x[idx.as_index] = src[idx.as_index]
        x.requires_grad_()
        if r is not None:
            r.requires_grad_()
        y = fbn.bn_act(x, bn, r, relu=True, splice=None if pre else (idx, src))
        y.backward(g0)
        outs.append((y.detach(), x.grad, r.grad if r is not None else None, bn.weight.grad, bn.bias.grad,
                     bn.running_mean.clone(), bn.running_var.clone()))
    (y1, dx1, dr1, dw1, db1, rm1, rv1), (y0, dx0, dr0, dw0, db0, rm0, rv0) = outs
    # equal up to the order of the fp32 atomic statistics sums (a last-bit difference can flip a bf16 rounding)
    close = lambda a, b: rel(a, b) < 2e-3  # noqa: E731
    assert close(y1, y0) and close(rm1, rm0) and close(rv1, rv0)
    assert close(dw1, dw0) and close(db1, db0)
    if res:
        assert close(dr1, dr0)
    assert int((dx1[idx.as_index] != 0).sum()) == 0  # the spliced elements carry no gradient
    exp = dx0.clone()
    exp[idx.as_index] = 0
    assert close(dx1, exp)


def test_resnet_conv_mirror_matches_autocast_path(monkeypatch):
    """resnet.Conv2d under bf16 autocast with its weight in a flat arena convolves with the arena's bf16 mirror
    (torch_ops._MirrorWeight) and adds the bf16 weight gradient into the fp32 slot.  Against the fp32 model, its
    logits and every parameter gradient are within the autocast cast path's own bf16 error (plus a small floor: the
    mirror holds the same bf16 rounding of the master, but the fused BN statistics' fp32 atomics make no two bf16
    runs bitwise equal), and every convolution took the mirror."""
    from iit_amd.engine.flat import FlatParams
    from iit_amd.models.resnet import resnet18
    from iit_amd.ops import torch_ops
    torch.manual_seed(3)
    ms = [resnet18(num_classes=10).to(dev).to(memory_format=torch.channels_last) for _ in range(3)]
    for m in ms[1:]:
        m.load_state_dict(ms[0].state_dict())
    for m in ms[:2]:
        FlatParams(m)
    x = torch.rand(32, 3, 84, 84, device=dev).contiguous(memory_format=torch.channels_last)
    t = torch.randint(0, 10, (32,), device=dev)
    from iit_amd.ops import conv as hconv
    calls = []
    orig = torch_ops._MirrorWeight.apply
    monkeypatch.setattr(torch_ops._MirrorWeight, "apply", lambda *a: calls.append(1) or orig(*a))
    # the 3x3 / stride-1 convolutions read the mirror through the implicit-GEMM op instead (ops/conv.py)
    orig_c = hconv.Conv3x3Fn.apply
    monkeypatch.setattr(hconv.Conv3x3Fn, "apply", lambda *a: calls.append(1) or orig_c(*a))
    outs = []
    for m, env, amp in ((ms[0], "1", True), (ms[1], "0", True), (ms[2], "0", False)):
        monkeypatch.setenv("IIT_CONV_MIRROR", env)
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=amp):
            y = m(x)
            loss = torch.nn.functional.cross_entropy(y.float(), t)
        loss.backward()
        outs.append(y.float().detach())
    assert len(calls) == 20  # every convolution of ResNet-18 took the mirror (model 0 only)
    ym, yc, yr = outs
    assert rel(ym, yr) <= 1.5 * rel(yc, yr) + 1e-2, (rel(ym, yr), rel(yc, yr))
    for (n, pm), (_, pc), (_, pr) in zip(*(m.named_parameters() for m in ms)):
        assert pm.grad is not None and pc.grad is not None, n
        em, ec = rel(pm.grad, pr.grad), rel(pc.grad, pr.grad)
        assert em <= 1.5 * ec + 2e-2, (n, em, ec)


@pytest.mark.parametrize("shape,ties", [((4, 64, 42, 42), False), ((2, 16, 9, 7), True), ((3, 8, 10, 11), True)])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_maxpool3s2_matches_torch(shape, ties, dtype):
    """The NHWC bf16 3x3/s2/p1 max pool (byte argmax, gather backward) against torch's max_pool2d on the same bf16
    input: outputs equal exactly, and the input gradient equals torch's (ties resolved to the first tap in scan order,
    as torch's kernel does; integer-valued inputs make ties common)."""
    from iit_amd.ops.bn import MaxPool3s2Fn
    torch.manual_seed(7)
    N, C, H, W = shape
    x = (torch.randint(-3, 4, shape, device=dev).float() if ties else torch.randn(shape, device=dev))
    x = x.to(dtype).contiguous(memory_format=torch.channels_last)
    g = torch.randn(N, C, (H - 1) // 2 + 1, (W - 1) // 2 + 1, device=dev).to(dtype)
    xa = x.clone().requires_grad_(True)
    ya = MaxPool3s2Fn.apply(xa)
    ya.backward(g)
    xb = x.clone().requires_grad_(True)
    yb = torch.nn.functional.max_pool2d(xb, 3, 2, 1)
    yb.backward(g)
    assert ya.is_contiguous(memory_format=torch.channels_last)
    assert torch.equal(ya, yb)
    assert rel(xa.grad, xb.grad) < (1e-2 if dtype == torch.bfloat16 else 1e-6), rel(xa.grad, xb.grad)
    # routing: the gradient lands on the same elements
    assert torch.equal(xa.grad != 0, xb.grad != 0)


@pytest.mark.parametrize("C,hw,N", [(64, 42, 256), (512, 3, 64)])
def test_bn_stats_large_mean_offset(C, hw, N):
    """the batch variance is formed from sums of x - p and (x - p)^2 around a per-channel pivot (the batch's
    first row) -- not E[x^2] - mean^2, which cancels when |mean| >> std.  fp32 activations with a per-channel mean of
    ~1000 and unit std: output and running variance against a float64 reference."""
    from iit_amd.ops import bn as fbn
    torch.manual_seed(3)
    bn = torch.nn.BatchNorm2d(C).to(dev)
    with torch.no_grad():
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.uniform_(-0.5, 0.5)
    bn.train(True)
    off = (torch.rand(C, device=dev) * 200 + 900)[None, :, None, None]
    x = (torch.randn(N, C, hw, hw, device=dev) * (torch.rand(C, device=dev)[None, :, None, None] + 0.5) + off)
    x = x.contiguous(memory_format=torch.channels_last)
    rv0 = bn.running_var.clone()
    y = fbn.bn_act(x, bn, None, relu=False)
    xd = x.double()
    mean = xd.mean((0, 2, 3))
    var = xd.var((0, 2, 3), unbiased=False)
    n = x.numel() // C
    ref = ((xd - mean[None, :, None, None]) * torch.rsqrt(var + bn.eps)[None, :, None, None]
           * bn.weight.double()[None, :, None, None] + bn.bias.double()[None, :, None, None])
    assert rel(y, ref) < 1e-4
    rv = 0.9 * rv0.double() + 0.1 * var * n / (n - 1)
    assert torch.allclose(bn.running_var.double(), rv, rtol=1e-4, atol=1e-6)



def test_bn_two_level_reduction_is_deterministic(monkeypatch):
    """Deterministic mode (IIT_DETERMINISTIC=1): the BatchNorm statistics take the fixed-order two-level reduction --
    forward + backward twice give bit-identical outputs, gradients and running statistics, equal to the atomic path
    within fp32 summation-order noise."""
    from iit_amd.ops import bn as fbn
    outs = []
    for mode in ("1", "1", "0"):
        monkeypatch.setenv("IIT_DETERMINISTIC", mode)
        torch.manual_seed(5)
        bn = torch.nn.BatchNorm2d(64).to(dev)
        x = torch.randn(256, 64, 21, 21, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        x.requires_grad_()
        y = fbn.bn_act(x, bn, None, relu=True)
        y.backward(torch.ones_like(y))
        outs.append((y.detach().clone(), x.grad.clone(), bn.weight.grad.clone(), bn.running_var.clone()))
    for a, b in zip(outs[0], outs[1]):
        assert torch.equal(a, b)
    for a, b in zip(outs[0], outs[2]):
        assert rel(a, b) < 1e-3
