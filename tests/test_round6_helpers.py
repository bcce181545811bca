"""CPU checks of round-6 host-side logic: the conv geometry filter (ops/conv.py), the dual-pair prefetch registry
(ops/hip_ops.py: each pair prefetches the operands of the pair that runs right after it in the backward, i.e. the
previous registration in forward order) and the prefetch argument packing (ops/hip_kernels.py)."""
import torch


def test_conv_geometry_filter(monkeypatch):
    from iit_amd.ops import conv as hconv
    monkeypatch.setattr(hconv, "GEOMS", {"k3s1", "k3s2", "k1s1", "k1s2"})
    C = torch.nn.Conv2d
    assert hconv.geometry(C(64, 64, 3, 1, 1, bias=False)) == (3, 1, 1)
    assert hconv.geometry(C(64, 128, 3, 2, 1, bias=False)) == (3, 2, 1)
    assert hconv.geometry(C(64, 128, 1, 2, 0, bias=False)) == (1, 2, 0)
    assert hconv.geometry(C(3, 64, 7, 2, 3, bias=False)) is None  # the stem
    assert hconv.geometry(C(64, 64, 3, 1, 1, bias=True)) is None
    assert hconv.geometry(C(64, 64, 3, 1, 2, bias=False)) is None  # padding other than k // 2
    assert hconv.geometry(C(64, 64, 3, 1, 1, bias=False, groups=2)) is None
    assert hconv.geometry(C(64, 64, 3, 1, 1, bias=False, dilation=2)) is None
    monkeypatch.setattr(hconv, "GEOMS", {"k3s1", "k1s2"})  # the default: 3 x 3 stride 2 opt-in
    assert hconv.geometry(C(64, 128, 3, 2, 1, bias=False)) is None
    assert hconv.geometry(C(64, 128, 1, 2, 0, bias=False)) == (1, 2, 0)
    for H, k, s, p in ((21, 3, 2, 1), (84, 7, 2, 3), (11, 1, 2, 0), (6, 3, 1, 1)):
        ref = C(1, 1, k, s, p)(torch.zeros(1, 1, H, H)).shape[-1]
        assert hconv._out_hw(H, H, k, s, p) == (ref, ref)
    x = torch.zeros(2, 64, 8, 8).contiguous(memory_format=torch.channels_last)
    assert not hconv.covered(x, C(64, 64, 3, 1, 1, bias=False))  # CPU tensors never take the HIP kernels


class _Ctx:
    def __init__(self, grad=True):
        self.needs_input_grad = (grad, False)


def test_dual_prefetch_registry_order(monkeypatch):
    from iit_amd.ops import hip_ops
    monkeypatch.setattr(hip_ops, "_PF_ON", [True])
    hip_ops._PF_SEQ.clear()
    ctxs = [_Ctx() for _ in range(4)]
    ops = [(torch.zeros(1), torch.zeros(2)) for _ in range(4)]  # (X, W) of QKV, W_O, W_in, W_out in forward order
    nograd = _Ctx(False)
    for c, (x, w) in zip(ctxs, ops):
        hip_ops._pf_register(c, x, w)
    hip_ops._pf_register(nograd, torch.zeros(3), torch.zeros(3))  # a no-grad (source-only) op never registers
    assert not hasattr(nograd, "pf_idx") and len(hip_ops._PF_SEQ) == 4
    # backward runs W_out, W_in, W_O, QKV: each prefetches the one that runs after it
    assert hip_ops._pf_next(ctxs[3])[0] is ops[2][0] and hip_ops._pf_next(ctxs[3])[1] is ops[2][1]
    assert hip_ops._pf_next(ctxs[1])[0] is ops[0][0]
    assert hip_ops._pf_next(ctxs[0]) is None  # the last pair of the backward has nothing after it
    hip_ops._PF_SEQ.clear()  # (begin_forward) a stale index finds nothing
    assert hip_ops._pf_next(ctxs[3]) is None
    hip_ops._PF_ON[0] = False  # a model whose policy is off (the encoder) registers nothing
    c = _Ctx()
    hip_ops._pf_register(c, torch.zeros(1), torch.zeros(1))
    assert not hasattr(c, "pf_idx") and not hip_ops._PF_SEQ


def test_prefetch_args_packing():
    from iit_amd.ops import hip_kernels as K
    assert K._prefetch_args(None) == (None, 0, None, 0, 0)
    assert K._prefetch_args((torch.zeros(4),)) == (None, 0, None, 0, 0)  # host tensors are never prefetched


def test_torch_ops_bf16_emulation(monkeypatch):
    """IIT_EMULATE_BF16 (precision study): "w" rounds weights to bf16 with a straight-through gradient, "act" rounds
    op outputs to bf16; an fp32 backend without it is unchanged."""
    from iit_amd.ops.torch_ops import TorchOps
    torch.manual_seed(0)
    x = torch.randn(4, 8)
    W = torch.randn(8, 5, requires_grad=True)
    ref = TorchOps(torch.float32).lin(x, W)
    assert torch.equal(ref, x @ W)
    monkeypatch.setenv("IIT_EMULATE_BF16", "w")
    y = TorchOps(torch.float32).lin(x, W)
    assert torch.equal(y, x @ W.detach().bfloat16().float())
    y.sum().backward()
    assert torch.allclose(W.grad, x.sum(0)[:, None].expand(8, 5))
    monkeypatch.setenv("IIT_EMULATE_BF16", "act")
    ops = TorchOps(torch.float32)
    z = ops.layer_norm(torch.randn(3, 16), None, None, 1e-5)
    assert torch.equal(z, z.bfloat16().float())
    q, k, v = (torch.randn(2, 5, 2, 4) for _ in range(3))
    out = ops.attention(q, k, v, True, 2.0)
    assert torch.equal(out, out.bfloat16().float())
    monkeypatch.setenv("IIT_EMULATE_BF16", "w,act")
    assert TorchOps(torch.bfloat16).emu_w is False  # only an fp32 backend emulates
