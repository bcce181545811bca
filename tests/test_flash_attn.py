"""Tiled (flash-style) MFMA attention (csrc/flash_attn.hip) vs a plain fp32 PyTorch reference.

Covers forward + backward for causal and bidirectional attention, head dims 64 / 128, grouped-query heads,
sequence lengths that are not multiples of the 64-row tile, strided (packed-qkv) inputs and the
interchange-splice head mask.  SURVEY.md §2.3 K04 / §7.3 kernel 3 ("attention_tiled" for long S).
"""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu

dev = "cuda"


def ref_attention(q, k, v, causal, scale):
    """fp32 reference on the bf16-rounded inputs; k/v expanded for GQA."""
    q, k, v = (t.float() for t in (q, k, v))
    rep = q.shape[2] // k.shape[2]
    k = k.repeat_interleave(rep, dim=2)
    v = v.repeat_interleave(rep, dim=2)
    s = torch.einsum("bqhd,bkhd->bhqk", q, k) * scale
    if causal:
        S = q.shape[1]
        s = s.masked_fill(~torch.ones(S, S, dtype=torch.bool, device=q.device).tril(), float("-inf"))
    return torch.einsum("bhqk,bkhd->bqhd", s.softmax(-1), v)


def rel(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


@pytest.mark.parametrize("S", [17, 64, 100, 257])
@pytest.mark.parametrize("dh", [64, 128])
@pytest.mark.parametrize("causal", [True, False])
@pytest.mark.parametrize("hkv", [4, 1])
def test_flash_forward_backward_matches_fp32(S, dh, causal, hkv):
    from iit_amd.ops import hip_ops
    torch.manual_seed(S + dh + hkv)
    B, Hq = 2, 4
    q = torch.randn(B, S, Hq, dh, device=dev).bfloat16().requires_grad_()
    k = torch.randn(B, S, hkv, dh, device=dev).bfloat16().requires_grad_()
    v = torch.randn(B, S, hkv, dh, device=dev).bfloat16().requires_grad_()
    attn_scale = math.sqrt(dh)
    z = hip_ops.flash_attention(q, k, v, causal, attn_scale)
    qr, kr, vr = (t.detach().float().requires_grad_() for t in (q, k, v))
    zr = ref_attention(qr, kr, vr, causal, 1.0 / attn_scale)
    assert rel(z, zr) < 1e-2
    g = torch.randn_like(zr)
    z.backward(g.bfloat16())
    zr.backward(g)
    for name, a, b in (("dq", q.grad, qr.grad), ("dk", k.grad, kr.grad), ("dv", v.grad, vr.grad)):
        assert rel(a, b) < 2e-2, name


def test_flash_packed_qkv_with_head_splice():
    """HipOps.attention on a packed [B,S,3,H,dh] buffer: spliced heads copy the source and get no gradient."""
    from iit_amd.ops import hip_ops
    torch.manual_seed(0)
    B, S, H, dh = 3, 80, 4, 64
    packed = torch.randn(B, S, 3, H, dh, device=dev).bfloat16().requires_grad_()
    src = torch.randn(B, S, H, dh, device=dev).bfloat16()
    heads = [1, 3]
    z = hip_ops.FlashPackedFn.apply(packed, src, (1 << 1) | (1 << 3), True, 1.0 / math.sqrt(dh))
    pr = packed.detach().float().requires_grad_()
    zr = ref_attention(pr[:, :, 0], pr[:, :, 1], pr[:, :, 2], True, 1.0 / math.sqrt(dh)).clone()
    zr[:, :, heads] = src[:, :, heads].float()
    assert rel(z, zr) < 1e-2
    assert torch.equal(z[:, :, heads], src[:, :, heads])
    g = torch.randn_like(zr)
    z.backward(g.bfloat16())
    zr.backward(g)
    assert rel(packed.grad, pr.grad) < 2e-2
    assert packed.grad[:, :, :, heads].abs().max().item() == 0.0


def test_long_context_gpt2_hip_backend_matches_torch_backend():
    """A GPT-2-architecture model at S=192 (> the short-sequence kernels' 64) on the HIP backend uses the tiled
    kernel; its loss and gradients match the torch op backend."""
    from iit_amd.models.config import gpt2_config_dict
    from iit_amd.models.transformer import HookedTransformer
    torch.manual_seed(0)
    cfg = gpt2_config_dict()
    cfg.update(n_layers=2, d_model=128, n_heads=2, d_head=64, d_mlp=256, d_vocab=512, d_vocab_out=512, n_ctx=256,
               device=dev, dtype=torch.bfloat16)
    a = HookedTransformer(cfg)
    b = HookedTransformer(cfg)
    b.load_state_dict(a.state_dict())
    a.set_op_backend("hip")
    b.set_op_backend("torch")
    x = torch.randint(0, 512, (2, 192), device=dev)
    la = a(x, return_type="loss")
    lb = b(x, return_type="loss")
    assert abs(la.item() - lb.item()) < 2e-2 * abs(lb.item())
    la.backward()
    lb.backward()
    ga, gb = a.blocks[0].attn.W_Q.grad, b.blocks[0].attn.W_Q.grad
    assert rel(ga, gb) < 5e-2


@pytest.mark.parametrize("which", ["positions_heads", "dims", "batch_pos", "broadcast_src"])
def test_flash_general_splice_in_store_equals_splice_pass(which):
    """flash_attention_spliced (the splice applied by the kernel's output store, dO masked at every backward load)
    equals flash_attention followed by the separate splice pass (SpliceFn) -- forward bitwise, q/k/v gradients
    bitwise -- for patch-spec indices the head mask cannot express."""
    from iit_amd.core.index import Ix
    from iit_amd.ops import hip_ops
    from iit_amd.ops import splice as sp
    torch.manual_seed(7)
    B, S, Hq, Hkv, dh = 3, 130, 8, 2, 128
    idx = {"positions_heads": Ix[None, 5:70, [1, 6], None], "dims": Ix[None, None, 3, 16:80],
           "batch_pos": Ix[[0, 2], -1, None, None], "broadcast_src": Ix[None, 10:20, 2:4, None]}[which]
    q = torch.randn(B, S, Hq, dh, device=dev).bfloat16().requires_grad_()
    k = torch.randn(B, S, Hkv, dh, device=dev).bfloat16().requires_grad_()
    v = torch.randn(B, S, Hkv, dh, device=dev).bfloat16().requires_grad_()
    src = torch.randn(B, S, Hq, dh, device=dev).bfloat16()
    if which == "broadcast_src":
        src = src[:1]  # broadcast over the batch (stride 0)
    z = hip_ops.flash_attention_spliced(q, k, v, True, math.sqrt(dh), idx, src)
    assert z is not None
    q2, k2, v2 = (t.detach().clone().requires_grad_() for t in (q, k, v))
    zr = sp.splice(hip_ops.flash_attention(q2, k2, v2, True, math.sqrt(dh)), idx, src)
    assert torch.equal(z, zr)
    g = torch.randn(B, S, Hq, dh, device=dev).bfloat16()
    z.backward(g)
    zr.backward(g)
    for a, b in ((q.grad, q2.grad), (k.grad, k2.grad), (v.grad, v2.grad)):
        assert torch.equal(a, b)


def test_llama_hook_z_splice_runs_in_the_flash_store():
    """A rotary / GQA / RMS model on the torch op backend (the Llama path) with a hook_z splice at S > 16: no
    splice_kernel launch, same output and gradients as IIT_FLASH_SPLICE=0 (the separate splice pass)."""
    import os
    from iit_amd.core.index import Ix
    from iit_amd.engine.plan import RunPlan
    from iit_amd.models.transformer import HookedTransformer
    from iit_amd.ops import hip_kernels as K
    torch.manual_seed(0)
    cfg = dict(n_layers=2, d_model=256, n_heads=4, n_key_value_heads=2, d_head=64, d_mlp=512, d_vocab=300, n_ctx=64,
               act_fn="silu", gated_mlp=True, normalization_type="RMS", positional_embedding_type="rotary",
               rotary_dim=64, final_rms=True, attention_dir="causal", device=dev, dtype=torch.bfloat16, seed=0)
    m = HookedTransformer(cfg).set_op_backend("torch")
    x = torch.randint(0, 300, (2, 48), device=dev)
    name = "blocks.1.attn.hook_z"
    src = m.run_capture(torch.randint(0, 300, (2, 48), device=dev), [name])[name]
    outs = []
    for env in ("1", "0"):
        os.environ["IIT_FLASH_SPLICE"] = env
        try:
            m.zero_grad(set_to_none=True)
            calls = []
            orig = K.splice
            K.splice = lambda *a, **kw: (calls.append(1), orig(*a, **kw))[1]
            try:
                plan = RunPlan.with_splices([(name, Ix[None, 10:40, 1, None], src)])
                y = m(x, plan=plan).float()
                y.logsumexp(-1).mean().backward()
            finally:
                K.splice = orig
            outs.append((y.detach(), m.blocks[0].attn.W_Q.grad.clone(), len(calls)))
        finally:
            os.environ.pop("IIT_FLASH_SPLICE", None)
    (y1, g1, c1), (y0, g0, c0) = outs
    assert c1 == 0 and c0 >= 2  # forward splice + backward gradient mask as separate passes only with the switch off
    assert torch.equal(y1, y0)
    assert torch.equal(g1, g0)
