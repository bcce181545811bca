"""P1: TL-compatible hooks + native transformer (CPU oracle path) and node_picker (tests/test_node_picker.py)."""
import torch

from iit_amd.core.index import Ix
from iit_amd.core.nodes import HLNode, LLNode
from iit_amd.engine.plan import RunPlan
from iit_amd.models.transformer import HookedTransformer
from iit_amd.utils import node_picker


def tiny(**kw):
    cfg = dict(n_layers=2, n_heads=4, d_model=8, d_head=2, d_mlp=16, n_ctx=16, act_fn="gelu", d_vocab=21, device="cpu")
    cfg.update(kw)
    torch.manual_seed(0)
    return HookedTransformer(cfg)


def test_get_all_nodes():
    model = tiny()
    assert node_picker.get_all_nodes(model) == [
        LLNode("blocks.0.attn.hook_result", Ix[:, :, 0, :]), LLNode("blocks.0.attn.hook_result", Ix[:, :, 1, :]),
        LLNode("blocks.0.attn.hook_result", Ix[:, :, 2, :]), LLNode("blocks.0.attn.hook_result", Ix[:, :, 3, :]),
        LLNode("blocks.0.mlp.hook_post", Ix[[None]]),
        LLNode("blocks.1.attn.hook_result", Ix[:, :, 0, :]), LLNode("blocks.1.attn.hook_result", Ix[:, :, 1, :]),
        LLNode("blocks.1.attn.hook_result", Ix[:, :, 2, :]), LLNode("blocks.1.attn.hook_result", Ix[:, :, 3, :]),
        LLNode("blocks.1.mlp.hook_post", Ix[[None]]),
    ]


def test_get_params_in_circuit():
    ll = tiny(n_heads=4, d_head=3, d_model=12, act_fn="relu", d_vocab=6, n_ctx=5)
    corr = {"blocks.0.mlp.hook_post": {LLNode("blocks.0.mlp.hook_post", Ix[[None]])},
            "blocks.1.attn.hook_result": {LLNode("blocks.1.attn.hook_result", Ix[:, :, :2, :])}}
    expect = [
        LLNode("blocks.0.mlp.W_in", Ix[[None]]), LLNode("blocks.0.mlp.b_in", Ix[[None]]),
        LLNode("blocks.0.mlp.W_out", Ix[[None]]), LLNode("blocks.0.mlp.b_out", Ix[[None]]),
        LLNode("blocks.1.attn.W_Q", Ix[:, :, :2]), LLNode("blocks.1.attn.W_K", Ix[:, :, :2]),
        LLNode("blocks.1.attn.W_V", Ix[:, :, :2]), LLNode("blocks.1.attn.W_O", Ix[:, :2, :]),
        LLNode("blocks.1.attn.b_Q", Ix[:, :2]), LLNode("blocks.1.attn.b_K", Ix[:, :2]),
        LLNode("blocks.1.attn.b_V", Ix[:, :2]), LLNode("blocks.1.attn.b_O", Ix[[None]]),
    ]
    assert node_picker.get_params_in_circuit(corr, ll) == expect
    corr["blocks.1.attn.hook_result"] = {LLNode("blocks.1.attn.hook_result", Ix[[None]])}
    assert node_picker.get_params_in_circuit(corr, ll) == [
        LLNode(n.name, Ix[[None]]) for n in expect]


def test_parameter_names_layouts_and_state_dict():
    m = tiny(normalization_type="LNPre")
    names = [n for n, _ in m.named_parameters()]
    assert names[:2] == ["embed.W_E", "pos_embed.W_pos"]
    assert names[2:14] == [f"blocks.0.attn.{k}" for k in ("W_Q", "W_K", "W_V", "W_O", "b_Q", "b_K", "b_V", "b_O")] + \
        [f"blocks.0.mlp.{k}" for k in ("W_in", "b_in", "W_out", "b_out")]
    p = dict(m.named_parameters())
    assert p["blocks.0.attn.W_Q"].shape == (4, 8, 2) and p["blocks.0.attn.W_O"].shape == (4, 2, 8)
    assert p["unembed.W_U"].shape == (8, 21)
    sd = m.state_dict()
    assert "blocks.0.attn.mask" in sd and "blocks.0.attn.IGNORE" in sd
    m2 = tiny(normalization_type="LNPre")
    m2.load_state_dict(sd)
    x = torch.randint(0, 21, (2, 5))
    assert torch.allclose(m(x), m2(x))


def test_hook_shapes_and_cache():
    m = tiny()
    x = torch.randint(0, 21, (3, 7))
    logits, cache = m.run_with_cache(x)
    assert logits.shape == (3, 7, 21)
    assert cache["blocks.0.attn.hook_z"].shape == (3, 7, 4, 2)
    assert cache["blocks.1.attn.hook_pattern"].shape == (3, 4, 7, 7)
    assert cache["blocks.1.mlp.hook_post"].shape == (3, 7, 16)
    assert cache["z", 0].shape == (3, 7, 4, 2)
    assert not cache["blocks.0.hook_resid_pre"].requires_grad


def test_run_with_hooks_and_reset():
    m = tiny()
    x = torch.randint(0, 21, (2, 5))
    base = m(x)
    seen = []
    out = m.run_with_hooks(x, fwd_hooks=[("blocks.0.attn.hook_z", lambda a, hook: (seen.append(hook.name), a * 0)[1])])
    assert seen == ["blocks.0.attn.hook_z"] and not torch.allclose(out, base)
    assert torch.allclose(m(x), base)  # hooks reset
    m.run_with_hooks(x, fwd_hooks=[("blocks.0.attn.hook_z", lambda a, hook: a * 0)], reset_hooks_end=False)
    assert not torch.allclose(m(x), base)  # persisted (Q7 semantics)
    m.reset_hooks()
    assert torch.allclose(m(x), base)


def test_backward_hooks():
    m = tiny()
    x = torch.randint(0, 21, (2, 5))
    got = []

    def bwd(g, hook):
        got.append(g.shape)
        return torch.zeros_like(g)

    with m.hooks(bwd_hooks=[("blocks.1.mlp.hook_post", bwd)]):
        m(x).sum().backward()
    assert got == [torch.Size([2, 5, 16])]
    assert m.blocks[1].mlp.W_in.grad.abs().max() == 0  # gradient zeroed at the hook


def test_plan_capture_truncates_and_splice_matches_hooks():
    m = tiny()
    src = torch.randint(0, 21, (2, 5))
    base = torch.randint(0, 21, (2, 5))
    cache = m.run_capture(src, ["blocks.0.attn.hook_z"])
    _, full = m.run_with_cache(src)
    assert torch.allclose(cache["blocks.0.attn.hook_z"], full["blocks.0.attn.hook_z"])
    for idx in (Ix[[None]], Ix[:, :, 1, :], Ix[:, 2:, :, :]):
        want = m.run_with_hooks(base, fwd_hooks=[("blocks.0.attn.hook_z", _hook(idx, full["blocks.0.attn.hook_z"]))])
        got = m(base, plan=RunPlan.with_splices([("blocks.0.attn.hook_z", idx, cache["blocks.0.attn.hook_z"])]))
        assert torch.allclose(want, got, atol=1e-6)


def _hook(idx, src):
    def f(act, hook):
        out = act.clone()
        out[idx.as_index] = src[idx.as_index]
        return out
    return f


def test_last_position_logits_and_argmax_cpu():
    m = tiny()
    x = torch.randint(0, 21, (3, 6))
    full = m(x)
    assert torch.allclose(m(x, plan=RunPlan(logits="last")), full[:, -1], atol=1e-6)
    assert torch.equal(m(x, plan=RunPlan(logits="argmax")), full.argmax(-1))


def test_last_position_final_block_exact_with_gradients():
    """With last-position logits the final block runs W_O / LN2 / MLP on position -1 only; losses and every
    parameter gradient equal the full-width forward's."""
    m = tiny()
    x = torch.randint(0, 21, (3, 6))
    src = torch.randint(0, 21, (3, 6))
    cache = m.run_capture(src, ["blocks.0.mlp.hook_post"])
    spl = [("blocks.0.mlp.hook_post", Ix[:, 2:4, :], cache["blocks.0.mlp.hook_post"])]
    grads = []
    for fast in (True, False):
        m.last_position_final_block = fast
        m.zero_grad(set_to_none=True)
        out = m(x, plan=RunPlan.with_splices(spl, logits="last"))
        assert out.shape == (3, 21)
        (out.square().sum() + out[:, 3].sum()).backward()
        grads.append({n: p.grad.clone() for n, p in m.named_parameters() if p.grad is not None})
    assert grads[0].keys() == grads[1].keys()
    for n in grads[0]:
        assert torch.allclose(grads[0][n], grads[1][n], atol=1e-5), n
    # a live site after attention in the final block keeps the full-width path
    last = str(len(m.blocks) - 1)
    plan = RunPlan.with_splices([(f"blocks.{last}.hook_resid_mid", Ix[:, 1:2, :],
                                  m.run_capture(src, [f"blocks.{last}.hook_resid_mid"])[f"blocks.{last}.hook_resid_mid"])],
                                logits="last")
    m.last_position_final_block = True
    a = m(x, plan=plan)
    m.last_position_final_block = False
    assert torch.allclose(a, m(x, plan=plan), atol=1e-6)
    del m.last_position_final_block


def test_attn_only_and_result_hooks():
    m = tiny(attn_only=True, use_attn_result=True)
    x = torch.randint(0, 21, (2, 5))
    _, cache = m.run_with_cache(x)
    assert cache["blocks.0.attn.hook_result"].shape == (2, 5, 4, 8)
    assert "blocks.0.mlp.hook_post" not in cache
    assert all("mlp" not in n.name for n in node_picker.get_all_nodes(m))
