"""Llama-family fused kernels (csrc/llama_ops.hip) vs plain fp32 PyTorch: RMSNorm (+ weight gradient),
rotary embedding (NeoX halves and adjacent pairs, partial rotary_dim, strided input), SwiGLU."""
import pytest
import torch

pytestmark = pytest.mark.gpu

dev = "cuda"


def rel(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


@pytest.mark.parametrize("d", [64, 520, 4096])
@pytest.mark.parametrize("x_dtype", [torch.bfloat16, torch.float32])
def test_rmsnorm_fwd_bwd(d, x_dtype):
    from iit_amd.ops import hip_ops
    torch.manual_seed(d)
    x = torch.randn(3, 37, d, device=dev).to(x_dtype).requires_grad_()
    w = (1 + 0.1 * torch.randn(d, device=dev)).requires_grad_()
    y = hip_ops.RMSNormFn.apply(x, w, 1e-5)
    xr = x.detach().float().requires_grad_()
    wr = w.detach().clone().requires_grad_()
    yr = xr * torch.rsqrt(xr.pow(2).mean(-1, keepdim=True) + 1e-5) * wr
    assert y.dtype == torch.bfloat16 and rel(y, yr) < 1e-2
    g = torch.randn_like(yr)
    y.backward(g.bfloat16())
    yr.backward(g)
    assert x.grad.dtype == x_dtype
    assert rel(x.grad, xr.grad) < 2e-2
    assert rel(w.grad, wr.grad) < 2e-2


@pytest.mark.parametrize("adjacent", [False, True])
@pytest.mark.parametrize("rd", [128, 64, 24])  # 24: the per-pair kernel (NeoX halves need rd % 16 == 0)
def test_rotary_matches_torch_ops(adjacent, rd):
    from iit_amd.ops import hip_ops
    from iit_amd.ops.torch_ops import TorchOps
    from iit_amd.models.config import HookedTransformerConfig
    from iit_amd.models.transformer import rotary_tables
    cfg = HookedTransformerConfig.from_dict(dict(n_layers=1, d_model=256, n_heads=2, d_head=128, n_ctx=64,
                                                 d_vocab=16, act_fn="silu", rotary_dim=rd, rotary_adjacent_pairs=adjacent,
                                                 positional_embedding_type="rotary"))
    sin, cos = (t.to(dev) for t in rotary_tables(cfg))
    torch.manual_seed(0)
    packed = torch.randn(2, 20, 3, 4, 128, device=dev).bfloat16()
    x = packed[:, :, 1].detach().requires_grad_()  # strided view, as q/k of a packed QKV projection
    assert not x.is_contiguous()
    y = hip_ops.RotaryFn.apply(x, cos, sin, rd, 3, adjacent)
    ops = TorchOps(torch.float32)
    xr = x.detach().float().requires_grad_()
    yr = TorchOps.rotary(ops, xr, cos, sin, rd, adjacent, offset=3)
    assert rel(y, yr) < 1e-2
    g = torch.randn_like(yr)
    y.backward(g.bfloat16())
    yr.backward(g)
    assert rel(x.grad, xr.grad) < 1e-2


def test_swiglu_fwd_bwd():
    from iit_amd.ops import hip_ops
    torch.manual_seed(0)
    gate = torch.randn(5, 7, 344, device=dev).bfloat16().requires_grad_()
    up = torch.randn(5, 7, 344, device=dev).bfloat16().requires_grad_()
    post = hip_ops.SwiGLUFn.apply(gate, up)
    gr, ur = (t.detach().float().requires_grad_() for t in (gate, up))
    pr = torch.nn.functional.silu(gr) * ur
    assert rel(post, pr) < 1e-2
    g = torch.randn_like(pr)
    post.backward(g.bfloat16())
    pr.backward(g)
    assert rel(gate.grad, gr.grad) < 2e-2 and rel(up.grad, ur.grad) < 2e-2


@pytest.mark.parametrize("x_dtype", [torch.bfloat16, torch.float32])
def test_rmsnorm_fork_adds_skip_gradient(x_dtype):
    """RMSNormForkFn: (RMSNorm(x), x) whose backward sums the norm gradient and the skip-connection gradient in
    the kernel -- equal to RMSNormFn + autograd's add."""
    from iit_amd.ops import hip_ops
    torch.manual_seed(3)
    d = 512
    x = torch.randn(4, 9, d, device=dev).to(x_dtype).requires_grad_()
    w = (1 + 0.1 * torch.randn(d, device=dev)).requires_grad_()
    y, xp = hip_ops.RMSNormForkFn.apply(x, w, 1e-5)
    g1, g2 = torch.randn(4, 9, d, device=dev), torch.randn(4, 9, d, device=dev)
    (y.float() * g1).sum().add((xp.float() * g2).sum()).backward()
    x2 = x.detach().clone().requires_grad_()
    w2 = w.detach().clone().requires_grad_()
    y2 = hip_ops.RMSNormFn.apply(x2, w2, 1e-5)
    (y2.float() * g1).sum().add((x2.float() * g2).sum()).backward()
    assert torch.equal(y, y2)
    assert rel(x.grad, x2.grad) < 1e-2 and rel(w.grad, w2.grad) < 1e-3


def test_llama_torch_backend_residual_epilogue_matches_unfused(monkeypatch):
    """Llama (torch op backend, bf16 arena mirror): W_O / W_out with the residual add in the GEMM epilogue
    (hipBLASLt beta = 1) and the RMSNorm fork give the unfused path's logits and gradients."""
    import copy
    from iit_amd.engine.flat import FlatParams
    from iit_amd.models.convert import llama_config_dict
    from iit_amd.models.transformer import HookedTransformer
    cfg = llama_config_dict("llama-tiny", device=dev, dtype=torch.bfloat16)
    torch.manual_seed(0)
    a = HookedTransformer(cfg)
    b = copy.deepcopy(a)
    FlatParams(a, with_bf16_shadow=True)
    FlatParams(b, with_bf16_shadow=True)
    tok = torch.randint(0, cfg["d_vocab"], (4, 24), device=dev)
    outs, grads = [], []
    for model, fused in ((a, "1"), (b, "0")):
        monkeypatch.setenv("IIT_TORCH_RESID_EPI", fused)
        monkeypatch.setenv("IIT_RMS_FORK", fused)
        monkeypatch.setenv("IIT_LLAMA_FUSED", "1")
        out = model(tok)
        out.float().pow(2).mean().backward()
        outs.append(out.detach().float())
        grads.append({n: p.grad.detach().float().clone() for n, p in model.named_parameters() if p.grad is not None})
    assert rel(outs[0], outs[1]) < 1e-2
    assert grads[0].keys() == grads[1].keys()
    for n in grads[1]:
        if grads[1][n].norm() > 1e-6:
            assert rel(grads[0][n], grads[1][n]) < 3e-2, n


def test_llama_torch_backend_matches_fp32_oracle():
    """Llama (torch op backend on the bf16 arena mirror: packed QKV GEMM with the one-launch q/k/v gradient split,
    rotary / RMSNorm / SwiGLU kernels, flash attention, dispatcher weight gradients) vs the same model in fp32 torch
    ops: logits and every parameter gradient."""
    import copy
    from iit_amd.engine.flat import FlatParams
    from iit_amd.models.convert import llama_config_dict
    from iit_amd.models.transformer import HookedTransformer
    cfg = llama_config_dict("llama-tiny", device=dev, dtype=torch.bfloat16)
    torch.manual_seed(0)
    a = HookedTransformer(cfg)
    ref = copy.deepcopy(a)
    ref.cfg.dtype = torch.float32
    FlatParams(a, with_bf16_shadow=True)
    tok = torch.randint(0, cfg["d_vocab"], (4, 40), device=dev)
    out = a(tok)
    out.float().pow(2).mean().backward()
    ref.set_op_backend("torch")
    oref = ref(tok)
    oref.float().pow(2).mean().backward()
    assert rel(out, oref) < 2e-2
    ga = {n: p.grad for n, p in a.named_parameters() if p.grad is not None}
    gr = {n: p.grad for n, p in ref.named_parameters() if p.grad is not None}
    assert ga.keys() == gr.keys() and any("W_Q" in n for n in ga)
    for n in gr:
        if gr[n].norm() > 1e-6:
            assert rel(ga[n], gr[n]) < 5e-2, n


@pytest.mark.parametrize("index_kind", ["last_half", "positions"])
def test_swiglu_splice_in_kernel_matches_separate_pass(monkeypatch, index_kind):
    """A ``mlp.hook_post`` splice applied inside the SwiGLU kernel (the producer) gives the separate patch-spec pass's
    output and gradients exactly (forward: selected elements = source; backward: their gate / up gradients zero)."""
    import copy
    from iit_amd.core.index import Ix
    from iit_amd.engine.flat import FlatParams
    from iit_amd.engine.plan import RunPlan
    from iit_amd.models.convert import llama_config_dict
    from iit_amd.models.transformer import HookedTransformer
    cfg = llama_config_dict("llama-tiny", device=dev, dtype=torch.bfloat16)
    torch.manual_seed(1)
    a = HookedTransformer(cfg)
    b = copy.deepcopy(a)
    FlatParams(a, with_bf16_shadow=True)
    FlatParams(b, with_bf16_shadow=True)
    tok = torch.randint(0, cfg["d_vocab"], (4, 24), device=dev)
    src_tok = torch.randint(0, cfg["d_vocab"], (4, 24), device=dev)
    name = "blocks.1.mlp.hook_post"
    dm = cfg["d_mlp"]
    idx = Ix[:, -1, :dm // 2] if index_kind == "last_half" else Ix[:, [2, 5, 6]]
    outs, grads = [], []
    for model, fused in ((a, "1"), (b, "0")):
        monkeypatch.setenv("IIT_SWIGLU_SPLICE", fused)
        with torch.no_grad():
            src = model.run_capture(src_tok, [name])[name]
        out = model(tok, plan=RunPlan.with_splices([(name, idx, src)]))
        out.float().pow(2).mean().backward()
        outs.append(out.detach().float())
        grads.append({n: p.grad.detach().float().clone() for n, p in model.named_parameters() if p.grad is not None})
    assert torch.equal(outs[0], outs[1])
    for n in grads[1]:
        assert torch.allclose(grads[0][n], grads[1][n], rtol=1e-3, atol=1e-6), n


@pytest.mark.parametrize("index_kind", ["position", "features"])
def test_embed_splice_in_gather_matches_separate_pass(monkeypatch, index_kind):
    """A ``hook_embed`` splice applied inside the embedding gather (``csrc/llama_ops.hip`` embed_splice_*) gives the
    separate patch-spec pass's output and gradients (forward: selected elements = source, exactly; backward: no W_E
    gradient from the selected elements), and the fused path is the one that ran."""
    import copy
    from iit_amd.core.index import Ix
    from iit_amd.engine.flat import FlatParams
    from iit_amd.engine.plan import RunPlan
    from iit_amd.models.convert import llama_config_dict
    from iit_amd.models.transformer import HookedTransformer
    from iit_amd.ops import hip_ops
    cfg = llama_config_dict("llama-tiny", device=dev, dtype=torch.bfloat16)
    torch.manual_seed(2)
    a = HookedTransformer(cfg)
    b = copy.deepcopy(a)
    FlatParams(a, with_bf16_shadow=True)
    FlatParams(b, with_bf16_shadow=True)
    tok = torch.randint(0, cfg["d_vocab"], (4, 24), device=dev)
    src_tok = torch.randint(0, cfg["d_vocab"], (4, 24), device=dev)
    name = "hook_embed"
    d = cfg["d_model"]
    idx = Ix[:, 3] if index_kind == "position" else Ix[:, [1, 7], : d // 2]
    calls = []
    orig = hip_ops.EmbedSpliceFn.apply
    monkeypatch.setattr(hip_ops.EmbedSpliceFn, "apply", lambda *a_: calls.append(1) or orig(*a_))
    outs, grads = [], []
    for model, fused in ((a, "1"), (b, "0")):
        monkeypatch.setenv("IIT_EMBED_SPLICE", fused)
        with torch.no_grad():
            src = model.run_capture(src_tok, [name])[name]
        out = model(tok, plan=RunPlan.with_splices([(name, idx, src)]))
        out.float().pow(2).mean().backward()
        outs.append(out.detach().float())
        grads.append({n: p.grad.detach().float().clone() for n, p in model.named_parameters() if p.grad is not None})
    assert len(calls) == 1  # the fused gather ran for model a only
    assert torch.equal(outs[0], outs[1])
    assert "embed.W_E" in grads[1]
    for n in grads[1]:
        assert torch.allclose(grads[0][n], grads[1][n], rtol=1e-3, atol=1e-6), n
    # the spliced elements take no gradient: a source token's W_E row gets none from a fully spliced position
    if index_kind == "position":
        only = set(tok[:, 3].tolist()) - set(tok[:, [i for i in range(24) if i != 3]].flatten().tolist())
        for t in only:
            assert float(grads[0]["embed.W_E"][t].abs().max()) == 0.0


@pytest.mark.parametrize("sites_kind", ["z_and_post", "embed", "post_last"])
def test_llama_paired_forward_matches_two_forwards(monkeypatch, sites_kind):
    """the paired source + base forward on the torch op backend (ops/torch_pairs.py: RMSNorm,
    packed QKV, rotary, GQA flash attention, SwiGLU, residual adds over 2B rows, row-restricted backwards) against the
    reference's two forwards (source run under no_grad, base run with the source activations spliced in): the same
    intervened logits, the same captured source activations and the same parameter gradients; and both against the
    fp32 torch-op oracle of the same two forwards."""
    import copy
    from iit_amd.core.index import Ix
    from iit_amd.engine.flat import FlatParams
    from iit_amd.engine.plan import RunPlan
    from iit_amd.models.convert import llama_config_dict
    from iit_amd.models.transformer import HookedTransformer
    from iit_amd.ops import torch_pairs
    # flash-attention head size (64) and an 8-aligned MLP width: the shapes the paired kernels cover
    cfg = llama_config_dict("llama-tiny", device=dev, dtype=torch.bfloat16, d_model=256, d_head=64, rotary_dim=64,
                            d_mlp=192)
    torch.manual_seed(3)
    a = HookedTransformer(cfg)
    b = copy.deepcopy(a)
    ref = copy.deepcopy(a)
    ref.cfg.dtype = torch.float32
    ref.set_op_backend("torch")
    FlatParams(a, with_bf16_shadow=True)
    FlatParams(b, with_bf16_shadow=True)
    H, dm, n = cfg["n_heads"], cfg["d_mlp"], cfg["n_layers"]
    tok = torch.randint(0, cfg["d_vocab"], (4, 24), device=dev)
    src_tok = torch.randint(0, cfg["d_vocab"], (4, 24), device=dev)
    if sites_kind == "z_and_post":
        sites = {"blocks.0.attn.hook_z": [Ix[:, -1, :H // 2, :]], "blocks.1.mlp.hook_post": [Ix[:, -1, :dm // 2]]}
    elif sites_kind == "embed":
        sites = {"hook_embed": [Ix[:, 3]]}
    else:
        sites = {f"blocks.{n - 1}.mlp.hook_post": [Ix[:, -1]]}
    calls = []
    orig = torch_pairs.RMSNormPairFn.apply
    monkeypatch.setattr(torch_pairs.RMSNormPairFn, "apply", lambda *a_: calls.append(1) or orig(*a_))
    monkeypatch.setenv("IIT_PAIRED_TORCH", "1")  # (opt-in: measured slower at Llama-3-8B scale)
    res = a.run_paired(tok, src_tok, sites, logits="full")
    assert res is not None, "the torch-backend paired forward did not engage"
    out_p, caps = res
    assert calls or sites_kind == "embed"
    out_p.float().pow(2).mean().backward()

    def two_forwards(model):
        with torch.no_grad():
            cache = model.run_capture(src_tok, list(sites))
        spl = [(nm, ix, cache[nm]) for nm, ixs in sites.items() for ix in ixs]
        out = model(tok, plan=RunPlan.with_splices(spl))
        out.float().pow(2).mean().backward()
        return out, cache

    out_u, cache_u = two_forwards(b)
    out_r, cache_r = two_forwards(ref)
    for nm in sites:
        assert rel(caps[nm], cache_u[nm]) < 1e-2, nm
    assert rel(out_p, out_u) < 1e-2
    assert rel(out_p, out_r) <= 1.25 * rel(out_u, out_r) + 5e-3
    ga = {nm: p.grad for nm, p in a.named_parameters() if p.grad is not None}
    gb = {nm: p.grad for nm, p in b.named_parameters() if p.grad is not None}
    gr = {nm: p.grad for nm, p in ref.named_parameters() if p.grad is not None}
    assert ga.keys() == gb.keys()
    for nm in gb:
        if gb[nm].norm() > 1e-6:
            assert rel(ga[nm], gb[nm]) < 3e-2, nm
            assert rel(ga[nm], gr[nm]) <= 1.25 * rel(gb[nm], gr[nm]) + 5e-3, nm
