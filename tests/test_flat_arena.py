"""Flat parameter arena in kernel layout (iit_amd/engine/flat.py) on CPU.

The arena re-binds every parameter as a (possibly strided) view: W_Q|W_K|W_V
interleaved into one [d][3HD] matrix, b_Q|b_K|b_V into [3][H][dh], W_U with padded
rows.  Public shapes, values, forward results, gradients and state_dict are unchanged.
"""
import pytest
import torch

from iit_amd.engine.flat import FlatParams
from iit_amd.models.transformer import HookedTransformer
from iit_amd.ops.optim import FusedAdam


def tiny(**kw):
    cfg = dict(n_layers=2, n_heads=3, d_model=12, d_head=4, d_mlp=24, n_ctx=16, act_fn="gelu_new", d_vocab=29,
               device="cpu", normalization_type="LNPre")
    cfg.update(kw)
    torch.manual_seed(0)
    return HookedTransformer(cfg)


def test_arena_layout_views_and_values():
    m = tiny()
    before = {k: v.detach().clone() for k, v in m.state_dict().items()}
    tok = torch.randint(0, 29, (3, 7))
    out_before = m(tok).detach()
    flat = FlatParams(m)
    H, d, dh = 3, 12, 4
    HD = H * dh
    for blk in m.blocks:
        a = blk.attn
        assert a.W_Q.shape == (H, d, dh) and a.W_Q.stride() == (dh, 3 * HD, 1)
        assert a.W_K.data_ptr() == a.W_Q.data_ptr() + HD * 4
        assert a.W_V.data_ptr() == a.W_Q.data_ptr() + 2 * HD * 4
        assert a.b_K.data_ptr() == a.b_Q.data_ptr() + HD * 4
        packed = flat.data[flat.offset_of(a.W_Q):flat.offset_of(a.W_Q) + 3 * d * HD].view(d, 3, H, dh)
        assert torch.equal(packed[:, 1].permute(1, 0, 2), a.W_K.detach())
    Vp = 32
    assert m.unembed.W_U.shape == (12, 29) and m.unembed.W_U.stride() == (Vp, 1)
    for k, v in m.state_dict().items():
        assert torch.equal(v, before[k]), k
    assert torch.allclose(m(tok), out_before, atol=1e-6)
    # slots never overlap and all params live in the arena
    ends = [(o, o + n) for o, n in flat.slots]
    for (s0, e0), (s1, e1) in zip(ends, ends[1:]):
        assert e0 <= s1
    assert all(flat.owns(p) for p in m.parameters())


def test_arena_grads_are_views_and_match_contiguous_model():
    m_ref = tiny()
    m = tiny()
    flat = FlatParams(m)
    tok = torch.randint(0, 29, (4, 9))
    m_ref(tok).pow(2).mean().backward()
    m(tok).pow(2).mean().backward()
    for (n, pr), (_, pf) in zip(m_ref.named_parameters(), m.named_parameters()):
        assert pf.grad.data_ptr() == flat.grad_view(pf).data_ptr(), n
        assert pf.grad.stride() == pf.stride(), n
        assert torch.allclose(pf.grad, pr.grad, atol=1e-6, rtol=1e-5), n
    flat.zero_grad()
    assert all(p.grad.abs().max() == 0 for p in m.parameters())


def test_arena_adam_matches_torch_adam_and_padding_stays_zero():
    m_ref = tiny()
    m = tiny()
    flat = FlatParams(m)
    opt = FusedAdam(flat, lr=1e-2, use_hip=False)
    opt_ref = torch.optim.Adam(m_ref.parameters(), lr=1e-2)
    for _ in range(3):
        tok = torch.randint(0, 29, (4, 9))
        opt.zero_grad()
        m(tok).pow(2).mean().backward()
        opt.step(clip_norm=1.0)
        opt_ref.zero_grad()
        m_ref(tok).pow(2).mean().backward()
        torch.nn.utils.clip_grad_norm_(m_ref.parameters(), 1.0)
        opt_ref.step()
    for (n, pr), (_, pf) in zip(m_ref.named_parameters(), m.named_parameters()):
        if n.endswith("b_K"):  # gradient is zero in exact arithmetic: Adam normalises rounding noise
            continue
        assert torch.allclose(pf, pr, atol=1e-5, rtol=1e-4), n
    W_U = m.unembed.W_U
    pad = flat.data[flat.offset_of(W_U):flat.offset_of(W_U) + 12 * 32].view(12, 32)[:, 29:]
    assert pad.abs().max() == 0


def test_arena_mirror_and_buckets():
    m = tiny()
    flat = FlatParams(m, with_bf16_shadow=True)
    for p in m.parameters():
        assert torch.equal(flat.shadow_view(p).float(), p.detach().to(torch.bfloat16).float())
    bks = flat.buckets(256)
    assert bks[0][1] == flat.numel and bks[-1][0] == 0
    starts = {o for o, _ in flat.slots}
    for s, e in bks:
        assert s in starts
    covered = sorted(bks)
    for (s0, e0), (s1, e1) in zip(covered, covered[1:]):
        assert e0 == s1


def test_frozen_attention_falls_back_to_contiguous():
    m = tiny()
    for blk in m.blocks:
        blk.attn.W_K.requires_grad_(False)
    FlatParams(m)
    a = m.blocks[0].attn
    assert a.W_Q.is_contiguous() and a.W_V.is_contiguous()


def test_row_restriction_span_table():
    """Span table covers the arena minus the dead embedding rows, in <= max_len4 float4 pieces."""
    m = torch.nn.ModuleDict({"emb": torch.nn.Embedding(100, 8), "lin": torch.nn.Linear(8, 3)})
    flat = FlatParams(m)
    full, nfull = flat.span_table(max_len4=16, restricted=False)
    assert int(full[:, 2].sum()) * 4 == flat.numel and nfull == full.shape[0]
    assert torch.equal(full[:, 0], full[:, 1])  # replicated optimizer: gradient / moments at the arena offset
    assert flat.restrict_rows(m["emb"].weight, torch.tensor([0, 1, 2, 50, 99, 99]))
    tab, n = flat.span_table(max_len4=16)
    covered = torch.zeros(flat.numel, dtype=torch.bool)
    for st, _loc, ln in tab.tolist():
        assert 0 < ln <= 16
        covered[st * 4:(st + ln) * 4] = True
    off = flat.offset_of(m["emb"].weight)
    live = torch.zeros(100, dtype=torch.bool)
    live[[0, 1, 2, 50, 99]] = True
    for r in range(100):
        assert bool(covered[off + r * 8:off + (r + 1) * 8].all()) == bool(live[r])
    rest = torch.ones(flat.numel, dtype=torch.bool)
    rest[off:off + 800] = False
    assert bool(covered[rest].all())
    assert flat.check_inactive_zero()
    flat.grad[off + 3 * 8] = 1.0
    assert not flat.check_inactive_zero()
    assert flat.restrict_rows(m["emb"].weight, None) and not flat.inactive_ranges()


def test_lazy_zero_grad_store_claims():
    """FlatParams.zero_grad leaves store-claimed slots to their producer (grad None, no memset); a claim on a
    live gradient accumulates; unclaimed None slots read as zero when consumed."""
    from iit_amd.engine.flat import FlatParams
    torch.manual_seed(0)
    m = torch.nn.Sequential(torch.nn.Linear(6, 5), torch.nn.Linear(5, 3))
    flat = FlatParams(m)
    W0, b0, W1, b1 = m[0].weight, m[0].bias, m[1].weight, m[1].bias
    flat.grad.fill_(7.0)  # stale values
    flat.zero_grad()  # nothing claimed yet: full memset
    assert float(flat.grad.abs().sum()) == 0.0 and W0.grad is not None
    assert not flat.claim(W1)  # live (zeroed) gradient: accumulate -- but W1 is now known to be store-produced
    flat.grad.fill_(7.0)
    flat.zero_grad()
    assert W1.grad is None and W0.grad is not None  # W1 lazily zeroed, W0 memset
    assert float(W0.grad.abs().sum()) == 0.0 and float(b1.grad.abs().sum()) == 0.0
    assert float(flat.grad_view(W1).abs().sum()) > 0  # its slot still holds stale values ...
    assert flat.claim(W1)  # ... which the producer overwrites (store)
    W1.grad.copy_(torch.ones_like(W1))
    assert torch.equal(flat.grad_view(W1), torch.ones_like(W1))
    # a claimed slot no producer wrote reads as zero once consumed
    flat.grad.fill_(7.0)
    flat.zero_grad()
    assert W1.grad is None
    flat.rebind_grads(zero_missing=True)
    assert float(W1.grad.abs().sum()) == 0.0


@pytest.mark.gpu
def test_zero_plans_by_value_ranges_and_claim_changes():
    """The multi-range memset passes its ranges as kernel arguments (no device table: capturable anywhere); plans
    are cached per claim set and a plan reused after the claims change zeroes exactly its slots."""
    from iit_amd.engine.flat import FlatParams
    m = torch.nn.Sequential(torch.nn.Linear(64, 64), torch.nn.Linear(64, 64)).cuda()
    flat = FlatParams(m)
    flat.claim(m[1].weight)
    flat.grad.fill_(3.0)
    flat.zero_grad()
    plan1 = flat._zero_plan
    assert m[1].weight.grad is None and float(flat.grad_view(m[0].weight).abs().sum()) == 0.0
    assert float(flat.grad_view(m[1].weight).abs().sum()) > 0  # lazy slot untouched
    flat.claim(m[0].weight)
    flat.zero_grad()
    assert flat._zero_plan is not plan1
    flat.grad.fill_(3.0)
    flat.unclaim(m[0].weight)
    flat.zero_grad()  # back to the first claim set: its plan is reused
    assert flat._zero_plan is plan1
    assert float(flat.grad_view(m[0].weight).abs().sum()) == 0.0 and m[1].weight.grad is None
    # inside a capture: one node, replayed
    flat.grad.fill_(5.0)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        flat.zero_grad()
    flat.grad.fill_(5.0)
    g.replay()
    torch.cuda.synchronize()
    assert float(flat.grad_view(m[0].weight).abs().sum()) == 0.0 and float(flat.grad_view(m[0].bias).abs().sum()) == 0.0


def test_zero_grad_skips_restricted_rows():
    """Rows excluded by restrict_rows (never written by a backward over the data) are left out of the memset;
    every other element is zeroed, and lifting the restriction zeroes them again."""
    from iit_amd.engine.flat import FlatParams
    emb = torch.nn.Embedding(10, 8)
    lin = torch.nn.Linear(8, 4)
    m = torch.nn.ModuleDict({"e": emb, "l": lin})
    flat = FlatParams(m)
    assert flat.restrict_rows(emb.weight, torch.tensor([1, 4, 5]))
    flat.grad.fill_(2.0)
    flat.zero_grad()
    g = flat.grad_view(emb.weight)
    live = torch.zeros(10, dtype=torch.bool)
    live[[1, 4, 5]] = True
    assert float(g[live].abs().sum()) == 0.0 and bool((g[~live] == 2.0).all())
    assert float(flat.grad_view(lin.weight).abs().sum()) == 0.0 and float(flat.grad_view(lin.bias).abs().sum()) == 0.0
    flat.restrict_rows(emb.weight, None)
    flat.zero_grad()
    assert float(flat.grad.abs().sum()) == 0.0


def test_rebind_zeroes_missing_slots_only():
    """rebind_grads zeroes the slots of missing gradients in one batched launch, never a live member's values."""
    from iit_amd.engine.flat import FlatParams
    from iit_amd.models.transformer import HookedTransformer
    torch.manual_seed(0)
    m = HookedTransformer(dict(n_layers=1, n_heads=2, d_model=8, d_head=4, d_mlp=16, n_ctx=8, act_fn="gelu",
                               d_vocab=11, device="cpu"))
    flat = FlatParams(m)
    a = m.blocks[0].attn
    flat.grad.fill_(3.0)
    a.W_Q.grad = a.W_K.grad = a.W_V.grad = None  # a whole packed QKV slot missing
    m.blocks[0].mlp.W_in.grad = None              # a plain slot missing
    a.b_Q.grad = None                             # one member of the packed bias slot missing
    flat.rebind_grads()
    assert float(a.W_Q.grad.abs().sum() + a.W_K.grad.abs().sum() + a.W_V.grad.abs().sum()) == 0.0
    assert float(m.blocks[0].mlp.W_in.grad.abs().sum()) == 0.0
    assert float(a.b_Q.grad.abs().sum()) == 0.0 and bool((a.b_K.grad == 3.0).all()) and bool((a.b_V.grad == 3.0).all())
    assert bool((m.blocks[0].mlp.W_out.grad == 3.0).all())


def test_optimizer_state_refuses_other_arena_layout():
    """Adam moments saved for an NCHW arena must not load into an NHWC one (they would be permuted)."""
    import pytest
    from iit_amd.engine.flat import FlatParams
    from iit_amd.ops.optim import FusedAdam

    def make(channels_last):
        torch.manual_seed(0)
        m = torch.nn.Sequential(torch.nn.Conv2d(3, 4, 3, bias=False), torch.nn.Linear(4, 2))
        if channels_last:
            m = m.to(memory_format=torch.channels_last)
        flat = FlatParams(m)
        return flat, FusedAdam(flat, lr=1e-3, use_hip=False)

    f_a, o_a = make(False)
    f_b, o_b = make(True)
    assert f_a.layout_tag() != f_b.layout_tag()
    sd = o_a.state_dict()
    assert sd["arena_layout"] == f_a.layout_tag()
    o_a.load_state_dict(sd)  # same layout: fine
    with pytest.raises(ValueError, match="arena layout"):
        o_b.load_state_dict(sd)
    legacy = {k: v for k, v in sd.items() if k != "arena_layout"}
    o_b.load_state_dict(legacy)  # pre-tag state: loaded with a warning
