"""Paired source + base forward (HookedTransformer.run_paired, ops.hip_ops Paired functions): the source run of an
interchange intervention folded into the base forward as one batch of 2B rows up to the deepest splice site
(the reference runs two forwards, /root/reference/iit/model_pairs/base_model_pair.py:80-98).
Oracle: the same model's unpaired path (truncated source capture + spliced forward)."""
import pytest
import torch

from iit_amd.core.index import Ix

pytestmark = pytest.mark.gpu

L, D, H, DH, DM, V, S, B = 4, 128, 4, 32, 512, 1000, 16, 32


def _model(vocab=V):
    from iit_amd.models.transformer import HookedTransformer
    cfg = dict(n_layers=L, d_model=D, n_heads=H, d_head=DH, d_mlp=DM, n_ctx=S, d_vocab=vocab, act_fn="gelu_new",
               normalization_type="LNPre", device="cuda", dtype=torch.bfloat16, positional_embedding_type="standard")
    torch.manual_seed(0)
    m = HookedTransformer(cfg)
    m.set_op_backend("hip")
    return m


SITES = [
    {"blocks.0.attn.hook_z": [Ix[[None]]]},                                   # whole z (dead base attention)
    {"blocks.1.attn.hook_z": [Ix[:, :, 2]]},                                  # one head
    {"blocks.1.mlp.hook_post": [Ix[[None]]]},                                 # whole MLP post
    {"blocks.2.mlp.hook_post": [Ix[:, :, :64]]},                              # neuron range
    {"blocks.0.attn.hook_z": [Ix[[None]]], "blocks.2.attn.hook_z": [Ix[[None]]]},  # two layers
    {"blocks.3.attn.hook_z": [Ix[:, :, 1]]},                                  # final block: last-position tail
    {"blocks.3.mlp.hook_post": [Ix[:, -1, :128]]},                            # final block MLP, last position
    {"blocks.1.attn.hook_z": [Ix[:, [3, 7]]]},                                # position list
    {"blocks.1.attn.hook_z": [Ix[:, -1, :2, :]]},                             # causal graph: last position, heads
    {"blocks.2.mlp.hook_post": [Ix[2:5]]},                                    # batch subset: (base | source) axis
    {"blocks.2.attn.hook_z": [Ix[:, :, [0, 3]]]},                             # two heads (mirrored in-kernel)
    {"blocks.1.attn.hook_z": [Ix[:, :, :, :20]]},                             # feature range (partial 16-B chunks)
    {"blocks.2.attn.hook_z": [Ix[3:9, 5]]},                                   # batch subset x one position
]


def _unpaired(m, base, src, sites, logits):
    from iit_amd.engine.plan import RunPlan
    cache = m.run_capture(src, list(sites))
    plan = RunPlan.with_splices([(n, ix, cache[n]) for n, ixs in sites.items() for ix in ixs], logits=logits)
    return m(base, plan=plan), cache


@pytest.mark.parametrize("sites", SITES, ids=[",".join(s) for s in SITES])
@pytest.mark.parametrize("logits", ["last", "full"])
def test_paired_matches_two_forwards(sites, logits):
    m = _model()
    g = torch.Generator(device="cuda").manual_seed(1)
    base = torch.randint(0, V, (B, S), device="cuda", generator=g)
    src = torch.randint(0, V, (B, S), device="cuda", generator=g)
    w = torch.randn(B, V, device="cuda", generator=g)

    def loss_of(out):
        o = out[:, -1] if out.dim() == 3 else out
        return (o.float() * w).sum()

    m.zero_grad(set_to_none=True)
    ref, ref_cache = _unpaired(m, base, src, sites, logits)
    loss_of(ref).backward()
    g_ref = {k: p.grad.clone() for k, p in m.named_parameters() if p.grad is not None}

    m.zero_grad(set_to_none=True)
    res = m.run_paired(base, src, sites, logits=logits)
    assert res is not None, "paired path not taken"
    out, cache = res
    loss_of(out).backward()
    g_pair = {k: p.grad.clone() for k, p in m.named_parameters() if p.grad is not None}

    assert out.shape == ref.shape
    assert torch.allclose(out.float(), ref.float(), rtol=2e-2, atol=2e-2), (out.float() - ref.float()).abs().max()
    for n in sites:
        assert torch.allclose(cache[n].float(), ref_cache[n].float(), rtol=1e-2, atol=1e-2), n
    assert set(g_pair) == set(g_ref)
    for k in g_ref:
        # b_K's gradient is zero in exact arithmetic (softmax is shift-invariant per query): rounding noise only,
        # so it is measured against the scale of the same layer's b_Q gradient
        scale = g_ref[k[:-3] + "b_Q"].norm() if k.endswith("b_K") else g_ref[k].norm()
        err = float((g_pair[k] - g_ref[k]).norm() / (scale + 1e-12))
        assert err < 2e-2, (k, err)


@pytest.mark.parametrize("sites", [SITES[0], SITES[1], SITES[3], SITES[7]], ids=["whole_z", "head", "neurons", "pos"])
def test_paired_longer_sequences(sites):
    """16 < S <= 64: the short-sequence attention kernel (no in-kernel head mirroring; head sites go through the
    paired patch-spec splice) -- same outputs and gradients as the two forwards."""
    from iit_amd.models.transformer import HookedTransformer
    S2 = 40
    cfg = dict(n_layers=L, d_model=D, n_heads=H, d_head=DH, d_mlp=DM, n_ctx=S2, d_vocab=V, act_fn="gelu_new",
               normalization_type="LNPre", device="cuda", dtype=torch.bfloat16, positional_embedding_type="standard")
    torch.manual_seed(0)
    m = HookedTransformer(cfg)
    m.set_op_backend("hip")
    g = torch.Generator(device="cuda").manual_seed(2)
    base = torch.randint(0, V, (B, S2), device="cuda", generator=g)
    src = torch.randint(0, V, (B, S2), device="cuda", generator=g)
    w = torch.randn(B, V, device="cuda", generator=g)
    m.zero_grad(set_to_none=True)
    ref, _ = _unpaired(m, base, src, sites, "last")
    (ref.float() * w).sum().backward()
    g_ref = {k: p.grad.clone() for k, p in m.named_parameters() if p.grad is not None}
    m.zero_grad(set_to_none=True)
    res = m.run_paired(base, src, sites, logits="last")
    assert res is not None
    out, _ = res
    (out.float() * w).sum().backward()
    assert torch.allclose(out.float(), ref.float(), rtol=2e-2, atol=2e-2)
    for k, gr in g_ref.items():
        gp = m.get_parameter(k).grad
        scale = g_ref[k[:-3] + "b_Q"].norm() if k.endswith("b_K") else gr.norm()
        assert float((gp - gr).norm() / (scale + 1e-12)) < 2e-2, k


def test_paired_source_rows_get_no_gradient_and_no_graph():
    """The source activations returned by the paired forward are plain tensors (no autograd history)."""
    m = _model()
    base = torch.randint(0, V, (B, S), device="cuda")
    src = torch.randint(0, V, (B, S), device="cuda")
    out, cache = m.run_paired(base, src, {"blocks.2.attn.hook_z": [Ix[:, :, 0]]}, logits="last")
    assert out.requires_grad
    assert not cache["blocks.2.attn.hook_z"].requires_grad


def test_paired_declines_what_it_does_not_cover():
    m = _model()
    base = torch.randint(0, V, (B, S), device="cuda")
    src = torch.randint(0, V, (B, S), device="cuda")
    assert m.run_paired(base, src, {"blocks.1.hook_resid_pre": [Ix[[None]]]}) is None
    assert m.run_paired(base, src[:, :8], {"blocks.1.attn.hook_z": [Ix[[None]]]}) is None
    long = torch.randint(0, V, (B, 65), device="cuda")
    assert m.run_paired(long, long, {"blocks.1.attn.hook_z": [Ix[[None]]]}) is None  # S > 64
    h = m.blocks[0].attn.hook_z.add_hook(lambda x, hook: x)
    try:
        assert m.run_paired(base, src, {"blocks.1.attn.hook_z": [Ix[[None]]]}) is None
    finally:
        m.reset_hooks()


def test_ioi_pair_step_paired_equals_unpaired():
    """A whole IOI_ModelPair training step (IIT + strict + behaviour phases, eager) with and without pairing."""
    from iit_amd.data.iit_dataset import IITDataset
    from iit_amd.model_pairs import IOI_ModelPair
    from iit_amd.ops import hip_ops
    from iit_amd.tasks.ioi import NAMES, make_ioi_corr, make_ioi_dataset_and_hl

    calls = []
    orig = hip_ops.HipOps.pair_embed_pos
    hip_ops.HipOps.pair_embed_pos = lambda self, *a, **k: (calls.append(1), orig(self, *a, **k))[1]
    try:
        losses = {}
        for paired in (False, True):
            m = _model(50257)
            ds, hl = make_ioi_dataset_and_hl(512, m, NAMES, device="cuda")
            train = IITDataset(ds, ds, seed=0, device="cuda")
            pair = IOI_ModelPair(hl, m, make_ioi_corr(L), training_args={
                "batch_size": 64, "lr": 1e-3, "lr_scheduler": None, "paired": paired, "graphs": False})
            opt = pair.make_optimizer(1e-3)
            base, abl = next(iter(train.make_loader(64, 0)))
            out = []
            for node in list(pair.corr.keys()):
                pair.sample_hl_name = lambda node=node: node
                out.append({k: float(v) for k, v in pair.run_train_step(base, abl, pair.loss_fn, opt).items()})
            losses[paired] = out
            if paired:
                assert calls, "the paired path never ran"
        for a, b in zip(losses[False], losses[True]):
            for k in a:
                assert abs(a[k] - b[k]) <= 2e-2 * max(1.0, abs(a[k])), (k, a[k], b[k])
    finally:
        hip_ops.HipOps.pair_embed_pos = orig


def test_paired_with_staged_backward_cuts():
    """The data-parallel schedule cuts the residual stream at block boundaries (engine.staged): the paired forward
    cuts its base rows there, and the staged backward reproduces the uncut gradients."""
    from iit_amd.engine.staged import StagedBackward
    m = _model()
    g = torch.Generator(device="cuda").manual_seed(3)
    base = torch.randint(0, V, (B, S), device="cuda", generator=g)
    src = torch.randint(0, V, (B, S), device="cuda", generator=g)
    w = torch.randn(B, V, device="cuda", generator=g)
    sites = {"blocks.2.attn.hook_z": [Ix[:, :, 1]], "blocks.0.mlp.hook_post": [Ix[[None]]]}

    def grads():
        return {k: p.grad.clone() for k, p in m.named_parameters() if p.grad is not None}

    m.zero_grad(set_to_none=True)
    out, _ = m.run_paired(base, src, sites, logits="last")
    (out.float() * w).sum().backward()
    ref = grads()
    st = StagedBackward(m, 4)
    m.zero_grad(set_to_none=True)
    st.arm()
    try:
        out, _ = m.run_paired(base, src, sites, logits="last")
        assert m._cut_log, "no cut was taken"
        (out.float() * w).sum().backward()
        for k in st.stages():
            st.run_stage(k)
    finally:
        st.release()
        st.disarm()
    got = grads()
    assert set(got) == set(ref)
    for k in ref:
        assert torch.allclose(got[k], ref[k], rtol=1e-3, atol=1e-5), k


@pytest.mark.parametrize("index", [Ix[:, [3, 7]], Ix[:, -1, :2, :], Ix[:, :, :, :20], Ix[3:9, 5]],
                         ids=["positions", "last_pos_heads", "features", "batch_pos"])
def test_paired_hook_z_spec_splice_runs_in_the_attention_kernel(monkeypatch, index):
    """Non-head ``hook_z`` splices of the paired forward are applied in the attention kernel's store (K04 / K10:
    per-position and per-feature patch points), not by the separate patch-spec pass."""
    from iit_amd.ops import hip_ops

    def no_pass(self, p, ix):
        raise AssertionError("separate splice pass used for a hook_z site")

    monkeypatch.setattr(hip_ops.HipOps, "pair_splice", no_pass)
    m = _model()
    base = torch.randint(0, V, (B, S), device="cuda")
    src = torch.randint(0, V, (B, S), device="cuda")
    res = m.run_paired(base, src, {"blocks.1.attn.hook_z": [index]}, logits="last")
    assert res is not None
    out, cache = res
    ref, _ = _unpaired(m, base, src, {"blocks.1.attn.hook_z": [index]}, "last")
    assert torch.allclose(out.float(), ref.float(), rtol=2e-2, atol=2e-2)


@pytest.mark.parametrize("index", [Ix[:, :, :64], Ix[:, -1, :128], Ix[2:5], Ix[:, [3, 7], 100:130]],
                         ids=["neurons", "last_pos_neurons", "batch", "pos_neurons"])
def test_paired_mlp_post_splice_runs_inside_the_mlp_op(monkeypatch, index):
    """``mlp.hook_post`` splices of the paired forward run inside the W_in op (sparse copy of the selected source
    elements into the base rows, masked dpre in its backward), not by the separate patch-spec pass; outputs and
    gradients equal the two-forward path."""
    from iit_amd.ops import hip_ops

    def no_pass(self, p, ix):
        raise AssertionError("separate splice pass used for an mlp.hook_post site")

    m = _model()
    g = torch.Generator(device="cuda").manual_seed(5)
    base = torch.randint(0, V, (B, S), device="cuda", generator=g)
    src = torch.randint(0, V, (B, S), device="cuda", generator=g)
    w = torch.randn(B, V, device="cuda", generator=g)
    sites = {"blocks.2.mlp.hook_post": [index]}
    m.zero_grad(set_to_none=True)
    ref, _ = _unpaired(m, base, src, sites, "last")
    (ref.float() * w).sum().backward()
    g_ref = {k: p.grad.clone() for k, p in m.named_parameters() if p.grad is not None}
    monkeypatch.setattr(hip_ops.HipOps, "pair_splice", no_pass)
    m.zero_grad(set_to_none=True)
    res = m.run_paired(base, src, sites, logits="last")
    assert res is not None
    out, _ = res
    (out.float() * w).sum().backward()
    assert torch.allclose(out.float(), ref.float(), rtol=2e-2, atol=2e-2)
    for k, gr in g_ref.items():
        gp = m.get_parameter(k).grad
        scale = g_ref[k[:-3] + "b_Q"].norm() if k.endswith("b_K") else gr.norm()
        assert float((gp - gr).norm() / (scale + 1e-12)) < 2e-2, k
