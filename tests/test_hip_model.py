"""T1 at model level: HIP engine (bf16) vs the fp32 PyTorch oracle on the same weights.

Covers plain forward/backward, capture-only truncated source runs, in-kernel
whole-tensor and per-head splices (incl. zero gradient through spliced slices),
last-position logits, and a full IOI_ModelPair train step.
"""
import copy

import pytest
import torch

pytestmark = pytest.mark.gpu
dev = "cuda"


def make_models(n_layers=2, d_model=128, n_heads=4, d_head=32, d_vocab=1000, normalization="LNPre"):
    from iit_amd.models.transformer import HookedTransformer
    cfg = dict(n_layers=n_layers, d_model=d_model, n_heads=n_heads, d_head=d_head, d_mlp=4 * d_model, n_ctx=64,
               act_fn="gelu_new", d_vocab=d_vocab, normalization_type=normalization, device=dev, initializer_range=0.05)
    torch.manual_seed(0)
    ref = HookedTransformer(cfg)
    fast = HookedTransformer({**cfg, "dtype": torch.bfloat16})
    fast.load_state_dict(ref.state_dict())
    fast.set_op_backend("hip")
    ref.set_op_backend("torch")
    return ref, fast


def rel(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


@pytest.mark.parametrize("norm", ["LNPre", "LN"])
def test_forward_backward_parity(norm):
    ref, fast = make_models(normalization=norm)
    tok = torch.randint(0, 1000, (8, 16), device=dev)
    lr = ref(tok)
    lf = fast(tok)
    assert rel(lf, lr) < 2e-2
    lr.float().pow(2).mean().backward()
    lf.float().pow(2).mean().backward()
    scale = max(p.grad.norm().item() for p in ref.parameters())
    for (n, pr), (_, pf) in zip(ref.named_parameters(), fast.named_parameters()):
        assert pf.grad is not None, n
        if pr.grad.norm().item() < 1e-4 * scale:  # e.g. b_K: exactly zero in exact arithmetic
            assert pf.grad.norm().item() < 1e-3 * scale, n
            continue
        assert rel(pf.grad, pr.grad) < 6e-2, n


def test_last_position_logits_and_argmax():
    ref, fast = make_models()
    from iit_amd.engine.plan import RunPlan
    tok = torch.randint(0, 1000, (8, 16), device=dev)
    full = ref(tok)
    last = fast(tok, plan=RunPlan(logits="last"))
    assert last.shape == (8, 1000)
    assert rel(last, full[:, -1]) < 2e-2
    am = fast(tok, plan=RunPlan(logits="argmax"))
    assert (am == fast(tok).argmax(-1)).float().mean() > 0.97


def test_capture_and_splice_semantics():
    ref, fast = make_models()
    from iit_amd.core.index import Ix
    from iit_amd.engine.plan import RunPlan
    src = torch.randint(0, 1000, (8, 16), device=dev)
    base = torch.randint(0, 1000, (8, 16), device=dev)
    names = ["blocks.0.attn.hook_z", "blocks.1.mlp.hook_post"]
    cr = ref.run_capture(src, names)
    cf = fast.run_capture(src, names)
    for n in names:
        assert rel(cf[n], cr[n]) < 2e-2
    for index in (Ix[[None]], Ix[:, :, 2, :]):
        spl = [("blocks.0.attn.hook_z", index, cf["blocks.0.attn.hook_z"]),
               ("blocks.1.mlp.hook_post", Ix[[None]], cf["blocks.1.mlp.hook_post"])]
        out_r = ref(base, plan=RunPlan.with_splices([(n, i, s.float()) for n, i, s in spl], logits="last"))
        out_f = fast(base, plan=RunPlan.with_splices(spl, logits="last"))
        assert rel(out_f, out_r) < 3e-2
        ref.zero_grad(set_to_none=True)
        fast.zero_grad(set_to_none=True)
        out_r.float().pow(2).mean().backward()
        out_f.float().pow(2).mean().backward()
        scale = max(p.grad.norm().item() for p in ref.parameters() if p.grad is not None)
        for (n, pr), (_, pf) in zip(ref.named_parameters(), fast.named_parameters()):
            gr = pr.grad if pr.grad is not None else torch.zeros_like(pr)
            gf = pf.grad if pf.grad is not None else torch.zeros_like(pf)
            if gr.abs().max() == 0:
                assert gf.abs().max() == 0, n  # spliced-away producers get exactly no gradient
            elif gr.norm().item() < 1e-4 * scale:  # b_K: zero in exact arithmetic
                assert gf.norm().item() < 1e-3 * scale, n
            else:
                assert rel(gf, gr) < 8e-2, n


def test_ioi_pair_train_step_hip():
    from iit_amd.data.iit_dataset import IITDataset
    from iit_amd.model_pairs import IOI_ModelPair
    from iit_amd.models.config import gpt2_config_dict
    from iit_amd.models.transformer import HookedTransformer
    from iit_amd.tasks.ioi import ioi_cfg, make_ioi_corr, make_ioi_dataset_and_hl
    cfg = gpt2_config_dict()
    cfg.update(ioi_cfg)
    cfg.update(device=dev, dtype=torch.bfloat16)
    torch.manual_seed(0)
    ll = HookedTransformer(cfg)
    ds, hl = make_ioi_dataset_and_hl(512, ll, device=dev)
    train = IITDataset(ds, ds, seed=0, device=dev)
    pair = IOI_ModelPair(hl, ll, make_ioi_corr(6), training_args={"batch_size": 128, "lr": 1e-3, "strict_weight": 0.4,
                                                                   "lr_scheduler": None})
    opt = pair.make_optimizer(1e-3)
    loader = train.make_loader(128, 0)
    losses = []
    for _ in range(3):
        for base, abl in loader:
            out = pair.run_train_step(base, abl, pair.loss_fn, opt)
            losses.append(out["train/behavior_loss"].item())
    assert all(torch.isfinite(torch.tensor(losses)))
    assert losses[-1] < losses[0]


def test_arena_mirror_training_matches_fp32_reference():
    """Flat arena in kernel layout + fused clip/Adam writing the bf16 mirror vs fp32 torch Adam."""
    from iit_amd.engine.flat import FlatParams
    from iit_amd.ops.optim import FusedAdam
    ref, fast = make_models()
    p0 = {n: p.detach().clone() for n, p in ref.named_parameters()}
    flat = FlatParams(fast)
    opt = FusedAdam(flat, lr=1e-3)
    opt_ref = torch.optim.Adam(ref.parameters(), lr=1e-3)
    for step in range(3):
        tok = torch.randint(0, 1000, (8, 16), device=dev)
        opt.zero_grad()
        fast(tok).float().pow(2).mean().backward()
        opt.step(clip_norm=1.0)
        opt_ref.zero_grad()
        ref(tok).float().pow(2).mean().backward()
        torch.nn.utils.clip_grad_norm_(ref.parameters(), 1.0)
        opt_ref.step()
        sh = fast._iit_hip_ops.shadow
        assert sh.mode == "mirror"
        # the mirror the kernels read is exactly bf16(master) after every fused step
        assert torch.equal(flat.shadow, flat.data.to(torch.bfloat16))
    assert int(opt._step_dev.item()) == 3
    for (n, pr), (_, pf) in zip(ref.named_parameters(), fast.named_parameters()):
        if n.endswith("b_K"):
            continue
        # Adam moves every weight by ~lr per step regardless of gradient scale, so elements whose
        # gradient is at bf16 noise level may move differently: compare the update direction in bulk
        assert rel(pf.detach() - p0[n], pr.detach() - p0[n]) < 0.35, n
        assert ((pf - pr).abs() > 2.5e-3).float().mean().item() < 0.05, n


def _bert_pair_models():
    from iit_amd.models.bert import HookedEncoder, bert_config_dict
    cfg = bert_config_dict("bert-tiny", n_layers=2, d_model=128, n_heads=2, d_head=64, d_mlp=256, d_vocab=64,
                           n_ctx=32, device=dev)
    torch.manual_seed(0)
    ref = HookedEncoder(cfg, n_classes=3)
    fast = HookedEncoder({**cfg, "dtype": torch.bfloat16}, n_classes=3)
    fast.load_state_dict(ref.state_dict())
    ref.set_op_backend("torch")
    for m in (ref, fast):
        m.sep_token_id = 2
    return ref, fast


def test_bert_encoder_on_hip_matches_fp32_oracle():
    """BERT (post-LN, affine LN, bidirectional attention, erf-GELU) on the HIP backend vs the fp32 oracle."""
    from iit_amd.ops.hip_ops import HipOps
    ref, fast = _bert_pair_models()
    assert isinstance(fast.ops(), HipOps)
    tok = torch.randint(3, 64, (16, 15), device=dev)
    tok[:, 0], tok[:, 7], tok[:, 14] = 1, 2, 2
    lr, lf = ref(tok), fast(tok)
    assert rel(lf, lr) < 3e-2
    lr.float().pow(2).mean().backward()
    lf.float().pow(2).mean().backward()
    scale = max(p.grad.norm().item() for p in ref.parameters())
    for (n, pr), (_, pf) in zip(ref.named_parameters(), fast.named_parameters()):
        assert pf.grad is not None, n
        if pr.grad.norm().item() < 1e-3 * scale:
            continue
        assert rel(pf.grad, pr.grad) < 8e-2, n


def test_bert_paired_forward_equals_two_forwards(monkeypatch):
    """HookedEncoder.run_paired (source rows folded into the base forward, MQNLI's hook_normalized_resid_post
    position sites, a head site and an MLP site) vs the truncated source capture + spliced base forward: same
    outputs and captured activations, same gradients, and the source rows get none."""
    from iit_amd.core.index import Ix
    from iit_amd.engine.plan import RunPlan
    monkeypatch.setenv("IIT_BERT_PAIRED", "1")
    _, fast = _bert_pair_models()
    torch.manual_seed(1)
    tok = torch.randint(3, 64, (16, 15), device=dev)
    src = torch.randint(3, 64, (16, 15), device=dev)
    for t in (tok, src):
        t[:, 0], t[:, 7], t[:, 14] = 1, 2, 2
    cases = [{"blocks.0.hook_normalized_resid_post": [Ix[:, [2, 3]]]},
             {"blocks.1.hook_normalized_resid_post": [Ix[:, [0]]]},
             {"blocks.0.attn.hook_z": [Ix[:, :, 1, :]]},
             {"blocks.1.mlp.hook_post": [Ix[:, 4:9]]},
             {"blocks.0.hook_normalized_resid_post": [Ix[:, [5]]], "blocks.1.attn.hook_z": [Ix[:, :, 0, :]]}]
    for sites in cases:
        res = fast.run_paired(tok, src, sites)
        assert res is not None, sites
        out_p, caps = res
        cache = fast.run_capture(src, list(sites))
        for n in sites:
            # the paired run's GEMMs are M = 2T problems (other tiles / splits than the T-row capture run): equal up
            # to bf16 rounding of the last bit
            assert rel(caps[n], cache[n]) < 5e-3, (sites, n)
        spl = [(n, ix, cache[n]) for n, ixs in sites.items() for ix in ixs]
        out_2 = fast(tok, plan=RunPlan.with_splices(spl))
        assert rel(out_p, out_2) < 1e-2, sites
        grads = []
        for o in (out_p, out_2):
            fast.zero_grad(set_to_none=True)
            o.float().pow(2).mean().backward()
            grads.append({n: p.grad.detach().clone() for n, p in fast.named_parameters() if p.grad is not None})
        assert grads[0].keys() == grads[1].keys()
        for n in grads[1]:
            if grads[1][n].norm() < 1e-6:
                continue
            assert rel(grads[0][n], grads[1][n]) < 3e-2, (sites, n)


def test_mqnli_bert_pair_trains_on_hip_arena():
    """IIT + behaviour steps of the MQNLI pair with the flat arena mirror + fused Adam on the HIP backend."""
    from iit_amd.data.iit_dataset import IITDataset
    from iit_amd.model_pairs import IITBehaviorModelPair
    from iit_amd.tasks.mqnli import make_mqnli_task
    _, fast = _bert_pair_models()
    ds, hl, corr = make_mqnli_task(fast, n_samples=512, device=dev)
    pair = IITBehaviorModelPair(hl, fast, corr, training_args={"batch_size": 64, "lr": 1e-3, "lr_scheduler": None,
                                                                "early_stop": False})
    opt = pair.make_optimizer(1e-3)
    loader = IITDataset(ds, ds, seed=0, device=dev).make_loader(64, 0)
    losses = []
    for i, (base, abl) in enumerate(loader):
        if i >= 6:
            break
        out = pair.run_train_step(base, abl, pair.loss_fn, opt)
        losses.append(float(out["train/behavior_loss"]))
    assert fast.ops().shadow.mode == "mirror"
    assert all(torch.isfinite(torch.tensor(losses)))


def test_torch_backend_reads_arena_mirror_and_accumulates_in_place(monkeypatch):
    """Llama-family (torch op backend, bf16 on GPU): weights come from the arena's bf16 mirror and gradients land
    in the fp32 arena directly (fp32-output weight-gradient GEMMs, fp32 bias sums) -- the plain cast +
    AccumulateGrad path agrees to bf16 rounding (it rounds dW and the bias sums to bf16 first)."""
    from iit_amd.engine.flat import FlatParams
    from iit_amd.models.convert import llama_config_dict
    from iit_amd.models.transformer import HookedTransformer
    from iit_amd.ops import torch_ops
    cfg = llama_config_dict("llama-tiny", device=dev, dtype=torch.bfloat16)
    assert cfg["n_key_value_heads"] < cfg["n_heads"]  # grouped-query heads: packed [d][(H + 2 H_kv) dh] arena group
    calls = []
    orig = torch_ops._MirrorMat.apply
    # (monkeypatch removes the class attribute afterwards; assigning ``orig`` back would leave a bound _MirrorMat.apply
    # on the class, which its subclasses -- torch_pairs.MirrorMatPairFn -- would then inherit)
    monkeypatch.setattr(torch_ops._MirrorMat, "apply", lambda *a_: calls.append(1) or orig(*a_))
    for S in (9, 40):  # 40 > 16 with d_head 64: the tiled MFMA attention kernel on the torch backend
        if S > 16:
            cfg = llama_config_dict("llama-tiny", device=dev, dtype=torch.bfloat16, d_head=64, rotary_dim=64)
        torch.manual_seed(0)
        a = HookedTransformer(cfg)
        b = copy.deepcopy(a)
        flat = FlatParams(a)
        tok = torch.randint(0, cfg["d_vocab"], (4, S), device=dev)
        with torch.no_grad():
            assert rel(a(tok), b(tok)) < 1e-2
        for m in (a, b):
            m(tok).float().pow(2).mean().backward()
        assert flat.shadow is not None  # the mirror was used
        scale = max(pb.grad.float().norm().item() for pb in b.parameters())
        for (n, pa), (_, pb) in zip(a.named_parameters(), b.named_parameters()):
            # near-cancelling gradients (the key bias: softmax is shift-invariant up to the rotary) are noise
            # in both paths: relative to the model's gradient scale there
            err = (pa.grad.float() - pb.grad.float()).norm().item()
            assert err <= 1e-2 * pb.grad.float().norm().item() + 1e-4 * scale, (S, n)
        assert flat.grad.abs().sum() > 0
    assert calls  # packed QKV / 2-D W_O projections ran


def test_bias_sums_survive_a_failed_backward():
    """the batched bias column sums are flushed by the backward pass's final callback.  A
    backward that raises after queueing a bias (an aborted graph capture) never runs it; the next backward must
    still produce complete bias gradients (stale items of the failed pass are dropped, not summed)."""
    ref, fast = make_models()
    tok = torch.randint(0, 1000, (8, 16), device=dev)

    def grads(model, fail):
        model.zero_grad(set_to_none=True)
        if fail:
            # block 0's input gradient arrives last: by then every block has queued its bias sums
            def boom(g, hook):
                raise RuntimeError("injected backward failure")
            model.add_hook(model.blocks[0].hook_resid_pre.name, boom, dir="bwd")
        out = model(tok)
        try:
            out.float().pow(2).mean().backward()
        finally:
            model.reset_hooks()
        torch.cuda.synchronize()
        return {n: p.grad.detach().clone() for n, p in model.named_parameters() if n.endswith(("b_in", "b_out", "b_O"))}

    with pytest.raises(RuntimeError, match="injected"):
        grads(fast, fail=True)
    gf = grads(fast, fail=False)
    gr = grads(ref, fail=False)
    for n in gr:
        assert gf[n].abs().sum() > 0, n
        assert rel(gf[n], gr[n]) < 3e-2, (n, rel(gf[n], gr[n]))
