"""The headline step, whole stack, against the fp32 oracle.

GPT-2-small (12L / 768d / 12H, V 50257), B = 256, S = 16, ``IOI_ModelPair`` with the bench's training args: the bf16
HIP engine exactly as ``bench.py`` runs it -- fused kernels, dual dX / dW GEMM launches with fused bias sums and
sums of squares, reduction split-K, the paired source+base forward, fused clip + Adam on the flat arena, phases
captured and replayed as HIP graphs -- beside the fp32 torch-op engine with ``torch.optim.Adam`` +
``clip_grad_norm_`` (reference semantics: ``/root/reference/iit/model_pairs/strict_iit_model_pair.py:36-91``,
``ioi_model_pair.py:55-69``), both from the same weights and batches, with the HL / strict nodes forced so steps
2-3 are a capture and a replay of the same phase graphs and step 4 is a fresh eager node.

Asserted: identical HL labels for every HL node; per-phase gradient norms and per-parameter gradients of one
eager phase of each kind; per-step, per-phase losses; and after the four steps (12 Adam updates) the weight deltas
per parameter (cosine and relative norm).
"""
import math

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
dev = torch.device("cuda")

ARGS = {"batch_size": 256, "lr": 1e-4, "iit_weight": 1.0, "behavior_weight": 1.0, "strict_weight": 0.4,
        "next_token": False, "lr_scheduler": None, "clip_grad_norm": 1.0, "early_stop": True,
        "use_single_loss": False}


def _setup():
    from iit_amd.data.iit_dataset import IITDataset
    from iit_amd.model_pairs import IOI_ModelPair
    from iit_amd.models.config import gpt2_config_dict
    from iit_amd.models.transformer import HookedTransformer
    from iit_amd.tasks.ioi import make_ioi_corr, make_ioi_dataset_and_hl

    torch.manual_seed(0)
    cfg = gpt2_config_dict()
    cfg.update(device=str(dev), init_weights=True, dtype=torch.bfloat16)
    fast = HookedTransformer(cfg)
    ref = HookedTransformer({**cfg, "dtype": torch.float32})
    ref.load_state_dict({k: v.float() for k, v in fast.state_dict().items()})
    ref.set_op_backend("torch")
    ds, hl = make_ioi_dataset_and_hl(4096, fast, device=dev)
    train = IITDataset(ds, ds, seed=0, device=dev)
    pf = IOI_ModelPair(ll_model=fast, hl_model=hl, corr=make_ioi_corr(12), training_args=dict(ARGS))
    pr = IOI_ModelPair(ll_model=ref, hl_model=hl, corr=make_ioi_corr(12),
                       training_args={**ARGS, "fused_optimizer": False})
    return pf, pr, train


def _grads(pair, opt, loss):
    opt.zero_grad()
    pair.backward(loss) if hasattr(pair, "backward") else loss.backward()
    flat = getattr(pair.ll_model, "_flat_params", None)
    if flat is not None:
        flat.rebind_grads(zero_missing=True)
    return {n: (p.grad.detach().float().clone() if p.grad is not None else torch.zeros_like(p, dtype=torch.float32))
            for n, p in pair.ll_model.named_parameters()}


def _rel(a, b):
    return float((a - b).norm() / (b.norm() + 1e-12))


def test_headline_step_matches_fp32_oracle():
    from iit_amd.engine.graphs import GraphedTrainStep
    from iit_amd.model_pairs.ioi_model_pair import IOI_ModelPair

    pf, pr, train = _setup()
    of = pf.make_optimizer(ARGS["lr"])
    orf = pr.make_optimizer(ARGS["lr"])
    assert not hasattr(orf, "flat")  # the oracle steps with torch.optim.Adam
    pf.restrict_sparse_rows(train)
    batches = [b for _, b in zip(range(4), train.make_loader(256, 0))]
    hl_nodes = list(pf.corr.keys())
    strict_nodes = pf.nodes_not_in_circuit

    # ---- HL labels: the fused label kernel vs the HL model run with hooks (torch ops)
    base, abl = batches[0]
    for node in hl_nodes:
        lab_fast = pf.fast_hl_label(base[0], abl[0], node)
        assert lab_fast is not None, node
        hl_out, _ = pr.do_intervention(base, abl, node)
        assert torch.equal(lab_fast.long(), IOI_ModelPair._hl_label(hl_out).long()), node.name

    # ---- one eager phase of each kind: gradient norm and per-parameter gradients
    scale_print = []
    for kind in ("iit", "strict", "behavior"):
        gs = []
        for pair, opt in ((pf, of), (pr, orf)):
            if kind == "iit":
                loss = pair.get_IIT_loss_over_batch(base, abl, hl_nodes[1], pair.loss_fn)
            elif kind == "strict":
                loss = pair.get_strict_loss_over_batch(base, abl, strict_nodes[3], pair.loss_fn)
            else:
                loss = pair.get_behaviour_loss_over_batch(base, pair.loss_fn)
            gs.append(_grads(pair, opt, loss))
        gf, gr = gs
        nf = math.sqrt(sum(float(g.pow(2).sum()) for g in gf.values()))
        nr = math.sqrt(sum(float(g.pow(2).sum()) for g in gr.values()))
        scale_print.append((kind, nf, nr))
        assert abs(nf - nr) / nr < 3e-2, (kind, nf, nr)
        big = max(float(g.norm()) for g in gr.values())
        for n in gr:
            if float(gr[n].norm()) < 1e-3 * big:  # b_K and friends: zero in exact arithmetic
                assert float(gf[n].norm()) < 1e-2 * big, (kind, n)
                continue
            # measured worst 0.0146 (blocks.10.attn.W_K, strict); the bf16 torch-op engine's worst is 0.024
            assert _rel(gf[n], gr[n]) < 0.03, (kind, n, _rel(gf[n], gr[n]))
    print("grad norms (kind, bf16 HIP, fp32 oracle):", scale_print)
    for opt in (of, orf):
        opt.zero_grad()

    # ---- four full steps: graphs for the HIP engine (step 1 eager, 2 capture + replay, 3 replay, 4 a new node)
    w0 = {n: p.detach().float().clone() for n, p in pr.ll_model.named_parameters()}
    step = GraphedTrainStep(pf, of, pf.loss_fn)
    assert step.enabled
    forced = [(1, 3), (1, 3), (1, 3), (2, 5)]
    with step.stream_context():
        for (h, s), (b, a) in zip(forced, batches):
            outs = []
            for pair, fn, opt in ((pf, step, of), (pr, pr.run_train_step, orf)):
                pair.sample_hl_name = lambda h=h: hl_nodes[h]
                pair.sample_ll_node = lambda s=s: strict_nodes[s]
                outs.append({k: float(v) for k, v in fn(b, a, pair.loss_fn, opt).items()})
            print("step losses bf16 / fp32:", outs)
            for k in outs[1]:
                assert abs(outs[0][k] - outs[1][k]) <= 2e-2 * abs(outs[1][k]) + 2e-3, (k, outs)
    assert step.captures >= 3 and step.replays >= 6, (step.captures, step.replays)
    torch.cuda.synchronize()

    # ---- weight deltas after 12 Adam updates
    worst = []
    for (n, p_f), (_, p_r) in zip(pf.ll_model.named_parameters(), pr.ll_model.named_parameters()):
        df = p_f.detach().float() - w0[n]
        dr = p_r.detach().float() - w0[n]
        if n.endswith("b_K"):
            # zero gradient in exact arithmetic (softmax is shift-invariant along the key axis): the fp32 oracle's
            # gradient is ~1e-12 noise, below Adam's eps, so its update is ~0, while bf16 noise (> eps) moves it by ~lr;
            # only the size of the bf16 update is bounded
            assert float(df.abs().max()) <= 1.5 * ARGS["lr"] * 12, n
            continue
        if float(dr.norm()) == 0.0:
            assert float(df.norm()) == 0.0, n
            continue
        cos = float((df * dr).sum() / (df.norm() * dr.norm() + 1e-30))
        rn = float(df.norm() / dr.norm())
        worst.append((cos, rn, n))
        assert cos > 0.99 and 0.97 < rn < 1.03, (n, cos, rn)  # measured worst: cos 0.9989, ratio 0.9979-1.0017
    worst.sort()
    print("weight-delta cosine / norm ratio, worst 5:", worst[:5])
    assert np.isfinite([w[0] for w in worst]).all()


def test_headline_gradients_kernel_error_vs_precision_error():
    """Separates kernel error from bf16 precision error: the same phases run on three engines
    from the same weights and batch -- the bf16 HIP engine, the bf16 torch-op engine (``TorchOps(bf16)``: the same
    precision, library ops) and the fp32 torch-op oracle.  Per parameter, the HIP engine's gradient error against the
    oracle must not exceed the bf16 torch-op engine's by more than a small margin (measured on MI355X: the HIP engine's
    worst relative error is 0.0146, the torch-op engine's 0.024 -- the HIP engine keeps the residual stream in fp32,
    TorchOps(bf16) rounds it per op).  The two bf16 engines' mutual distance is bounded by the sum of their
    independent rounding errors (measured worst 0.0226), so the 2 % the round-4 review suggested for that pair is
    below what two correct bf16 engines can reach; the kernel-error criterion is the first assertion."""
    from iit_amd.model_pairs import IOI_ModelPair
    from iit_amd.models.transformer import HookedTransformer
    from iit_amd.tasks.ioi import make_ioi_corr

    pf, pr, train = _setup()
    from iit_amd.models.config import gpt2_config_dict
    tb = HookedTransformer({**gpt2_config_dict(), "device": str(dev), "init_weights": False, "dtype": torch.bfloat16})
    tb.load_state_dict({k: v.float() for k, v in pr.ll_model.state_dict().items()})
    tb.set_op_backend("torch")
    pt = IOI_ModelPair(ll_model=tb, hl_model=pf.hl_model, corr=make_ioi_corr(12),
                       training_args={**ARGS, "fused_optimizer": False})
    opts = [p.make_optimizer(ARGS["lr"]) for p in (pf, pt, pr)]
    pf.restrict_sparse_rows(train)
    base, abl = next(iter(train.make_loader(256, 0)))
    hl_nodes = list(pf.corr.keys())
    strict_nodes = pf.nodes_not_in_circuit
    rows = []
    for kind in ("iit", "strict", "behavior"):
        gs = []
        for pair, opt in zip((pf, pt, pr), opts):
            if kind == "iit":
                loss = pair.get_IIT_loss_over_batch(base, abl, hl_nodes[1], pair.loss_fn)
            elif kind == "strict":
                loss = pair.get_strict_loss_over_batch(base, abl, strict_nodes[3], pair.loss_fn)
            else:
                loss = pair.get_behaviour_loss_over_batch(base, pair.loss_fn)
            gs.append(_grads(pair, opt, loss))
        gf, gt, gr = gs
        big = max(float(g.norm()) for g in gr.values())
        for n in gr:
            if float(gr[n].norm()) < 1e-3 * big:  # zero in exact arithmetic (b_K, ...): bf16 noise on both sides
                continue
            rows.append((kind, n, _rel(gf[n], gr[n]), _rel(gt[n], gr[n]), _rel(gf[n], gt[n])))
    rows.sort(key=lambda r: -r[2])
    print("worst HIP-vs-fp32 rows (kind, param, HIP err, torch-bf16 err, HIP vs torch-bf16):")
    for r in rows[:12]:
        print("  %-9s %-28s %.4f %.4f %.4f" % r)
    print("max HIP err %.4f, max torch-bf16 err %.4f, max HIP-vs-torch-bf16 %.4f" % (
        max(r[2] for r in rows), max(r[3] for r in rows), max(r[4] for r in rows)))
    for kind, n, ef, et, eft in rows:
        assert ef <= 1.25 * et + 5e-3, (kind, n, ef, et)  # no kernel error beyond bf16 precision
        assert ef <= 0.02, (kind, n, ef)
        assert eft <= 0.035, (kind, n, eft)
