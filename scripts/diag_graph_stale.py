"""Which part of a stale torch-backend phase graph is wrong (tests/test_graphs.py fp32 setup): capture the IIT
phase for s_inhibition, then for all_nodes_hook; replay s_inhibition and compare the activation caches its graph
wrote (source LL capture, HL caches, logits) against an eager recomputation on the same weights and batch."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import test_graphs as tg  # noqa: E402
from iit_amd.engine.graphs import GraphedTrainStep  # noqa: E402

pair, opt, train = tg._setup(dtype=torch.float32)
torch.manual_seed(1)
batches = [b for _, b in zip(range(10), train.make_loader(64, 0))]
nodes = {n.name: n for n in pair.corr.keys()}
seq = ["hook_s_inhibition", "all_nodes_hook"] * 3
g = GraphedTrainStep(pair, opt, pair.loss_fn)
orig = g._run_phase
snap = {}


def sel(key, compute_loss, optimizer, step_fn):
    if key[0] != "iit":
        return g._eager(compute_loss, optimizer, step_fn)
    full = (key, g._sig)
    capturing = full not in g.graphs and g.seen.get(full, 0) >= g.warmup
    out = orig(key, compute_loss, optimizer, step_fn)
    if capturing:  # the caches this capture recorded live in the graph's pool: every replay rewrites them
        snap[key[1]] = (dict(pair.ll_cache.cache_dict if hasattr(pair.ll_cache, "cache_dict") else pair.ll_cache),
                        {k: v for k, v in dict(pair.hl_cache.cache_dict if hasattr(pair.hl_cache, "cache_dict")
                                               else pair.hl_cache).items()})
    return out


pair._phase_runner = sel
cnt = [0]
pair.sample_hl_name = lambda: nodes[seq[(cnt.__setitem__(0, cnt[0] + 1) or cnt[0]) - 1]]
pair.sample_ll_node = lambda: pair.nodes_not_in_circuit[0]
with g.stream_context():
    for i in range(4):
        g(*batches[i])
    # step 4: the s_inhibition IIT phase replays after all_nodes_hook's capture.  Weights before it:
    state = opt.flat.data.clone()
    mom = (opt.exp_avg.clone(), opt.exp_avg_sq.clone(), opt._step_dev.clone())
    base, abl = batches[4]
    sb, sa, _ = g._stage(base, abl)
    key = ("iit", "hook_s_inhibition")
    ent = g.graphs[(key, g._sig)]
    ent[0][0].replay() if isinstance(ent[0], tuple) else ent[0].replay()
    torch.cuda.synchronize()
    ll_g, hl_g = snap["hook_s_inhibition"]
    ll_g = {k: v.clone() for k, v in ll_g.items()}
    hl_g = {k: v.clone() for k, v in hl_g.items()}
    w_graph, g_graph = opt.flat.data.clone(), opt.flat.grad.clone()
    # eager recomputation of the source caches on the pre-step weights
    opt.flat.data.copy_(state)
    opt.flat.after_step()
    with torch.no_grad():
        hl_out, hl_c = pair.hl_model.run_with_cache(sa, **pair.hl_run_kwargs())
        ll_c = pair.ll_model.run_capture(sa[0], sorted(ll_g.keys()))
    torch.cuda.synchronize()
    # the whole phase eagerly from the same state
    opt.flat.data.copy_(state)
    opt.exp_avg.copy_(mom[0]); opt.exp_avg_sq.copy_(mom[1]); opt._step_dev.copy_(mom[2])
    opt.flat.after_step()
    node = nodes["hook_s_inhibition"]
    w = pair.training_args["iit_weight"]
    g._eager(lambda: pair.get_IIT_loss_over_batch(sb, sa, node, pair.loss_fn) * w, opt, pair.step_on_loss)
    torch.cuda.synchronize()
    w_eager, g_eager = opt.flat.data.clone(), opt.flat.grad.clone()
print("weights max|graph - eager|:", float((w_graph - w_eager).abs().max()),
      " grads:", float((g_graph - g_eager).abs().max()))
for n, p in pair.ll_model.named_parameters():
    if opt.flat.owns(p):
        o, k = opt.flat.offset_of(p), p.numel()
        dg = float((g_graph[o:o + k] - g_eager[o:o + k]).abs().max())
        if dg > 0:
            print(f"  grad {n:28s} max|d| {dg:.3e}  |g_eager| {float(g_eager[o:o + k].norm()):.3e} "
                  f"|g_graph| {float(g_graph[o:o + k].norm()):.3e}")
for k in ll_g:
    d = (ll_g[k].float() - ll_c[k].float()).abs().max()
    print(f"LL source cache {k}: max|graph - eager| = {float(d):.3e}")
for k in hl_g:
    if k in hl_c:
        d = (hl_g[k].float() - hl_c[k].float()).abs().max()
        print(f"HL cache {k}: max|graph - eager| = {float(d):.3e}")
