"""Graph runner vs eager in lock step (tests/test_graphs.py fp32 setup, IIT phases captured for s_inhibition then
all_nodes_hook): after every optimizer phase the weights are copied into preallocated buffers (no allocation in
between, so the schedule is not perturbed) and compared at the end; prints the first phase whose weights differ."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import test_graphs as tg  # noqa: E402
from iit_amd.engine.graphs import GraphedTrainStep  # noqa: E402

NPH = 15


def run(mode):
    pair, opt, train = tg._setup(dtype=torch.float32)
    torch.manual_seed(1)
    batches = [b for _, b in zip(range(10), train.make_loader(64, 0))]
    nodes = {n.name: n for n in pair.corr.keys()}
    seq = ["hook_s_inhibition", "all_nodes_hook"] * 4
    cnt = [0]

    def pick():
        cnt[0] += 1
        return nodes[seq[cnt[0] - 1]]
    pair.sample_hl_name = pick
    pair.sample_ll_node = lambda: pair.nodes_not_in_circuit[0]
    snaps = torch.empty(NPH, opt.flat.numel, device=opt.flat.data.device)
    hows = []
    k = [0]

    def record(how, key):
        if k[0] < NPH:
            snaps[k[0]].copy_(opt.flat.data)
            hows.append((key, how))
        k[0] += 1
    if mode == "graphs":
        g = GraphedTrainStep(pair, opt, pair.loss_fn)
        orig = g._run_phase

        def sel(key, compute_loss, optimizer, step_fn):
            full = (key, g._sig)
            if key[0] != "iit":
                out = g._eager(compute_loss, optimizer, step_fn)
                record("eager", key)
                return out
            how = "replay" if full in g.graphs else ("eager" if g.seen.get(full, 0) < g.warmup else "capture")
            out = orig(key, compute_loss, optimizer, step_fn)
            record(how, key)
            return out
        pair._phase_runner = sel
        step, ctx = g, g.stream_context()
    else:
        orig_rp = pair.run_phase

        def rp(key, *a):
            out = orig_rp(key, *a)
            record("eager", key)
            return out
        pair.run_phase = rp
        import contextlib
        step, ctx = pair.run_train_step, contextlib.nullcontext()
    with ctx:
        for i in range(5):
            step(*batches[i], pair.loss_fn, opt)
    torch.cuda.synchronize()
    return snaps.cpu(), hows


e, he = run("eager")
gg, hg = run("graphs")
for i in range(NPH):
    d = float((e[i] - gg[i]).abs().max())
    print(f"phase {i:2d} {hg[i][0][0]:8s} {hg[i][0][1] if len(hg[i][0]) > 1 else '':22s} {hg[i][1]:8s} max|dW| {d:.3e}")
