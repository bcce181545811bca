"""Per-HL-node graph check (fp32 torch-op backend, tests/test_graphs.py setup): every step samples the same HL node
and strict node, so step 0 runs eagerly, step 1 captures + replays, later steps replay; losses vs a plain eager
run of the same schedule."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import test_graphs as tg  # noqa: E402

if os.environ.get("NO_EMPTY_CACHE") == "1":
    torch.cuda.empty_cache = lambda: None
if os.environ.get("NO_GC") == "1":
    import gc
    gc.collect = lambda *a, **k: 0


def run(mode, hl_name, only_iit):
    from iit_amd.engine.graphs import GraphedTrainStep
    pair, opt, train = tg._setup(dtype=torch.float32)
    torch.manual_seed(1)
    batches = [b for _, b in zip(range(10), train.make_loader(64, 0))]
    names = hl_name.split(",")
    nodes = [next(n for n in pair.corr.keys() if n.name == nm) for nm in names]
    cnt = [0]

    def pick():
        cnt[0] += 1
        return nodes[(cnt[0] - 1) % len(nodes)]
    pair.sample_hl_name = pick
    lln = pair.nodes_not_in_circuit[0]
    pair.sample_ll_node = lambda: lln
    step = pair.run_train_step
    if mode == "graphs":
        g = step = GraphedTrainStep(pair, opt, pair.loss_fn)
        if only_iit:
            orig = g._run_phase

            eager_keys = set(os.environ.get("EAGER_KEYS", "").split(",")) - {""}

            def sel(key, compute_loss, optimizer, step_fn):
                if key[0] != "iit" or (len(key) > 1 and key[1] in eager_keys):
                    return g._eager(compute_loss, optimizer, step_fn)
                return orig(key, compute_loss, optimizer, step_fn)
            pair._phase_runner = sel
    out_l = []
    nsteps = int(os.environ.get("NSTEPS", "12"))
    import contextlib
    ctx = step.stream_context() if (mode == "graphs" and os.environ.get("CTX") == "1") else contextlib.nullcontext()
    with ctx:
        for base, abl in (batches * 2)[:nsteps]:
            out = step(base, abl, pair.loss_fn, opt)
            out_l.append(torch.stack([out[k] for k in sorted(out)]))
    torch.cuda.synchronize()
    if os.environ.get("PARAMS"):
        return torch.stack(out_l).cpu(), {n: p.detach().clone() for n, p in pair.ll_model.named_parameters()}
    return torch.stack(out_l).cpu()


if os.environ.get("PARAMS"):
    name = sys.argv[1]
    le, pe = run("eager", name, True)
    lg, pg = run("graphs", name, True)
    print("losses", [f"{float(x):.2e}" for x in (le - lg).abs().max(1).values])
    for n in pe:
        d = (pe[n] - pg[n]).abs()
        if d.max() > 0:
            print(f"  {n:28s} max|d| {float(d.max()):.3e} frac {float((d > 0).float().mean()):.3f}")
    sys.exit(0)
for name in (sys.argv[1:] or ["hook_s_inhibition,all_nodes_hook"]):
    e = run("eager", name, True)
    gg = run("graphs", name, True)
    print(name, "iit-only graphs: max|d| per step", [f"{float(x):.2e}" for x in (e - gg).abs().max(1).values],
          flush=True)
