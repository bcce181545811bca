"""Phase-by-phase gradient comparison, graph runner vs eager, fp32 torch-op backend (tests/test_graphs.py setup):
the optimizer stashes the clipped-gradient input of every step; the first phase whose gradient differs is printed
with the parameters that differ."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import test_graphs as tg  # noqa: E402


def run(mode, n_steps=12):
    from iit_amd.engine.graphs import GraphedTrainStep
    pair, opt, train = tg._setup(dtype=torch.float32)
    torch.manual_seed(1)
    batches = [b for _, b in zip(range(10), train.make_loader(64, 0))]
    stash = {"g": torch.zeros_like(opt.flat.grad)}
    orig_step = opt.step

    def step_hook(*a, **k):
        opt.flat.rebind_grads(zero_missing=True)
        stash["g"].copy_(opt.flat.grad)
        return orig_step(*a, **k)
    opt.step = step_hook
    grads, keys = [], []
    stepper = pair.run_train_step
    if mode == "graphs":
        g = stepper = GraphedTrainStep(pair, opt, pair.loss_fn)
        orig = g._run_phase

        def wrapped(key, *a):
            full = (key, g._sig)
            how = "replay" if full in g.graphs else ("eager" if g.seen.get(full, 0) < g.warmup else "capture")
            out = orig(key, *a)
            grads.append(stash["g"].clone())
            keys.append((key, how))
            return out
        pair._phase_runner = wrapped
    else:
        orig_rp = pair.run_phase

        def rp(key, *a):
            out = orig_rp(key, *a)
            grads.append(stash["g"].clone())
            keys.append((key, "eager"))
            return out
        pair.run_phase = rp
    for i, (base, abl) in enumerate(batches * 2):
        if i >= n_steps:
            break
        stepper(base, abl, pair.loss_fn, opt)
    torch.cuda.synchronize()
    names = {}
    for n, p in pair.ll_model.named_parameters():
        if opt.flat.owns(p):
            names[n] = (opt.flat.offset_of(p), p.numel())
    return grads, keys, names


ge, ke, names = run("eager")
gg, kg, _ = run("graphs")
for i, (a, b) in enumerate(zip(ge, gg)):
    if not torch.equal(a, b):
        print(f"phase {i} {kg[i]} differs; |eager| {float(a.norm()):.6e} |graph| {float(b.norm()):.6e}")
        for n, (o, k) in names.items():
            x, y = a[o:o + k], b[o:o + k]
            if not torch.equal(x, y):
                print(f"   {n:32s} |e| {float(x.norm()):.6e} |g| {float(y.norm()):.6e} max|d| {float((x - y).abs().max()):.3e}"
                      f" nz_e {int((x != 0).sum())} nz_g {int((y != 0).sum())}")
        break
else:
    print("all phase gradients identical")
print("schedule", kg[:36])
