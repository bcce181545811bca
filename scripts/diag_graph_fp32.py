"""Graph runner vs eager on the fp32 torch-op backend (tests/test_graphs.py setup): a device-side weight checksum
after every optimizer phase (no host sync), compared phase by phase; prints the first differing phases and how the
graph runner executed them (eager warm-up / capture / replay)."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import test_graphs as tg  # noqa: E402


def run(mode):
    from iit_amd.engine.graphs import GraphedTrainStep
    pair, opt, train = tg._setup(dtype=torch.float32)
    torch.manual_seed(1)
    batches = [b for _, b in zip(range(10), train.make_loader(64, 0))]
    sums, hows = [], []
    flat = opt.flat
    w = torch.arange(flat.numel, device=flat.data.device, dtype=torch.float64).remainder_(7.0).add_(1.0)

    def ck():
        sums.append(torch.stack([(flat.data.double() * w).sum(), flat.grad.double().abs().sum()]))

    step = pair.run_train_step
    if mode == "graphs":
        g = step = GraphedTrainStep(pair, opt, pair.loss_fn)
        orig = g._run_phase

        def wrapped(key, *a):
            full = (key, g._sig)
            hows.append((key, "replay" if full in g.graphs else
                         ("eager" if g.seen.get(full, 0) < g.warmup or full in g.failed else "capture")))
            out = orig(key, *a)
            ck()
            return out
        pair._phase_runner = wrapped
    else:
        orig_rp = pair.run_phase

        def rp(key, *a):
            out = orig_rp(key, *a)
            hows.append((key, "eager"))
            ck()
            return out
        pair.run_phase = rp
    for base, abl in batches * 3:
        step(base, abl, pair.loss_fn, opt)
    torch.cuda.synchronize()
    return torch.stack(sums).cpu(), hows


if os.environ.get("FILL") == "1":
    torch.use_deterministic_algorithms(True, warn_only=True)
    torch.utils.deterministic.fill_uninitialized_memory = True
elif os.environ.get("DET") == "1":
    torch.use_deterministic_algorithms(True, warn_only=True)
    torch.utils.deterministic.fill_uninitialized_memory = False
if len(sys.argv) > 1 and sys.argv[1] == "loss":
    def run_loss(mode):
        from iit_amd.engine.graphs import GraphedTrainStep
        pair, opt, train = tg._setup(dtype=torch.float32)
        torch.manual_seed(1)
        batches = [b for _, b in zip(range(10), train.make_loader(64, 0))]
        step = pair.run_train_step if mode == "eager" else GraphedTrainStep(pair, opt, pair.loss_fn)
        only = os.environ.get("ONLY")
        if mode != "eager" and only:
            orig = step._run_phase

            def sel(key, compute_loss, optimizer, step_fn, _o=orig):
                if key[0] != only:
                    return step._eager(compute_loss, optimizer, step_fn)
                return _o(key, compute_loss, optimizer, step_fn)
            pair._phase_runner = sel
        losses = []
        for base, abl in batches * 3:
            out = step(base, abl, pair.loss_fn, opt)
            losses.append(torch.stack([out[k] for k in sorted(out)]))
        torch.cuda.synchronize()
        return torch.stack(losses).cpu()
    le, lg = run_loss("eager"), run_loss("graphs")
    if os.environ.get("SAVE"):
        torch.save(le, os.environ["SAVE"])
    if os.environ.get("CMP"):
        ref = torch.load(os.environ["CMP"])
        print("eager vs saved eager:", [round(float(x), 5) for x in (le - ref).abs().max(1).values])
    print(f"fill={os.environ.get('FILL')} det={os.environ.get('DET')} only={os.environ.get('ONLY')} pool={os.environ.get('IIT_GRAPH_POOL', 'shared')} loss drift:",
          [round(float(x), 5) for x in (le - lg).abs().max(1).values])
    sys.exit(0)
e, eh = run("eager")
gs, gh = run("graphs")
print("phases", len(eh), len(gh))
bad = 0
for i in range(min(len(e), len(gs))):
    if not torch.equal(e[i], gs[i]):
        print(f"phase {i}: {gh[i]} (eager key {eh[i][0]}) weights {float(e[i][0]):.9e} vs {float(gs[i][0]):.9e}"
              f"  |grad| {float(e[i][1]):.6e} vs {float(gs[i][1]):.6e}")
        bad += 1
        if bad >= 6:
            break
print("schedule:", gh[:40])
