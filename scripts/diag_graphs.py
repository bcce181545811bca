"""Diagnose graph-vs-eager differences per phase key (GPU)."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
from test_graphs import _setup


def run(mode):
    from iit_amd.engine.graphs import GraphedTrainStep
    pair, opt, train = _setup()
    torch.manual_seed(1)
    batches = [b for _, b in zip(range(10), train.make_loader(64, 0))]
    log = []
    orig = pair.run_phase

    def logged(key, compute_loss, optimizer, step_fn):
        out = orig(key, compute_loss, optimizer, step_fn)
        log.append((key, float(out[0] if isinstance(out, tuple) else out)))
        return out
    pair.run_phase = logged
    step = pair.run_train_step
    if mode == "graphs":
        step = GraphedTrainStep(pair, opt, pair.loss_fn)
    for base, abl in batches * 3:
        step(base, abl, pair.loss_fn, opt)
    return log


a = run("eager")
a2 = run("eager")
b = run("graphs")
print("blas backend:", torch.backends.cuda.preferred_blas_library())
for i, ((ka, la), (_, la2), (kb, lb)) in enumerate(zip(a, a2, b)):
    flag = " <<<" if abs(la - lb) > 2e-3 else ""
    flag2 = " (eager-eager)" if abs(la - la2) > 2e-3 else ""
    print(i, ka, kb == ka, f"{la:.5f} {la2:.5f} {lb:.5f}{flag}{flag2}")
