"""Uninitialised-memory check: torch.empty outputs filled with NaN (deterministic mode's
``fill_uninitialized_memory``); a step whose loss turns NaN reads memory no kernel wrote."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import test_graphs as tg  # noqa: E402

torch.use_deterministic_algorithms(True, warn_only=True)
torch.utils.deterministic.fill_uninitialized_memory = True
dtype = torch.float32 if (len(sys.argv) < 2 or sys.argv[1] == "fp32") else torch.bfloat16
mode = sys.argv[2] if len(sys.argv) > 2 else "eager"
pair, opt, train = tg._setup(dtype=dtype)
torch.manual_seed(1)
batches = [b for _, b in zip(range(10), train.make_loader(64, 0))]
step = pair.run_train_step
if mode == "graphs":
    from iit_amd.engine.graphs import GraphedTrainStep
    step = GraphedTrainStep(pair, opt, pair.loss_fn)
for i, (base, abl) in enumerate(batches * 2):
    out = step(base, abl, pair.loss_fn, opt)
    vals = {k: round(float(v), 5) for k, v in out.items()}
    w = float(opt.flat.data.abs().sum())
    print(i, vals, "weights finite" if w == w else "WEIGHTS NAN", "skipped", opt.skipped_steps, flush=True)
