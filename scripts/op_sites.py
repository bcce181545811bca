"""Which lines of the engine issue the ATen ops of a family's training step (library GEMMs, casts, copies, fills,
adds): eager steps (no graphs) under a TorchDispatchMode that attributes every op to its innermost ``iit_amd`` frame
(the profiler's stacks are empty on this ROCm build), with call counts and output bytes per step.

    python scripts/op_sites.py --family mqnli-bert-base [--ops mm,addmm,_to_copy,copy_,add,fill_]
"""
import argparse
import collections
import os
import sys
import traceback

import torch
from torch.utils._python_dispatch import TorchDispatchMode

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "scripts"))


class Sites(TorchDispatchMode):
    def __init__(self, wanted):
        super().__init__()
        self.wanted = wanted
        self.rows = collections.defaultdict(lambda: [0, 0])

    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        out = func(*args, **(kwargs or {}))
        name = func.overloadpacket.__name__
        if name in self.wanted:
            site = "(no iit_amd frame)"
            for fr in reversed(traceback.extract_stack()[:-1]):
                if "iit_amd" in fr.filename:
                    site = f"{os.path.relpath(fr.filename, ROOT)}:{fr.lineno} {fr.name}"
                    break
            nbytes = sum(t.numel() * t.element_size() for t in (out if isinstance(out, (tuple, list)) else [out])
                         if isinstance(t, torch.Tensor))
            r = self.rows[(name, site)]
            r[0] += 1
            r[1] += nbytes
        return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--family", default="mqnli-bert-base")
    ap.add_argument("--ops", default="mm,addmm,bmm,matmul,linear,_to_copy,copy_,add,add_,fill_,zero_,cat,index_select,"
                                     "clone,mul,sum")
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--dtype", default="fp32", help="pvr-resnet18: bf16 = channels-last bf16 autocast (as the bench)")
    a = ap.parse_args()
    import contextlib
    import bench_families as bf
    args = bf.parse(["--family", a.family, "--graphs", "0", "--dtype", a.dtype])
    dev = torch.device("cuda", 0) if torch.cuda.is_available() else torch.device("cpu")
    if dev.type == "cuda":
        torch.cuda.set_device(0)
    pair, opt, it, step_fn, _, _, _ = bf.setup(args, dev)
    amp = (lambda: torch.autocast("cuda", dtype=torch.bfloat16, cache_enabled=False)) \
        if a.dtype == "bf16" and dev.type == "cuda" else contextlib.nullcontext
    for _ in range(3):
        base, abl = next(it)
        with amp():
            step_fn(base, abl, pair.loss_fn, opt)
    if dev.type == "cuda":
        torch.cuda.synchronize()
    mode = Sites(set(a.ops.split(",")))
    with mode:
        for _ in range(a.steps):
            base, abl = next(it)
            with amp():
                step_fn(base, abl, pair.loss_fn, opt)
    if dev.type == "cuda":
        torch.cuda.synchronize()
    print(f"{'op':14s} {'calls/step':>10s} {'MB out/step':>11s}  site")
    for (name, site), (n, b) in sorted(mode.rows.items(), key=lambda kv: -kv[1][1])[:50]:
        print(f"{name:14s} {n / a.steps:10.1f} {b / a.steps / 1e6:11.2f}  {site}")


if __name__ == "__main__":
    main()
