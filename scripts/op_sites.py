"""Which lines of the engine issue the library / cast / elementwise ops of a family's training step: eager steps
(no graphs) under ``torch.profiler`` with stacks, ATen ops grouped by their innermost ``iit_amd`` frame.

    python scripts/op_sites.py --family mqnli-bert-base [--ops copy_,_to_copy,add,mm,addmm,linear]
"""
import argparse
import collections
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "scripts"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--family", default="mqnli-bert-base")
    ap.add_argument("--ops", default="copy_,_to_copy,add,add_,mm,addmm,linear,matmul,bmm,cat,index_select,fill_,zero_")
    ap.add_argument("--steps", type=int, default=2)
    a = ap.parse_args()
    import bench_families as bf
    args = bf.parse(["--family", a.family, "--graphs", "0"])
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    pair, opt, it, step_fn, _, _, _ = bf.setup(args, dev)
    for _ in range(3):
        base, abl = next(it)
        step_fn(base, abl, pair.loss_fn, opt)
    torch.cuda.synchronize()
    wanted = {f"aten::{o}" for o in a.ops.split(",")}
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True) as prof:
        for _ in range(a.steps):
            base, abl = next(it)
            step_fn(base, abl, pair.loss_fn, opt)
        torch.cuda.synchronize()
    sites = collections.defaultdict(lambda: [0, 0.0])
    for ev in prof.events():
        if ev.name not in wanted:
            continue
        frames = [f for f in (ev.stack or []) if "iit_amd" in f]
        site = frames[0] if frames else "(no iit_amd frame)"
        s = sites[(ev.name, site)]
        s[0] += 1
        s[1] += ev.device_time_total if hasattr(ev, "device_time_total") else ev.cuda_time_total
    print(f"{'op':22s} {'calls/step':>10s} {'dev us/step':>11s}  site")
    for (name, site), (n, t) in sorted(sites.items(), key=lambda kv: -kv[1][1])[:40]:
        print(f"{name:22s} {n / a.steps:10.1f} {t / a.steps:11.1f}  {site}")


if __name__ == "__main__":
    main()
