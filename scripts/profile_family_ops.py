"""Attribute a model family's elementwise / copy / fill kernels to Python call sites (torch.profiler with stacks).

    python scripts/profile_family_ops.py --family llama-tiny-causal --seq 512 > gpurun_out/family_ops.txt

Runs a few training steps of ``scripts/bench_families.py``'s setup under torch.profiler and prints the aten ops by
device time, grouped by their top Python frames (the op backend's call site that launched them).
"""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "scripts"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--family", default="llama-tiny-causal")
    ap.add_argument("--seq", type=int, default=512)
    ap.add_argument("--steps", type=int, default=2)
    a = ap.parse_args()
    import bench_families as bf
    args = bf.parse([f"--family={a.family}", f"--seq={a.seq}", "--steps", "1", "--warmup", "1"])
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    pair, opt, it, step_fn, _, _, _ = bf.setup(args, dev)
    for _ in range(2):
        step_fn(*next(it), pair.loss_fn, opt)
    torch.cuda.synchronize()
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True) as prof:
        for _ in range(a.steps):
            step_fn(*next(it), pair.loss_fn, opt)
        torch.cuda.synchronize()
    keep = ("aten::add", "aten::copy_", "aten::fill_", "aten::zero_", "aten::mul", "aten::cat", "aten::to",
            "aten::_to_copy", "aten::contiguous", "aten::clone", "aten::sum", "aten::where", "aten::div")
    rows = [e for e in prof.key_averages(group_by_stack_n=7) if e.key in keep and e.device_time_total > 0]
    rows.sort(key=lambda e: -e.device_time_total)
    for e in rows[:25]:
        print(f"{e.device_time_total / 1e3 / a.steps:9.2f} ms/step  {e.count / a.steps:7.1f} calls/step  {e.key}")
        for fr in (e.stack or [])[:7]:
            print("        ", fr)


if __name__ == "__main__":
    main()
