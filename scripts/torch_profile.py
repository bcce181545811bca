"""Attribute the non-HIP (torch) kernels of a bench step to Python call sites.

    python scripts/torch_profile.py --steps 3 > gpurun_out/torch_profile.txt

Prints the top ops by device time, then for the elementwise / copy ops the
Python stacks that launched them (torch.profiler with_stack).
"""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--model", default="gpt2-small")
    ap.add_argument("--batch", type=int, default=256)
    a = ap.parse_args()
    args = argparse.Namespace(gpus=1, steps=a.steps, warmup=2, batch=a.batch, model=a.model, engine="native",
                              dtype="bf16", graphs=0, profile_dir=None)
    dev = torch.device("cuda", 0)
    pair, opt, loss_fn, it, step_fn, _, _ = bench.setup(args, dev)
    for _ in range(3):
        step_fn(*next(it), loss_fn, opt)
    torch.cuda.synchronize()
    acts = [torch.profiler.ProfilerActivity.CPU, torch.profiler.ProfilerActivity.CUDA]
    with torch.profiler.profile(activities=acts, with_stack=True, record_shapes=True) as prof:
        for _ in range(a.steps):
            step_fn(*next(it), loss_fn, opt)
        torch.cuda.synchronize()
    print(prof.key_averages().table(sort_by="self_cuda_time_total", row_limit=40, max_name_column_width=60))
    print(prof.key_averages(group_by_input_shape=True).table(sort_by="self_cuda_time_total", row_limit=40,
                                                             max_name_column_width=40, max_shapes_column_width=60))
    print(prof.key_averages(group_by_stack_n=6).table(sort_by="self_cuda_time_total", row_limit=60,
                                                      max_name_column_width=40))


if __name__ == "__main__":
    main()
