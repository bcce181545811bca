"""Shapes of the elementwise torch ops of one family-benchmark step (default llama-tiny), from torch.profiler
(record_shapes), sorted by device time -- to find the large fp32 adds / copies / fills."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.argv += [] if "--family" in sys.argv else ["--family", "llama-tiny-causal"]
import bench_families as bf  # noqa: E402


def main():
    args = bf.parse()
    dev = torch.device("cuda", 0)
    pair, opt, it, step_fn, _, _, _ = bf.setup(args, dev)
    for _ in range(2):
        step_fn(*next(it), pair.loss_fn, opt)
    torch.cuda.synchronize()
    acts = [torch.profiler.ProfilerActivity.CPU, torch.profiler.ProfilerActivity.CUDA]
    with torch.profiler.profile(activities=acts, record_shapes=True) as prof:
        step_fn(*next(it), pair.loss_fn, opt)
        torch.cuda.synchronize()
    rows = [ev for ev in prof.key_averages(group_by_input_shape=True)
            if ev.key.startswith("aten::") and ev.key not in ("aten::mm", "aten::addmm", "aten::bmm", "aten::matmul",
                                                                "aten::linear", "aten::einsum")]
    rows.sort(key=lambda ev: -ev.self_device_time_total)
    for ev in rows[:40]:
        print(f"{ev.key:22s} n={ev.count:5d} self_cuda={ev.self_device_time_total / 1e3:8.2f}ms  {str(ev.input_shapes)[:150]}")


if __name__ == "__main__":
    main()
