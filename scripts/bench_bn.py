"""The fused NHWC BatchNorm passes (csrc/bn_nhwc.hip) per PVR ResNet-18 layer shape at B = 256 (84 x 84 inputs),
in isolation: forward (stats + apply, graph-timed) and forward + backward (eager, event-timed), bf16 activations, with the HBM
floor of each (bytes / 6 TB/s) -- where the norm group's time goes.

    python scripts/bench_bn.py [--dtype bf16|fp32]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

SHAPES = [("stem", 64, 42), ("layer1", 64, 21), ("layer2", 128, 11), ("layer3", 256, 6), ("layer4", 512, 3)]


def _eager_time(fn, reps: int = 20) -> float:
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / reps * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--batch", type=int, default=256)
    args = ap.parse_args()
    from iit_amd.ops import bn as fbn
    from iit_amd.ops import gemm_dispatch as gd
    dt = torch.bfloat16 if args.dtype == "bf16" else torch.float32
    es = 2 if dt == torch.bfloat16 else 4
    dev = "cuda"
    for name, C, hw in SHAPES:
        torch.manual_seed(0)
        bn = torch.nn.BatchNorm2d(C).to(dev)
        x = torch.randn(args.batch, C, hw, hw, device=dev).to(dt).contiguous(memory_format=torch.channels_last)
        x.requires_grad_()
        g = torch.randn_like(x, memory_format=torch.channels_last)
        y = fbn.bn_act(x, bn, None, relu=True)

        def fwd():
            fbn.bn_act(x.detach(), bn, None, relu=True)

        def fwd_bwd():
            out = fbn.bn_act(x, bn, None, relu=True)
            out.backward(g)

        t_f = min(gd._time(fwd, reps=20) for _ in range(3))
        t_fb = min(_eager_time(fwd_bwd) for _ in range(3))  # (autograd is not captured: eager, events)
        nbytes = x.numel() * es
        floor_f = 3 * nbytes / 6e12 * 1e6       # stats read x; apply read x + write y
        floor_b = 7 * nbytes / 6e12 * 1e6       # + bwd stats read dy, y, x; bwd apply read dy, y, x + write dx
        print(json.dumps({"layer": name, "C": C, "HW": hw, "MB": round(nbytes / 1e6, 1), "fwd_us": round(t_f, 1),
                          "fwd_floor_us": round(floor_f, 1), "fwd_bwd_us": round(t_fb, 1),
                          "fwd_bwd_floor_us": round(floor_f + floor_b, 1)}), flush=True)
        del x, g, y


if __name__ == "__main__":
    main()
