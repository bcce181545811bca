"""The PVR ResNet-18's 3x3 / stride-1 convolutions (B = 256, 84 x 84 inputs) on the repo's implicit-GEMM kernel
(csrc/conv_nhwc.hip, every tile) against the library convolution (MIOpen / CK through F.conv2d), forward and input
gradient and weight gradient, graph-timed in isolation on random bf16 NHWC operands.

    python scripts/bench_conv.py
"""
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

SHAPES = [("layer1", 64, 64, 21), ("layer2", 128, 128, 11), ("layer3", 256, 256, 6), ("layer4", 512, 512, 3)]


def main():
    from iit_amd.ops import gemm_dispatch as gd
    from iit_amd.ops import hip_kernels as K
    from iit_amd.ops.conv import _name, _tile_splits
    CL = torch.channels_last
    N = int(os.environ.get("BATCH", "256"))
    for name, Cin, Cout, hw in SHAPES:
        torch.manual_seed(0)
        x = torch.randn(N, Cin, hw, hw, device="cuda").to(torch.bfloat16).contiguous(memory_format=CL)
        w = (torch.randn(Cout, Cin, 3, 3, device="cuda") / 24).to(torch.bfloat16).contiguous(memory_format=CL)
        y = torch.empty(N, Cout, hw, hw, device="cuda", dtype=torch.bfloat16).contiguous(memory_format=CL)
        dy = torch.randn_like(y)
        wf = w  # the transposed kernel reads the forward weight in place
        dx = torch.empty_like(x)
        row = {"layer": name, "N": N, "Cin": Cin, "Cout": Cout, "HW": hw,
               "GFLOP": round(2 * N * hw * hw * Cout * 9 * Cin / 1e9, 2)}
        fwd = {"lib": lambda: F.conv2d(x, w, None, 1, 1)}
        bwd = {"lib": lambda: torch.nn.grad.conv2d_input(x.shape, w, dy, 1, 1)}
        for t, sp in _tile_splits(N, hw, hw, Cin, hw, hw, Cout):
            fwd[_name(t, sp)] = lambda t=t, sp=sp: K.conv3x3(x, w, y, N, hw, hw, Cin, Cout, False, t, sp)
        for t, sp in _tile_splits(N, hw, hw, Cout, hw, hw, Cin, 3, 1, 1, True):
            bwd[_name(t, sp)] = lambda t=t, sp=sp: K.conv3x3(dy, wf, dx, N, hw, hw, Cout, Cin, True, t, sp)
        dwt = torch.empty(Cout, Cin, 3, 3, device="cuda", dtype=torch.float32).contiguous(memory_format=CL)
        wgr = {"lib": lambda: torch.ops.aten.convolution_backward(dy, x, w, None, (1, 1), (1, 1), (1, 1), False, (0, 0),
                                                                   1, (False, True, False))}
        for t in K.CONV_WG_TILES:
            for sp in K.conv3x3_wgrad_splits(N * hw * hw):
                if K.conv3x3_wgrad_ok(N, hw, hw, Cin, Cout, t, sp):
                    wgr[f"hip{t}k{sp}"] = lambda t=t, sp=sp: K.conv3x3_wgrad(dy, x, dwt, N, hw, hw, Cin, Cout, False,
                                                                             t, sp)
        for tag, cands in (("fwd", fwd), ("dgrad", bwd), ("wgrad", wgr)):
            times = {k: min(gd._time(f, reps=20) for _ in range(3)) for k, f in cands.items()}
            row[tag] = {k: round(v, 1) for k, v in sorted(times.items(), key=lambda kv: kv[1])[:5]}
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
