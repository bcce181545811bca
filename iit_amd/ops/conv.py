"""3 x 3 / stride-1 / pad-1 NHWC bf16 convolution on the repo's implicit-GEMM MFMA kernel (``csrc/conv_nhwc.hip``).

The PVR task's low-level ResNet-18 (``/root/reference/iit/tasks/mnist_pvr/get_alignment.py:9-15``, trained by
``/root/reference/train.py:16-23``) spends most of its convolution time in the BasicBlock 3 x 3 convolutions.  The
forward and the input gradient run as implicit GEMMs on the LDS-DMA kernel (the im2col rows gathered by the DMA's
per-lane addresses, the padding read from a zero page); the weight gradient stays on MIOpen's backward-weights
kernel.  Per problem shape the kernel's tiles compete with the library's convolution once (graph-timed, outside
capture, like :mod:`iit_amd.ops.gemm_dispatch`) and the faster runs; ``IIT_CONV_HIP=0`` keeps the library,
``=1`` forces the repo's kernel (best tile) wherever it applies.
"""
from __future__ import annotations

import os
from typing import Dict, Optional, Tuple

import torch
import torch.nn.functional as F
from torch.autograd import Function

from . import hip_kernels as K

BF16 = torch.bfloat16
CL = torch.channels_last
POLICY = os.environ.get("IIT_CONV_HIP", "auto")
DECISIONS: Dict[Tuple, Tuple[Optional[int], Dict[str, float]]] = {}  # (N,H,W,Cin,Cout,flip) -> (tile | None, times)


def covered(x: torch.Tensor, conv: torch.nn.Conv2d) -> bool:
    """A 3 x 3 / stride 1 / pad 1 / ungrouped, bias-free convolution of a channels-last bf16 CUDA activation whose
    channel counts fit the kernel (Cin, Cout multiples of 64)."""
    if POLICY == "0" or not K.available():
        return False
    if conv.kernel_size != (3, 3) or conv.stride != (1, 1) or conv.padding != (1, 1) or conv.dilation != (1, 1):
        return False
    if conv.groups != 1 or conv.bias is not None or conv.padding_mode != "zeros":
        return False
    return (x.is_cuda and x.dim() == 4 and x.is_contiguous(memory_format=CL) and x.shape[1] % 64 == 0
            and conv.out_channels % 64 == 0)


def _lib_conv(x, w):
    return F.conv2d(x, w, None, 1, 1)


def _decide(x, w, flip: bool) -> Optional[int]:
    """The fastest of the kernel's tiles and the library for this shape (None = the library)."""
    N, Cin, H, W = x.shape
    Cout = w.shape[0]
    key = (N, H, W, Cin, Cout, flip)
    d = DECISIONS.get(key)
    if d is not None:
        return d[0]
    tiles = [t for t in range(K.conv3x3_tiles()) if K.conv3x3_ok(N, H, W, Cin, Cout, t)]
    if not tiles:
        DECISIONS[key] = (None, {})
        return None
    if POLICY == "1" and torch.cuda.is_current_stream_capturing():
        return tiles[0]
    if torch.cuda.is_current_stream_capturing():
        return None  # never time inside a capture: the library this time, decided at the next eager call
    from .gemm_dispatch import _time
    y = torch.empty(N, Cout, H, W, dtype=BF16, device=x.device, memory_format=CL)
    cands = {f"hip{t}": (lambda t=t: K.conv3x3(x, w, y, N, H, W, Cin, Cout, flip, t)) for t in tiles}
    if POLICY != "1" and not flip:
        cands["lib"] = lambda: _lib_conv(x, w)
    times = {n: min(_time(f, reps=10) for _ in range(2)) for n, f in cands.items()}
    best = min(times, key=times.get)
    tile = None if best == "lib" else int(best[3:])
    DECISIONS[key] = (tile, times)
    return tile


def _flip_weight(w: torch.Tensor) -> torch.Tensor:
    """[Cout, Cin, 3, 3] (memory [Cout][3][3][Cin]) -> [Cin, Cout, 3, 3] with memory [Cin][3][3][Cout]."""
    return w.permute(1, 0, 2, 3).contiguous(memory_format=CL)


class Conv3x3Fn(Function):
    """``conv2d(x, w, stride 1, pad 1)`` with the repo's implicit-GEMM kernel for the forward (tile ``tile``) and,
    when it wins, for the input gradient; the weight gradient is the library's backward-weights convolution."""

    @staticmethod
    def forward(ctx, x, w, tile):
        N, Cin, H, W = x.shape
        Cout = w.shape[0]
        y = torch.empty(N, Cout, H, W, dtype=BF16, device=x.device, memory_format=CL)
        K.conv3x3(x, w, y, N, H, W, Cin, Cout, False, tile)
        ctx.save_for_backward(x, w)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        N, Cin, H, W = x.shape
        Cout = w.shape[0]
        dy = dy.to(BF16).contiguous(memory_format=CL)
        dx = dw = None
        if ctx.needs_input_grad[0]:
            wf = _flip_weight(w)
            tile = _decide(dy, wf, True) if POLICY != "0" else None
            if tile is not None:
                dx = torch.empty(N, Cin, H, W, dtype=BF16, device=x.device, memory_format=CL)
                K.conv3x3(dy, wf, dx, N, H, W, Cout, Cin, True, tile)
        if ctx.needs_input_grad[1] or dx is None and ctx.needs_input_grad[0]:
            mask = (dx is None and ctx.needs_input_grad[0], bool(ctx.needs_input_grad[1]), False)
            gi, gw, _ = torch.ops.aten.convolution_backward(dy, x, w, None, (1, 1), (1, 1), (1, 1), False, (0, 0), 1,
                                                           mask)
            if dx is None:
                dx = gi
            dw = gw
        return dx, dw, None


def conv3x3(x: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    """The convolution on the repo's kernel when it is the measured winner for the shape, else the library's."""
    x = x.to(BF16)
    if not w.is_contiguous(memory_format=CL):
        return _lib_conv(x, w)
    tile = _decide(x, w, False)
    if tile is None:
        return _lib_conv(x, w)
    return Conv3x3Fn.apply(x, w, tile)


def report() -> str:
    lines = []
    for (N, H, W, Cin, Cout, flip), (tile, times) in sorted(DECISIONS.items()):
        ts = "  ".join(f"{k} {v:7.1f}us" for k, v in sorted(times.items(), key=lambda kv: kv[1]))
        lines.append(f"N={N} H={H} W={W} Cin={Cin} Cout={Cout} {'dgrad' if flip else 'fwd  '} -> "
                     f"{'lib' if tile is None else f'hip{tile}'}  {ts}")
    return "\n".join(lines)
