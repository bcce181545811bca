"""3 x 3 / stride-1 / pad-1 NHWC bf16 convolution on the repo's implicit-GEMM MFMA kernels (``csrc/conv_nhwc.hip``).

The PVR task's low-level ResNet-18 (``/root/reference/iit/tasks/mnist_pvr/get_alignment.py:9-15``, trained by
``/root/reference/train.py:16-23``) spends most of its convolution time in the BasicBlock 3 x 3 convolutions.  All
three passes run as implicit GEMMs on the LDS-DMA kernel:

* forward: ``Y [N H W][Cout] = im2col(x) W^T`` -- the im2col rows gathered by the DMA's per-lane addresses, the
  padding read from a zero page;
* input gradient: the same kernel with the tap offsets negated, on ``dY`` and the weight re-laid [Cin][3][3][Cout];
* weight gradient: ``dW [Cout][9 Cin] = dY^T im2col(x)`` (reduction over the pixels, deterministic reduction
  split-K), written in fp32 straight into the parameter's arena gradient slot (no bf16 ``dW``, no accumulate pass).

Per problem shape and pass the kernel's tiles (and, for the weight gradient, K-splits) compete with the library's
convolution once (graph-timed, outside capture, like :mod:`iit_amd.ops.gemm_dispatch`) and the faster runs;
``IIT_CONV_HIP=0`` keeps the library everywhere, ``=1`` forces the repo's kernels wherever they apply.
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
# the forward kernel's epilogue also writes per-tile column statistics of its output when the consumer is a training
# BatchNorm (set around the conv by models/resnet.py), which then skips its statistics pass (ops/bn.py);
# IIT_BN_CONV_STATS=0 keeps the BatchNorm's own pass
CONV_STATS = os.environ.get("IIT_BN_CONV_STATS", "1") != "0"
_WANT_STATS = [False]


class stats_for_bn:
    """Context: convolutions issued inside feed a training-mode BatchNorm (their outputs carry ``_iit_cstat``)."""

    def __init__(self, on: bool):
        self.on = bool(on) and CONV_STATS

    def __enter__(self):
        self.prev = _WANT_STATS[0]
        _WANT_STATS[0] = self.on

    def __exit__(self, *exc):
        _WANT_STATS[0] = self.prev
# (pass, N, H, W, Cin, Cout) -> (choice: (tile, splits) | None = the library, {candidate: us})
DECISIONS: Dict[Tuple, Tuple[Optional[Tuple[int, int]], Dict[str, float]]] = {}


def covered(x: torch.Tensor, conv: torch.nn.Conv2d) -> bool:
    """A 3 x 3 / stride 1 / pad 1 / ungrouped, bias-free convolution of a channels-last CUDA activation whose channel
    counts fit the kernels (Cin, Cout multiples of 64)."""
    if POLICY == "0" or not K.available():
        return False
    if conv.kernel_size != (3, 3) or conv.stride != (1, 1) or conv.padding != (1, 1) or conv.dilation != (1, 1):
        return False
    if conv.groups != 1 or conv.bias is not None or conv.padding_mode != "zeros":
        return False
    return (x.is_cuda and x.dim() == 4 and x.is_contiguous(memory_format=CL) and x.shape[1] % 64 == 0
            and conv.out_channels % 64 == 0)


def _decide(key, cands) -> Optional[Tuple[int, int]]:
    """The fastest of ``cands`` ({name: (choice | None, fn)}) for ``key``, measured once outside capture."""
    d = DECISIONS.get(key)
    if d is not None:
        return d[0]
    hip = [c for c, _ in cands.values() if c is not None]
    if not hip:
        DECISIONS[key] = (None, {})
        return None
    if torch.cuda.is_current_stream_capturing():
        return hip[0] if POLICY == "1" else None  # never time inside a capture (decided at the next eager call)
    from .gemm_dispatch import _time
    if POLICY == "1":
        cands = {n: v for n, v in cands.items() if v[0] is not None}
    times = {n: min(_time(fn, reps=10) for _ in range(2)) for n, (_, fn) in cands.items()}
    best = min(times, key=times.get)
    DECISIONS[key] = (cands[best][0], times)
    return cands[best][0]


def _flip_weight(w: torch.Tensor) -> torch.Tensor:
    """[Cout, Cin, 3, 3] (memory [Cout][3][3][Cin]) -> [Cin, Cout, 3, 3] with memory [Cin][3][3][Cout]."""
    return w.permute(1, 0, 2, 3).contiguous(memory_format=CL)


def _name(tile: int, splits: int) -> str:
    return f"hip{tile}" + (f"k{splits}" if splits > 1 else "")


def _tile_splits(N, H, W, Cin, Cout):
    """(tile, K-splits) candidates of the forward / input-gradient kernel: every tile, unsplit and split into 2..9
    equal K ranges (the reduction split: more workgroups for the few-tile deep layers, e.g. layer4's 2304 x 512
    output over K = 4608)."""
    return [(t, sp) for t in range(K.conv3x3_tiles()) for sp in (1, 2, 3, 4, 6, 8, 9)
            if K.conv3x3_ok(N, H, W, Cin, Cout, t, sp)]


def _fwd_choice(x, w):
    N, Cin, H, W = x.shape
    Cout = w.shape[0]
    if ("fwd", N, H, W, Cin, Cout) in DECISIONS:
        return DECISIONS["fwd", N, H, W, Cin, Cout][0]
    y = torch.empty(N, Cout, H, W, dtype=BF16, device=x.device, memory_format=CL)
    cands = {_name(t, sp): ((t, sp), lambda t=t, sp=sp: K.conv3x3(x, w, y, N, H, W, Cin, Cout, False, t, sp))
             for t, sp in _tile_splits(N, H, W, Cin, Cout)}
    cands["lib"] = (None, lambda: F.conv2d(x, w, None, 1, 1))
    return _decide(("fwd", N, H, W, Cin, Cout), cands)


def _dgrad_choice(dy, wf, x_shape):
    N, Cout, H, W = dy.shape
    Cin = wf.shape[0]
    if ("dgrad", N, H, W, Cin, Cout) in DECISIONS:
        return DECISIONS["dgrad", N, H, W, Cin, Cout][0]
    dx = torch.empty(N, Cin, H, W, dtype=BF16, device=dy.device, memory_format=CL)
    cands = {_name(t, sp): ((t, sp), lambda t=t, sp=sp: K.conv3x3(dy, wf, dx, N, H, W, Cout, Cin, True, t, sp))
             for t, sp in _tile_splits(N, H, W, Cout, Cin)}
    w = wf.permute(1, 0, 2, 3)
    cands["lib"] = (None, lambda: torch.nn.grad.conv2d_input(x_shape, w, dy, 1, 1))
    return _decide(("dgrad", N, H, W, Cin, Cout), cands)


def _wgrad_choice(dy, x, w16):
    N, Cin, H, W = x.shape
    Cout = dy.shape[1]
    if ("wgrad", N, H, W, Cin, Cout) in DECISIONS:
        return DECISIONS["wgrad", N, H, W, Cin, Cout][0]
    dw = torch.empty(Cout, Cin, 3, 3, dtype=torch.float32, device=x.device, memory_format=CL)
    cands = {}
    for t in K.CONV_WG_TILES:
        for sp in K.conv3x3_wgrad_splits(N * H * W) if (N * H * W) % 64 == 0 else ():
            if K.conv3x3_wgrad_ok(N, H, W, Cin, Cout, t, sp):
                cands[f"hip{t}k{sp}"] = ((t, sp), lambda t=t, sp=sp: K.conv3x3_wgrad(dy, x, dw, N, H, W, Cin, Cout,
                                                                                    False, t, sp))
    cands["lib"] = (None, lambda: torch.ops.aten.convolution_backward(
        dy, x, w16, None, (1, 1), (1, 1), (1, 1), False, (0, 0), 1, (False, True, False)))
    return _decide(("wgrad", N, H, W, Cin, Cout), cands)


class Conv3x3Fn(Function):
    """``conv2d(x, W, stride 1, pad 1)`` for an arena weight ``W`` (fp32 master, bf16 mirror ``flat.shadow_view``):
    forward / input gradient / weight gradient each on the repo's kernel or the library, whichever measured faster
    for the shape; the weight gradient lands in W's fp32 arena slot (stored when the slot is claimable, else added)."""

    @staticmethod
    def forward(ctx, x, W, flat, want_stats=False):
        w = flat.shadow_view(W)
        N, Cin, H, Wd = x.shape
        Cout = w.shape[0]
        ch = _fwd_choice(x, w)
        cstat = None
        if ch is None:
            y = F.conv2d(x, w, None, 1, 1)
        else:
            y = torch.empty(N, Cout, H, Wd, dtype=BF16, device=x.device, memory_format=CL)
            if want_stats:  # per-tile column statistics for the consuming BatchNorm (3 x Cout x T fp32)
                cstat = torch.empty(3 * Cout * (N * H * Wd // K.conv3x3_rows(ch[0])), dtype=torch.float32,
                                    device=x.device)
            K.conv3x3(x, w, y, N, H, Wd, Cin, Cout, False, ch[0], ch[1], cstat=cstat)
        ctx.save_for_backward(x)
        ctx.W, ctx.flat = W, flat
        ctx.stat_rows = K.conv3x3_rows(ch[0]) if cstat is not None else 0
        if cstat is None:
            cstat = torch.empty(0, dtype=torch.float32, device=x.device)
        ctx.mark_non_differentiable(cstat)
        return y, cstat

    @staticmethod
    def backward(ctx, dy, _dstat=None):
        from ..engine import grad_hooks
        (x,) = ctx.saved_tensors
        W, flat = ctx.W, ctx.flat
        w = flat.shadow_view(W)
        N, Cin, H, Wd = x.shape
        Cout = w.shape[0]
        dy = dy.to(BF16).contiguous(memory_format=CL)
        dx = None
        if ctx.needs_input_grad[0]:
            wf = _flip_weight(w)
            ch = _dgrad_choice(dy, wf, x.shape)
            if ch is None:
                dx = torch.nn.grad.conv2d_input(x.shape, w, dy, 1, 1)
            else:
                dx = torch.empty(N, Cin, H, Wd, dtype=BF16, device=x.device, memory_format=CL)
                K.conv3x3(dy, wf, dx, N, H, Wd, Cout, Cin, True, ch[0], ch[1])
        if W.requires_grad:
            ch = _wgrad_choice(dy, x, w)
            if ch is None:
                from .torch_ops import _accumulate
                gw = torch.ops.aten.convolution_backward(dy, x, w, None, (1, 1), (1, 1), (1, 1), False, (0, 0), 1,
                                                        (False, True, False))[1]
                _accumulate(W, gw)
            else:
                store = flat.claim(W)  # a lazily-zeroed slot: store (beta = 0), else accumulate
                if W.grad is None:
                    flat.bind_zero(W)
                K.conv3x3_wgrad(dy, x, W.grad, N, H, Wd, Cin, Cout, not store, ch[0], ch[1])
                grad_hooks.notify(W)
        return dx, None, None, None


def conv3x3(x: torch.Tensor, W: torch.Tensor, flat) -> torch.Tensor:
    """The convolution of ``x`` with the arena weight ``W`` (bf16 mirror) on the measured-faster implementation.
    Inside :class:`stats_for_bn`, an output of the repo's kernel carries ``_iit_cstat`` = (records, T, rows per tile,
    the output's version): its BatchNorm statistics, valid while the tensor is not modified in place."""
    x = x.to(BF16)
    if not W.is_contiguous(memory_format=CL):
        return F.conv2d(x, flat.shadow_view(W), None, 1, 1)
    y, cstat = Conv3x3Fn.apply(x, W, flat, _WANT_STATS[0])
    if cstat.numel():
        N, C, H, Wd = y.shape
        rows = N * H * Wd // (cstat.numel() // (3 * C))
        y._iit_cstat = (cstat, N * H * Wd // rows, rows, y._version)
    return y


def report() -> str:
    lines = []
    for (kind, N, H, W, Cin, Cout), (ch, times) in sorted(DECISIONS.items()):
        ts = "  ".join(f"{k} {v:7.1f}us" for k, v in sorted(times.items(), key=lambda kv: kv[1])[:4])
        lines.append(f"{kind:5s} N={N} H={H} W={W} Cin={Cin} Cout={Cout} -> {'lib' if ch is None else ch}  {ts}")
    return "\n".join(lines)
