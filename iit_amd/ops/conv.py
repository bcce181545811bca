"""NHWC bf16 convolutions (kernel 3 x 3 / pad 1 or 1 x 1 / pad 0, stride 1 or 2) on the repo's implicit-GEMM MFMA
kernels (``csrc/conv_nhwc.hip``).

The PVR task's low-level ResNet-18 (``/root/reference/iit/tasks/mnist_pvr/get_alignment.py:9-15``, trained by
``/root/reference/train.py:16-23``) spends its convolution time in the BasicBlock convolutions: the 3 x 3 stride-1
ones, the first 3 x 3 of layers 2-4 (stride 2) and the 1 x 1 stride-2 downsamples.  All three passes run as implicit
GEMMs on the LDS-DMA kernel:

* forward: ``Y [N Ho Wo][Cout] = im2col(x) W^T`` -- the im2col rows gathered by the DMA's per-lane addresses, the
  padding read from a zero page; optionally with per-tile column statistics of Y for the consuming BatchNorm;
* input gradient: the transposed convolution on ``dY`` with the forward weight read k-major in place, or with a
  re-laid k-contiguous copy where that measures faster including the copy (stride 2: the taps that do not divide read
  the zero page);
* weight gradient: ``dW [Cout][k k Cin] = dY^T im2col(x)`` (reduction over the output pixels, deterministic reduction
  split-K), written in fp32 straight into the parameter's arena gradient slot (no bf16 ``dW``, no accumulate pass).

Per problem shape and pass the kernel's tiles and K-splits compete with the library's convolution once (graph-timed,
outside capture, like :mod:`iit_amd.ops.gemm_dispatch`) and the faster runs; ``IIT_CONV_HIP=0`` keeps the library
everywhere, ``=1`` forces the repo's kernels wherever they apply.  (The 7 x 7 stem with its 3 input channels is not
covered: a K-tile is 64 channels of one tap.)
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
# the library's convolution is chosen over the repo's kernels only when it is faster in isolation by this fraction
# (IIT_CONV_LIB_MARGIN): MIOpen's find mode picks a solver per process, so its isolated time varies from run to run
# (layer1 forward 21.8-33.2 us against the repo kernel's 19.0-24.4), and a library call adds its own fills / casts
LIB_MARGIN = float(os.environ.get("IIT_CONV_LIB_MARGIN", "0.15"))
# (pass, N, H, W, Cin, Cout, k, stride) -> (choice: (tile, splits) | None = the library, {candidate: us})
DECISIONS: Dict[Tuple, Tuple[Optional[Tuple[int, int]], Dict[str, float]]] = {}


class stats_for_bn:
    """Context: convolutions issued inside feed a training-mode BatchNorm (their outputs carry ``_iit_cstat``)."""

    def __init__(self, on: bool):
        self.on = bool(on) and CONV_STATS

    def __enter__(self):
        self.prev = _WANT_STATS[0]
        _WANT_STATS[0] = self.on

    def __exit__(self, *exc):
        _WANT_STATS[0] = self.prev


# geometries offered to the kernels, "k{kernel}s{stride}" (IIT_CONV_GEOMS, comma-separated).  Default: the 3 x 3
# stride-1 and the 1 x 1 stride-2 (downsample) convolutions; the 3 x 3 stride-2 ones measured slower in the PVR step
# (7.92-7.94 vs 7.83-7.85 ms, profiles/pvr_step_r6.txt: their transposed input gradient reads the zero page for 3 of 4
# taps) and stay opt-in with k1s1
GEOMS = set(os.environ.get("IIT_CONV_GEOMS", "k3s1,k1s2").split(","))


def geometry(conv: torch.nn.Conv2d) -> Optional[Tuple[int, int, int]]:
    """(kernel, stride, pad) when the kernels cover the convolution's geometry -- 3 x 3 pad 1 or 1 x 1 pad 0, stride
    1 or 2, no dilation / groups / bias -- else None."""
    k, s, pd = conv.kernel_size, conv.stride, conv.padding
    if k not in ((3, 3), (1, 1)) or s not in ((1, 1), (2, 2)) or pd != (k[0] // 2, k[0] // 2):
        return None
    if conv.dilation != (1, 1) or conv.groups != 1 or conv.bias is not None or conv.padding_mode != "zeros":
        return None
    if f"k{k[0]}s{s[0]}" not in GEOMS:
        return None
    return k[0], s[0], pd[0]


def covered(x: torch.Tensor, conv: torch.nn.Conv2d) -> bool:
    """A covered geometry (:func:`geometry`) on a channels-last CUDA activation whose channel counts fit the kernels
    (Cin, Cout multiples of 64)."""
    if POLICY == "0" or not K.available() or geometry(conv) is None:
        return False
    return (x.is_cuda and x.dim() == 4 and x.is_contiguous(memory_format=CL) and x.shape[1] % 64 == 0
            and conv.out_channels % 64 == 0)


def _out_hw(H: int, W: int, k: int, s: int, pad: int) -> Tuple[int, int]:
    return (H + 2 * pad - k) // s + 1, (W + 2 * pad - k) // s + 1


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
    if best == "lib" and LIB_MARGIN > 0:  # the library only when it wins by the margin (its isolated time under-prices it)
        hip_best = min((t for n, t in times.items() if n != "lib"), default=None)
        if hip_best is not None and times["lib"] > hip_best * (1.0 - LIB_MARGIN):
            best = min((n for n in times if n != "lib"), key=times.get)
    DECISIONS[key] = (cands[best][0], times)
    return cands[best][0]


def _name(tile: int, splits: int) -> str:
    return f"hip{tile}" + (f"k{splits}" if splits > 1 else "")


def _tile_splits(N, SH, SW, Cs, OH, OW, Co, k=3, s=1, pad=1, transposed=False):
    """(tile, K-splits) candidates of the forward / input-gradient kernel: every tile, unsplit and split into 2..9
    equal K ranges (the reduction split: more workgroups for the few-tile deep layers, e.g. layer4's 2304 x 512
    output over K = 4608)."""
    return [(t, sp) for t in range(K.conv3x3_tiles()) for sp in (1, 2, 3, 4, 6, 8, 9)
            if K.conv2d_ok(N, SH, SW, Cs, OH, OW, Co, k, s, pad, transposed, t, sp)]


def _fwd_choice(x, w, k, s, pad):
    N, Cin, H, W = x.shape
    Cout = w.shape[0]
    key = ("fwd", N, H, W, Cin, Cout, k, s)
    if key in DECISIONS:
        return DECISIONS[key][0]
    OH, OW = _out_hw(H, W, k, s, pad)
    y = torch.empty(N, Cout, OH, OW, dtype=BF16, device=x.device, memory_format=CL)
    cands = {_name(t, sp): ((t, sp), lambda t=t, sp=sp: K.conv2d(x, w, y, N, H, W, Cin, OH, OW, Cout, k, s, pad,
                                                                 False, t, sp))
             for t, sp in _tile_splits(N, H, W, Cin, OH, OW, Cout, k, s, pad)}
    cands["lib"] = (None, lambda: F.conv2d(x, w, None, s, pad))
    return _decide(key, cands)


def _relaid(w: torch.Tensor) -> torch.Tensor:
    """[Cout, Cin, k, k] (memory [Cout][k][k][Cin]) -> memory [Cin][k][k][Cout]: the k-contiguous transposed weight."""
    return w.permute(1, 0, 2, 3).contiguous(memory_format=CL)


def _dgrad_choice(dy, w, x_shape, k, s, pad):
    """(tile, splits, mode): mode 1 = the transposed kernel reads the forward weight k-major in place, 2 = it reads a
    re-laid k-contiguous copy (faster per call; the candidate's time includes making the copy)."""
    N, Cout, OH, OW = dy.shape
    Cin, H, W = x_shape[1], x_shape[2], x_shape[3]
    key = ("dgrad", N, H, W, Cin, Cout, k, s)
    if key in DECISIONS:
        return DECISIONS[key][0]
    dx = torch.empty(N, Cin, H, W, dtype=BF16, device=dy.device, memory_format=CL)
    cands = {}
    for t, sp in _tile_splits(N, OH, OW, Cout, H, W, Cin, k, s, pad, True):
        cands[_name(t, sp)] = ((t, sp, 1), lambda t=t, sp=sp: K.conv2d(dy, w, dx, N, OH, OW, Cout, H, W, Cin, k, s,
                                                                         pad, 1, t, sp))
        cands[_name(t, sp) + "c"] = ((t, sp, 2), lambda t=t, sp=sp: K.conv2d(dy, _relaid(w), dx, N, OH, OW, Cout, H,
                                                                             W, Cin, k, s, pad, 2, t, sp))
    cands["lib"] = (None, lambda: torch.nn.grad.conv2d_input(x_shape, w, dy, s, pad))
    return _decide(key, cands)


def _wgrad_choice(dy, x, w16, k, s, pad):
    N, Cin, H, W = x.shape
    Cout, OH, OW = dy.shape[1], dy.shape[2], dy.shape[3]
    key = ("wgrad", N, H, W, Cin, Cout, k, s)
    if key in DECISIONS:
        return DECISIONS[key][0]
    dw = torch.empty(Cout, Cin, k, k, dtype=torch.float32, device=x.device, memory_format=CL)
    cands = {}
    pixels = N * OH * OW
    for t in K.CONV_WG_TILES:
        for sp in K.conv3x3_wgrad_splits(pixels) if pixels % 64 == 0 else ():
            if K.conv2d_wgrad_ok(N, H, W, Cin, OH, OW, Cout, k, s, pad, t, sp):
                cands[f"hip{t}k{sp}"] = ((t, sp), lambda t=t, sp=sp: K.conv2d_wgrad(
                    dy, x, dw, N, H, W, Cin, OH, OW, Cout, k, s, pad, False, t, sp))
    cands["lib"] = (None, lambda: torch.ops.aten.convolution_backward(
        dy, x, w16, None, (s, s), (pad, pad), (1, 1), False, (0, 0), 1, (False, True, False)))
    return _decide(key, cands)


class ConvFn(Function):
    """``conv2d(x, W, stride s, pad)`` for an arena weight ``W`` (fp32 master, bf16 mirror ``flat.shadow_view``):
    forward / input gradient / weight gradient each on the repo's kernel or the library, whichever measured faster
    for the shape; the weight gradient lands in W's fp32 arena slot (stored when the slot is claimable, else added)."""

    @staticmethod
    def forward(ctx, x, W, flat, want_stats=False, geom=(3, 1, 1)):
        k, s, pad = geom
        w = flat.shadow_view(W)
        N, Cin, H, Wd = x.shape
        Cout = w.shape[0]
        OH, OW = _out_hw(H, Wd, k, s, pad)
        ch = _fwd_choice(x, w, k, s, pad)
        cstat = None
        if ch is None:
            y = F.conv2d(x, w, None, s, pad)
        else:
            y = torch.empty(N, Cout, OH, OW, dtype=BF16, device=x.device, memory_format=CL)
            if want_stats:  # per-tile column statistics for the consuming BatchNorm (3 x Cout x T fp32)
                cstat = torch.empty(3 * Cout * (N * OH * OW // K.conv3x3_rows(ch[0])), dtype=torch.float32,
                                    device=x.device)
            K.conv2d(x, w, y, N, H, Wd, Cin, OH, OW, Cout, k, s, pad, False, ch[0], ch[1], cstat=cstat)
        ctx.save_for_backward(x)
        ctx.W, ctx.flat, ctx.geom = W, flat, geom
        if cstat is None:
            cstat = torch.empty(0, dtype=torch.float32, device=x.device)
        ctx.mark_non_differentiable(cstat)
        return y, cstat

    @staticmethod
    def backward(ctx, dy, _dstat=None):
        from ..engine import grad_hooks
        (x,) = ctx.saved_tensors
        W, flat = ctx.W, ctx.flat
        k, s, pad = ctx.geom
        w = flat.shadow_view(W)
        N, Cin, H, Wd = x.shape
        Cout = w.shape[0]
        dy = dy.to(BF16).contiguous(memory_format=CL)
        OH, OW = dy.shape[2], dy.shape[3]
        dx = None
        if ctx.needs_input_grad[0]:
            ch = _dgrad_choice(dy, w, x.shape, k, s, pad)
            if ch is None:
                dx = torch.nn.grad.conv2d_input(x.shape, w, dy, s, pad)
            else:
                dx = torch.empty(N, Cin, H, Wd, dtype=BF16, device=x.device, memory_format=CL)
                K.conv2d(dy, w if ch[2] == 1 else _relaid(w), dx, N, OH, OW, Cout, H, Wd, Cin, k, s, pad, ch[2],
                         ch[0], ch[1])
        if W.requires_grad:
            ch = _wgrad_choice(dy, x, w, k, s, pad)
            if ch is None:
                from .torch_ops import _accumulate
                gw = torch.ops.aten.convolution_backward(dy, x, w, None, (s, s), (pad, pad), (1, 1), False, (0, 0), 1,
                                                        (False, True, False))[1]
                _accumulate(W, gw)
            else:
                store = flat.claim(W)  # a lazily-zeroed slot: store (beta = 0), else accumulate
                if W.grad is None:
                    flat.bind_zero(W)
                K.conv2d_wgrad(dy, x, W.grad, N, H, Wd, Cin, OH, OW, Cout, k, s, pad, not store, ch[0], ch[1])
                grad_hooks.notify(W)
        return dx, None, None, None, None


Conv3x3Fn = ConvFn  # (the stride-1 3 x 3 name of round 6's first version)


def conv(x: torch.Tensor, W: torch.Tensor, flat, geom=(3, 1, 1)) -> torch.Tensor:
    """The convolution (``geom`` = (kernel, stride, pad)) of ``x`` with the arena weight ``W`` (bf16 mirror) on the
    measured-faster implementation.  Inside :class:`stats_for_bn`, an output of the repo's kernel carries
    ``_iit_cstat`` = (records, T, rows per tile, the output's version): its BatchNorm statistics, valid while the
    tensor is not modified in place."""
    x = x.to(BF16)
    k, s, pad = geom
    if not W.is_contiguous(memory_format=CL):
        return F.conv2d(x, flat.shadow_view(W), None, s, pad)
    y, cstat = ConvFn.apply(x, W, flat, _WANT_STATS[0], tuple(geom))
    if cstat.numel():
        N, C, H, Wd = y.shape
        rows = N * H * Wd // (cstat.numel() // (3 * C))
        y._iit_cstat = (cstat, N * H * Wd // rows, rows, y._version)
    return y


def conv3x3(x: torch.Tensor, W: torch.Tensor, flat) -> torch.Tensor:
    return conv(x, W, flat, (3, 1, 1))


def report() -> str:
    lines = []
    for (kind, N, H, W, Cin, Cout, k, s), (ch, times) in sorted(DECISIONS.items()):
        ts = "  ".join(f"{n} {v:7.1f}us" for n, v in sorted(times.items(), key=lambda kv: kv[1])[:4])
        lines.append(f"{kind:5s} N={N} H={H} W={W} Cin={Cin} Cout={Cout} k={k} s={s} -> "
                     f"{'lib' if ch is None else ch}  {ts}")
    return "\n".join(lines)
