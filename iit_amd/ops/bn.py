"""Fused BatchNorm (+ residual add) (+ ReLU) on channels-last bf16 or fp32 activations (``csrc/bn_nhwc.hip``).

The PVR ResNet-18's ``BatchNorm2d -> ReLU`` and ``BatchNorm2d -> + identity -> ReLU`` chains
(``/root/reference/iit/tasks/mnist_pvr/get_alignment.py:9-15``: torchvision's BasicBlock) as one autograd op: two
kernel launches forward (per-channel statistics, then normalise + add + ReLU + running-statistics update) and two
backward (per-channel sums of dz and dz * xhat, then dx, the residual's gradient and the parameter gradients) in
place of MIOpen's BatchNorm kernels, the ReLU, the residual add and ``num_batches_tracked += 1``.  Semantics are
``torch.nn.BatchNorm2d``'s (batch statistics with the biased variance in training, running statistics updated with
the unbiased variance and ``momentum``; running statistics in eval); the running buffers and ``num_batches_tracked``
are updated on the device by the forward kernel, so a graph-captured step replays them.

Used by :class:`iit_amd.models.resnet.BasicBlock` / :class:`ResNet` when the activation is a CUDA bf16
channels-last tensor, the BatchNorm has ``momentum`` set and affine parameters, no hook on the fused sites is live,
and ``IIT_FUSED_BN`` is not ``0``; everything else takes the module path unchanged.
"""
from __future__ import annotations

import os
from typing import Optional

import torch
from torch.autograd import Function

from . import hip_kernels as K

BF16 = torch.bfloat16
F32 = torch.float32


def enabled() -> bool:
    return os.environ.get("IIT_FUSED_BN", "1") != "0" and torch.cuda.is_available() and K.available()


def covered(x: torch.Tensor, bn: torch.nn.BatchNorm2d, res: Optional[torch.Tensor] = None) -> bool:
    if not (x.is_cuda and x.dtype in (BF16, F32) and x.dim() == 4
            and x.is_contiguous(memory_format=torch.channels_last)):
        return False
    if x.dtype == F32 and os.environ.get("IIT_FUSED_BN_F32", "1") == "0":
        return False
    C = x.shape[1]
    if C % 8 or C < 8 or 256 % (C // 8) or not bn.affine or bn.momentum is None:
        return False
    if bn.weight.dtype != F32 or bn.bias.dtype != F32 or not bn.track_running_stats or bn.running_mean is None:
        return False
    if res is not None and not (res.shape == x.shape and res.dtype == x.dtype
                                and res.is_contiguous(memory_format=torch.channels_last)):
        return False
    return True


def _ws(bn: torch.nn.BatchNorm2d, C: int, device) -> torch.Tensor:
    """The module's self-re-arming reduction accumulator: [slots][2C] floats + a ticket, zero at creation; every kernel call
    leaves it zero again (csrc/bn_nhwc.hip).  Shared by the forward and backward of every call on the stream."""
    n = K.bn_ws_floats(C)
    ws = bn.__dict__.get("_iit_bn_ws")
    if ws is None or ws.numel() < n or ws.device != device:
        ws = bn.__dict__["_iit_bn_ws"] = torch.zeros(n, dtype=F32, device=device)
    return ws


class BNActFn(Function):
    @staticmethod
    def forward(ctx, x, w, b, res, bn, relu, src=None, spec=None, cstat=None):
        C = x.shape[1]
        M = x.numel() // C
        H, W = x.shape[2], x.shape[3]
        training = bn.training
        y = torch.empty_like(x, memory_format=torch.channels_last)
        save = torch.empty(2 * C, dtype=F32, device=x.device)
        if cstat is not None:  # statistics from the producing conv's epilogue: no statistics pass over x
            K.bn_fwd_tiles(x, res, y, cstat[0], cstat[1], cstat[2], bn.running_mean, bn.running_var, w, b, M, C,
                           float(bn.eps), relu, save, float(bn.momentum), bn.num_batches_tracked)
        else:
            K.bn_fwd(x, res, y, _ws(bn, C, x.device), bn.running_mean, bn.running_var, w, b, M, C, float(bn.eps),
                     relu, training, save, float(bn.momentum), bn.num_batches_tracked, src=src, spec=spec, H=H, W=W)
        ctx.save_for_backward(x, y if relu else None, save, w)
        ctx.cfg = (M, C, training, res is not None, H, W)
        ctx.bn = bn
        ctx.splice = (src, spec)
        return y

    @staticmethod
    def backward(ctx, dy):
        if dy is None:
            return None, None, None, None, None, None, None, None, None
        from .hip_ops import _done, _grad_slot
        x, y, save, w = ctx.saved_tensors
        M, C, training, has_res, H, W = ctx.cfg
        src, spec = ctx.splice
        bn = ctx.bn
        dy = dy.to(x.dtype).contiguous(memory_format=torch.channels_last)
        dx = torch.empty_like(x, memory_format=torch.channels_last)
        dres = torch.empty_like(x, memory_format=torch.channels_last) if has_res else None
        coef = torch.empty(2 * C, dtype=F32, device=x.device)
        # the weight / bias gradients are added into their gradient buffers by the kernel (no autograd accumulation)
        dw, db = _grad_slot(bn.weight), _grad_slot(bn.bias)
        K.bn_bwd(dy, y, x, save, w, _ws(bn, C, x.device), coef, M, C, training, dx, dres, dw, db, src=src, spec=spec,
                 H=H, W=W)
        _done(bn.weight, bn.bias)
        return dx, None, None, dres, None, None, None, None, None


def bn_act(x: torch.Tensor, bn: torch.nn.BatchNorm2d, res: Optional[torch.Tensor] = None,
           relu: bool = True, splice=None) -> Optional[torch.Tensor]:
    """``relu?(bn(x') (+ res))`` fused (the caller checked :func:`covered`); ``splice`` = (index, src): x' = ``x``
    with ``x'[index] = src[index]`` (an interchange splice of the producing conv's hook, read in place by the
    kernels; the spliced elements get no gradient).  None when the splice's index is not expressible."""
    if splice is None:
        st = getattr(x, "_iit_cstat", None)
        if st is not None and not (bn.training and x.dtype == BF16 and st[3] == x._version
                                   and st[1] * st[2] * x.shape[1] == x.numel()):
            st = None  # (eval mode, or the activation was modified in place after its conv)
        return BNActFn.apply(x, bn.weight, bn.bias, res, bn, relu, None, None, st)
    from .splice import patch_spec
    index, src = splice
    src = src.to(device=x.device, dtype=x.dtype)
    spec = patch_spec(index, tuple(x.shape), src)
    if spec is None or tuple(d[0] for d in spec.dims) != tuple(x.shape):
        return None
    return BNActFn.apply(x, bn.weight, bn.bias, res, bn, relu, src, spec)


class MaxPool3s2Fn(Function):
    """``max_pool2d(x, 3, 2, 1)`` on a channels-last bf16 / fp32 activation (``csrc/bn_nhwc.hip``): one byte of argmax per
    output element and a gather-form backward (torch's NHWC pool keeps int64 indices and scatters its gradient)."""

    @staticmethod
    def forward(ctx, x):
        N, C, H, W = x.shape
        OH, OW = (H - 1) // 2 + 1, (W - 1) // 2 + 1
        y = torch.empty(N, C, OH, OW, dtype=x.dtype, device=x.device, memory_format=torch.channels_last)
        idx = torch.empty(N, OH, OW, C, dtype=torch.uint8, device=x.device)
        K.maxpool3s2_fwd(x, y, idx, N, H, W, C)
        ctx.save_for_backward(idx)
        ctx.shape = (N, C, H, W)
        ctx.dtype = x.dtype
        return y

    @staticmethod
    def backward(ctx, dy):
        (idx,) = ctx.saved_tensors
        N, C, H, W = ctx.shape
        dy = dy.to(ctx.dtype).contiguous(memory_format=torch.channels_last)
        dx = torch.empty(N, C, H, W, dtype=ctx.dtype, device=dy.device, memory_format=torch.channels_last)
        K.maxpool3s2_bwd(dy, idx, dx, N, H, W, C)
        return dx


def maxpool_covered(x: torch.Tensor, pool: torch.nn.Module) -> bool:
    """``pool`` is ``MaxPool2d(3, 2, 1)`` (dilation 1, floor mode, no indices) and ``x`` a channels-last bf16 / fp32 CUDA
    activation with C % 8 == 0 (``IIT_FUSED_POOL=0`` disables)."""
    if not (isinstance(pool, torch.nn.MaxPool2d) and enabled() and os.environ.get("IIT_FUSED_POOL", "1") != "0"):
        return False
    k, st, pd, dl = pool.kernel_size, pool.stride, pool.padding, pool.dilation
    if not all(v in (n, (n, n)) for v, n in ((k, 3), (st, 2), (pd, 1), (dl, 1))):
        return False
    if pool.ceil_mode or pool.return_indices:
        return False
    return (x.is_cuda and x.dtype in (BF16, F32) and x.dim() == 4 and x.shape[1] % 8 == 0
            and x.is_contiguous(memory_format=torch.channels_last))
