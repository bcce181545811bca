"""Fused interchange splice / gradient mask / activation scale over a ``TorchIndex`` patch spec (``csrc/splice.hip``).

Replaces the reference's per-site hook ``out = act.clone(); out[idx] = src[idx]``
(``/root/reference/iit/model_pairs/base_model_pair.py:151-163``) and StopGrad's ``act / scale`` forward hook and
``grad[idx] = 0`` backward hook (``/root/reference/iit/model_pairs/stop_grad_pair.py:37-75``) for any index that
:meth:`iit_amd.core.index.TorchIndex.to_ranges` can express (per-dimension ranges; batch / position / head /
feature / channel / spatial selections): one kernel launch per site and direction, no index tensors, no clone,
nothing host-synchronising, so the site stays inside a captured HIP graph.  The backward of a splice zeroes the
spliced elements' gradient (the source is a detached constant), exactly the gradient of the reference's clone +
index_put.  Indices the range table cannot express (paired list atoms, stepped slices) keep the generic
clone / index_put path.
"""
from __future__ import annotations

from typing import Optional, Sequence, Tuple

import numpy as np
import torch
from torch.autograd import Function

from . import hip_kernels as K

_SPEC_DTYPE = np.dtype([("shape", np.int32, 4), ("nr", np.int32, 4), ("lo", np.int32, (4, 8)), ("hi", np.int32, (4, 8)),
                        ("sstride", np.int64, 4)])
MODE_SPLICE, MODE_ZERO, MODE_DIVIDE = 0, 1, 2


def _collapse(shape: Sequence[int], ranges, strides: Sequence[int]):
    """Merge neighbouring whole dimensions until at most 4 remain (the kernel's rank) and pad to 4 with leading
    size-1 dimensions; ``strides`` (the source's, 0 = broadcast) follow along.  None when impossible."""
    dims = [(int(n), r, int(st)) for n, r, st in zip(shape, ranges, strides)]
    whole = lambda n, r: r == [(0, n)]  # noqa: E731
    i = len(dims) - 2
    while len(dims) > 4 and i >= 0:
        (n0, r0, s0), (n1, r1, s1) = dims[i], dims[i + 1]
        if whole(n0, r0) and whole(n1, r1) and s0 == s1 * n1:
            dims[i:i + 2] = [(n0 * n1, [(0, n0 * n1)], s1)]
        i -= 1
    if len(dims) > 4:
        return None
    while len(dims) < 4:
        dims.insert(0, (1, [(0, 1)], 0))
    return dims


class PatchSpec:
    """Host-packed range table of one (index, hook shape, source strides); cached on the TorchIndex."""

    __slots__ = ("buf", "dims")

    def __init__(self, dims):
        rec = np.zeros(1, dtype=_SPEC_DTYPE)
        for d, (n, runs, st) in enumerate(dims):
            rec["shape"][0, d] = n
            rec["nr"][0, d] = len(runs)
            for r, (lo, hi) in enumerate(runs):
                rec["lo"][0, d, r] = lo
                rec["hi"][0, d, r] = hi
            rec["sstride"][0, d] = st
        self.buf = rec.view(np.uint8).copy()
        self.dims = dims

    @property
    def ptr(self) -> int:
        return self.buf.ctypes.data


def patch_spec(index, shape: Tuple[int, ...], src: Optional[torch.Tensor] = None,
               perm: Optional[Tuple[int, ...]] = None) -> Optional[PatchSpec]:
    """The range table of ``index`` on a hook of ``shape`` (with ``src``'s strides, broadcast allowed), or None.
    ``perm``: the table for the activation's memory order instead (e.g. (0, 2, 3, 1) for a channels-last NCHW
    tensor, whose flat elements run N, H, W, C) -- dimensions, ranges and source strides permuted alike."""
    ranges = index.to_ranges(tuple(shape))
    if ranges is None:
        return None
    strides = [0] * len(shape)
    if src is not None:
        if src.dim() > len(shape) or any(sn not in (1, n) for sn, n in zip(src.shape[::-1], tuple(shape)[::-1])):
            return None
        strides = list(src.expand(tuple(shape)).stride())  # broadcast dimensions get stride 0
    if perm is not None:
        shape, ranges, strides = ([x[i] for i in perm] for x in (list(shape), list(ranges), strides))
    dims = _collapse(shape, ranges, strides)
    if dims is None:
        return None
    key = (tuple(shape), tuple(strides), perm)
    cache = getattr(index, "_iit_specs", None)
    if cache is None:
        cache = {}
        index._iit_specs = cache
    spec = cache.get(key)
    if spec is None:
        spec = cache[key] = PatchSpec(dims)
    return spec


def fused_ok(t: torch.Tensor) -> bool:
    return t.is_cuda and t.dtype in (torch.bfloat16, torch.float32) and K.available()


def _launch(act, src, out, spec: PatchSpec, mode: int, scale: float = 1.0):
    K.splice(act, src, out, act.numel(), spec.ptr, act.dtype == torch.float32, mode, scale)


_CL = (0, 2, 3, 1)  # the memory order of a channels-last NCHW tensor


def _channels_last(t: torch.Tensor) -> bool:
    return t.dim() == 4 and not t.is_contiguous() and t.is_contiguous(memory_format=torch.channels_last)


class SpliceFn(Function):
    """``out = act`` with ``out[index] = src[index]``; gradient: ``g`` with the spliced elements zeroed.  A
    channels-last ``act`` keeps its layout (the range table then runs in memory order, ``spec_cl``)."""

    @staticmethod
    def forward(ctx, act, src, spec, spec_cl=None):
        if spec_cl is not None and _channels_last(act):
            out = torch.empty_like(act, memory_format=torch.channels_last)
            _launch(act.permute(_CL), src, out.permute(_CL), spec_cl, MODE_SPLICE)
            ctx.spec = spec_cl
            ctx.cl = True
            return out
        act_c = act.contiguous()
        out = torch.empty_like(act_c)
        _launch(act_c, src, out, spec, MODE_SPLICE)
        ctx.spec = spec
        ctx.cl = False
        return out

    @staticmethod
    def backward(ctx, g):
        if g is None:
            return None, None, None, None
        if ctx.cl:
            g = g.contiguous(memory_format=torch.channels_last)
            out = torch.empty_like(g, memory_format=torch.channels_last)
            _launch(g.permute(_CL), None, out.permute(_CL), ctx.spec, MODE_ZERO)
            return out, None, None, None
        g = g.contiguous()
        out = torch.empty_like(g)
        _launch(g, None, out, ctx.spec, MODE_ZERO)
        return out, None, None, None


class GradMaskFn(Function):
    """Identity forward; backward zeroes the gradient at ``index`` (StopGrad's non-circuit zero-grad hook)."""

    @staticmethod
    def forward(ctx, x, spec):
        ctx.spec = spec
        return x.view_as(x)

    @staticmethod
    def backward(ctx, g):
        if g is None:
            return None, None
        g = g.contiguous()
        out = torch.empty_like(g)
        _launch(g, None, out, ctx.spec, MODE_ZERO)
        return out, None


class ScaleFn(Function):
    """``out = act`` with ``out[index] /= s``; gradient divided the same way (StopGrad's ``act / scale``)."""

    @staticmethod
    def forward(ctx, act, spec, s):
        act_c = act.contiguous()
        out = torch.empty_like(act_c)
        _launch(act_c, None, out, spec, MODE_DIVIDE, s)
        ctx.spec, ctx.s = spec, s
        return out

    @staticmethod
    def backward(ctx, g):
        if g is None:
            return None, None, None
        g = g.contiguous()
        out = torch.empty_like(g)
        _launch(g, None, out, ctx.spec, MODE_DIVIDE, ctx.s)
        return out, None, None


def splice(act: torch.Tensor, index, src: torch.Tensor) -> Optional[torch.Tensor]:
    """Fused ``act.clone(); out[index] = src[index]`` (None when the fused kernel does not cover the case)."""
    if not fused_ok(act):
        return None
    if src.dtype != act.dtype or src.device != act.device:
        src = src.to(device=act.device, dtype=act.dtype)
    spec = patch_spec(index, tuple(act.shape), src)
    if spec is None:
        return None
    spec_cl = patch_spec(index, tuple(act.shape), src, perm=_CL) if _channels_last(act) else None
    return SpliceFn.apply(act, src, spec, spec_cl)


def grad_mask(x: torch.Tensor, indices) -> Optional[torch.Tensor]:
    """``x`` whose gradient is zeroed at every index of ``indices`` (None when not covered)."""
    if not fused_ok(x):
        return None
    specs = [patch_spec(ix, tuple(x.shape)) for ix in indices]
    if any(s is None for s in specs):
        return None
    for s in specs:
        x = GradMaskFn.apply(x, s)
    return x


def divide(x: torch.Tensor, index, s: float) -> Optional[torch.Tensor]:
    """``x`` with ``x[index] / s`` (gradient likewise); None when not covered."""
    if not fused_ok(x):
        return None
    spec = patch_spec(index, tuple(x.shape))
    if spec is None:
        return None
    return ScaleFn.apply(x, spec, float(s))
