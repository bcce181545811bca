"""Paired source + base forwards on the torch op backend: the Llama family (RMSNorm, rotary, grouped-query flash
attention, SwiGLU) at bf16 on the GPU (VERDICT r5 missing #1 / next #4).

The reference runs an interchange intervention as two forwards -- the source run under ``no_grad``, then the base
run with the cached source activations spliced in (``/root/reference/iit/model_pairs/base_model_pair.py:75-105``).
``HookedTransformer.run_paired`` folds them into ONE forward of 2B rows up to the deepest splice site; the fused HIP
backend (GPT-2 family) does so with the ``*PairFn`` ops of :mod:`iit_amd.ops.hip_ops`.  The ops here are the same
pattern for the torch backend's Functions: each computes over the full rows with one launch (one GEMM of 2T rows,
one RMSNorm / rotary / SwiGLU / flash-attention pass over 2B sequences), returns the BASE rows as its autograd
output, appends the full result to ``box`` for the source side, and saves only base-row slices for its backward --
which is the unpaired op's backward, unchanged.  So the source rows cost no backward work and produce no gradient,
exactly as the reference's ``no_grad`` source run.
"""
from __future__ import annotations

from typing import Optional

import torch

from . import hip_kernels as K
from .hip_ops import (BF16, F32, FlashFn, Paired, PairSpliceFn, RMSNormFn, RotaryFn, SwiGLUFn, _c16, _flash_view,
                      _one, pair_specs)
from .torch_ops import _MirrorEmbed, _MirrorLinear, _MirrorMat, _SplitQKV, _arena_mirror, _bound_to_arena, _mm_bias


def _rows(t: torch.Tensor, B: int, B2: int) -> int:
    """Flattened row count of the first ``B`` of ``B2`` leading entries of ``t``."""
    return t.numel() // t.shape[-1] * B // B2


class EmbedPairFn(_MirrorEmbed):
    """``W_E[tokens]`` of both token sets from the bf16 mirror; backward = the base rows' index-add."""

    @staticmethod
    def forward(ctx, tokens, W_E, _flat, tokens_full, box):
        out = _flat.shadow_view(W_E)[tokens_full]
        ctx.save_for_backward(tokens)
        ctx.p, ctx.flat = W_E, _flat
        box.append(out)
        return out[:tokens.shape[0]]

    @staticmethod
    def backward(ctx, g):
        return _MirrorEmbed.backward(ctx, g) + (None, None)


class RMSNormPairFn(RMSNormFn):
    @staticmethod
    def forward(ctx, x, w, eps, x_full, box):
        ctx.set_materialize_grads(False)
        d = x_full.shape[-1]
        x2 = _c16(x_full.reshape(-1, d))
        T2 = x2.shape[0]
        T = _rows(x_full, x.shape[0], x_full.shape[0])
        y = torch.empty(T2, d, dtype=BF16, device=x.device)
        rstd = torch.empty(T2, dtype=F32, device=x.device)
        K.rms_fwd(x2, None if w is None else w.detach(), y, rstd, T2, d, eps)
        ctx.save_for_backward(x2[:T], rstd[:T])
        ctx.w = w
        ctx.shape = x.shape
        yf = y.view(*x_full.shape[:-1], d)
        box.append(yf)
        return yf[:x.shape[0]]

    @staticmethod
    def backward(ctx, dy):
        return RMSNormFn.backward(ctx, dy) + (None, None)


class MirrorMatPairFn(_MirrorMat):
    """:class:`_MirrorMat` (packed QKV / ``W_O``) over both row sets: one GEMM of 2T rows."""

    @staticmethod
    def forward(ctx, x, wm, bm, gw, gb, wparams, bparams, x_full, *rest):
        leaves, box = rest[:-1], rest[-1]  # (``_one`` appends the box last)
        lead = x.shape[:-1]
        x2f = x_full.reshape(-1, x_full.shape[-1])
        T = _rows(x_full, x.shape[0], x_full.shape[0])
        yf = _mm_bias(x2f, wm, bm)
        ctx.save_for_backward(x2f[:T])
        ctx.wm, ctx.gw, ctx.gb, ctx.lead, ctx.n_leaves = wm, gw, gb, lead, len(leaves)
        ctx.wparams, ctx.bparams = wparams, bparams
        yf = yf.view(*x_full.shape[:-1], yf.shape[-1])
        box.append(yf)
        return yf[:x.shape[0]]

    @staticmethod
    def backward(ctx, gy):
        r = _MirrorMat.backward(ctx, gy)
        return r[:7] + (None,) + r[7:] + (None,)


class MirrorLinearPairFn(_MirrorLinear):
    @staticmethod
    def forward(ctx, x, W, b, _flat, x_full, box):
        Wm = _flat.shadow_view(W)
        lead = x.shape[:-1]
        x2f = x_full.reshape(-1, x_full.shape[-1])
        T = _rows(x_full, x.shape[0], x_full.shape[0])
        yf = _mm_bias(x2f, Wm, _flat.shadow_view(b) if b is not None else None)
        ctx.save_for_backward(x2f[:T])
        ctx.W, ctx.b, ctx.flat, ctx.lead = W, b, _flat, lead
        yf = yf.view(*x_full.shape[:-1], yf.shape[-1])
        box.append(yf)
        return yf[:x.shape[0]]

    @staticmethod
    def backward(ctx, gy):
        return _MirrorLinear.backward(ctx, gy) + (None, None)


class RotaryPairFn(RotaryFn):
    @staticmethod
    def forward(ctx, x, cos, sin, rd, offset, adjacent, x_full, box):
        out = torch.empty(x_full.shape, dtype=BF16, device=x.device)
        K.rotary(x_full, out, cos, sin, rd, offset, adjacent, False)
        ctx.cfg = (cos, sin, rd, offset, adjacent)
        box.append(out)
        return out[:x.shape[0]]

    @staticmethod
    def backward(ctx, g):
        return RotaryFn.backward(ctx, g) + (None, None)


class FlashPairFn(FlashFn):
    """Flash attention over 2B sequences (one launch); the backward runs on the base sequences only."""

    @staticmethod
    def forward(ctx, q, k, v, causal, scale, q_full, k_full, v_full, box):
        ctx.set_materialize_grads(False)
        B2, S, Hq, dh = q_full.shape
        B = q.shape[0]
        z = torch.empty(B2, S, Hq, dh, dtype=BF16, device=q.device)
        lse = torch.empty(B2, Hq, S, dtype=F32, device=q.device)
        K.flash_fwd(q_full, k_full, v_full, z, lse, None, 0, scale, causal)
        ctx.save_for_backward(q_full[:B], k_full[:B], v_full[:B], z[:B], lse[:B])
        ctx.cfg = (0, causal, scale)
        ctx.spec = None
        ctx.keep = None
        box.append(z)
        return z[:B]

    @staticmethod
    def backward(ctx, dz):
        return FlashFn.backward(ctx, dz)[:5] + (None,) * 4


class SwiGLUPairFn(SwiGLUFn):
    @staticmethod
    def forward(ctx, gate, up, gate_full, up_full, box):
        gf, uf = _c16(gate_full.to(BF16)), _c16(up_full.to(BF16))
        post = torch.empty_like(gf)
        K.swiglu_fwd(gf, uf, post)
        B = gate.shape[0]
        ctx.save_for_backward(gf[:B], uf[:B])
        box.append(post)
        return post[:B]

    @staticmethod
    def backward(ctx, dpost):
        return SwiGLUFn.backward(ctx, dpost) + (None, None, None)


class PairAddFn(torch.autograd.Function):
    """``a + b`` of both row sets in one pass (the residual stream's skip connection)."""

    @staticmethod
    def forward(ctx, a, b, a_full, b_full, box):
        out = a_full + b_full
        ctx.dt = (a.dtype, b.dtype)
        box.append(out)
        return out[:a.shape[0]]

    @staticmethod
    def backward(ctx, g):
        if g is None:
            return None, None, None, None, None
        return g.to(ctx.dt[0]), g.to(ctx.dt[1]), None, None, None


# ---------------------------------------------------------------------------------------------------- paired ops
def pair_embed(tokens, src_tokens, W_E) -> Optional[Paired]:
    m = _arena_mirror(W_E)
    if m is None:
        return None
    full = torch.cat([tokens, src_tokens])
    out, f = _one(EmbedPairFn, tokens, W_E, m[0], full)
    return Paired(out, f)


def pair_rms(p: Paired, w, eps) -> Paired:
    out, f = _one(RMSNormPairFn, p.base, w, eps, p.full)
    return Paired(out, f)


def pair_qkv(x: Paired, W_Q, W_K, W_V, b_Q, b_K, b_V):
    """(q, k, v) Paired heads of the packed arena projection, or None when the arena layout does not apply."""
    m = _arena_mirror(W_Q)
    if m is None or W_Q.dim() != 3:
        return None
    flat = m[0]
    H, d, dh = W_Q.shape
    Hkv = W_K.shape[0]
    N = (H + 2 * Hkv) * dh
    ws = (W_Q, W_K, W_V)
    if any(w.stride() != (dh, N, 1) or not flat.owns(w) or not w.requires_grad for w in ws):
        return None
    off = flat.offset_of(W_Q)
    if flat.offset_of(W_K) != off + H * dh or flat.offset_of(W_V) != off + (H + Hkv) * dh:
        return None
    bs = (b_Q, b_K, b_V)
    boff = flat.offset_of(b_Q) if flat.owns(b_Q) else -1
    packed_b = boff >= 0 and all(b.requires_grad and flat.owns(b) and b.is_contiguous() for b in bs) and \
        flat.offset_of(b_K) == boff + H * dh and flat.offset_of(b_V) == boff + (H + Hkv) * dh
    if not packed_b and any(b is not None and b.requires_grad for b in bs):
        return None
    if not all(_bound_to_arena(flat, p) for p in ws + (bs if packed_b else ())):
        return None
    sh = flat.shadow
    wm = sh.as_strided((d, N), (N, 1), off)
    bm = sh.as_strided((N,), (1,), boff) if packed_b else None
    gw = flat.grad.as_strided((d, N), (N, 1), off)
    gb = flat.grad.as_strided((N,), (1,), boff) if packed_b else None
    bp = bs if packed_b else ()
    y, yf = _one(MirrorMatPairFn, x.base, wm, bm, gw, gb, ws, bp, x.full, *(ws + bp))
    q, k, v = _SplitQKV.apply(y, H, Hkv, dh)
    lead = yf.shape[:-1]
    qf = yf[..., :H * dh].view(*lead, H, dh)
    kf = yf[..., H * dh:(H + Hkv) * dh].view(*lead, Hkv, dh)
    vf = yf[..., (H + Hkv) * dh:].view(*lead, Hkv, dh)
    return Paired(q, qf), Paired(k, kf), Paired(v, vf)


def pair_rotary(p: Paired, cos, sin, rd: int, adjacent: bool) -> Paired:
    x = p.base.to(BF16)
    xf = p.full.to(BF16)
    if xf.stride(-1) != 1:
        xf = xf.contiguous()
    out, f = _one(RotaryPairFn, x, cos, sin, rd, 0, adjacent, xf)
    return Paired(out, f)


def pair_flash(q: Paired, k: Paired, v: Paired, causal: bool, attn_scale: float) -> Paired:
    qf, kf, vf = _flash_view(q.full), _flash_view(k.full), _flash_view(v.full)
    out, f = _one(FlashPairFn, q.base, k.base, v.base, causal, 1.0 / attn_scale, qf, kf, vf)
    return Paired(out, f)


def pair_o_proj(z: Paired, W_O, b_O) -> Optional[Paired]:
    m = _arena_mirror(W_O)
    mb = _arena_mirror(b_O) if (b_O is not None and b_O.is_contiguous()) else None
    if m is None or (b_O is not None and mb is None) or not W_O.is_contiguous():
        return None
    flat = m[0]
    if not (_bound_to_arena(flat, W_O) and (b_O is None or _bound_to_arena(flat, b_O))):
        return None
    H, dh, d = W_O.shape
    wm = m[1].view(H * dh, d)
    bp = () if b_O is None else (b_O,)
    gw = flat.grad.as_strided((H * dh, d), (d, 1), flat.offset_of(W_O))
    gb = None if b_O is None else flat.grad.as_strided((d,), (1,), flat.offset_of(b_O))
    zb = z.base.to(BF16).reshape(*z.base.shape[:-2], H * dh)
    zf = z.full.to(BF16).reshape(*z.full.shape[:-2], H * dh)
    out, f = _one(MirrorMatPairFn, zb, wm, None if mb is None else mb[1], gw, gb, (W_O,), bp, zf, W_O, *bp)
    return Paired(out, f)


def pair_linear(x: Paired, W, b=None) -> Optional[Paired]:
    m = _arena_mirror(W)
    if m is None or W.dim() != 2 or not W.is_contiguous() or (b is not None and (_arena_mirror(b) is None
                                                                                 or not b.is_contiguous())):
        return None
    out, f = _one(MirrorLinearPairFn, x.base.to(BF16), W, b, m[0], x.full.to(BF16))
    return Paired(out, f)


def pair_swiglu(gate: Paired, up: Paired) -> Paired:
    out, f = _one(SwiGLUPairFn, gate.base, up.base, gate.full, up.full)
    return Paired(out, f)


def pair_add(a: Paired, b: Paired) -> Paired:
    out, f = _one(PairAddFn, a.base, b.base, a.full, b.full)
    return Paired(out, f)


def pair_splice(p: Paired, index) -> Optional[Paired]:
    """Base rows take the source rows' values at ``index`` (one patch-spec launch over both row sets)."""
    full = p.full if p.full.is_contiguous() else p.full.contiguous()
    specs = pair_specs(index, tuple(p.base.shape))
    if specs is None:
        return None
    out, f = _one(PairSpliceFn, p.base, full, specs[0], specs[1])
    return Paired(out, f)
