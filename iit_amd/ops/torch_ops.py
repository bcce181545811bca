"""Reference-semantics ("oracle") implementations of the transformer block ops.

Pure PyTorch, any device, autograd-native.  This is the correctness reference the
HIP kernels are tested against and the CPU execution path.
It follows TransformerLens math exactly (einsum layouts of SURVEY.md §2.6,
``gelu_new``, LNPre, causal mask with -inf).
"""
from __future__ import annotations

import math
from typing import Optional, Sequence, Tuple

import torch
import torch.nn.functional as F


def gelu_new(x: torch.Tensor) -> torch.Tensor:
    return 0.5 * x * (1.0 + torch.tanh(math.sqrt(2.0 / math.pi) * (x + 0.044715 * torch.pow(x, 3.0))))


def act_fn(name: str):
    if name == "gelu_new" or name == "gelu_fast" or name == "gelu_pytorch_tanh":
        return gelu_new
    if name == "gelu":
        return F.gelu
    if name == "relu":
        return F.relu
    if name == "silu":
        return F.silu
    if name == "solu_ln":
        raise NotImplementedError("solu_ln is not supported")
    raise ValueError(f"unknown act_fn {name}")


def _arena_mirror(p: torch.Tensor):
    """(flat arena, bf16 mirror view of ``p``) when ``p`` lives in a :class:`~iit_amd.engine.flat.FlatParams` on
    a GPU and the mirror holds its current value (else None).  The fused Adam writes the mirror in its update
    pass, so a bf16 model reads its weights without a per-forward cast."""
    flat = getattr(p, "_iit_flat", None)
    if flat is None or not p.is_cuda or not p.requires_grad or not flat.owns(p):
        return None
    module = flat.module
    if flat.shadow is None or flat.mirror_version != getattr(module, "_iit_weights_version", 0):
        if torch.cuda.is_current_stream_capturing():
            return None
        flat.ensure_shadow()
        flat.refresh_shadow()
    return flat, flat.shadow_view(p)


def _accumulate(p: torch.Tensor, g: torch.Tensor) -> None:
    """fp32 grad slot += bf16 gradient in one mixed-precision pass; report it to the DP reducer."""
    from ..engine import grad_hooks
    slot = p.grad
    if slot is None:
        slot = p.grad = torch.zeros_like(p)
    slot.add_(g)
    grad_hooks.notify(p)


class _MirrorWeight(torch.autograd.Function):
    """bf16 compute copy of an arena weight: forward returns the mirror view (no cast kernel); backward adds the
    bf16 gradient straight into the fp32 grad slot (no cast-to-fp32 pass, no AccumulateGrad)."""

    @staticmethod
    def forward(ctx, p, _flat):
        ctx.p = p
        return _flat.shadow_view(p)

    @staticmethod
    def backward(ctx, g):
        _accumulate(ctx.p, g)
        return None, None


class _MirrorEmbed(torch.autograd.Function):
    """``W_E[tokens]`` from the bf16 mirror; backward index-adds the rows into the fp32 grad slot (no dense
    ``[V, d]`` gradient is ever materialised -- 128k x 4096 for Llama-3)."""

    @staticmethod
    def forward(ctx, tokens, W_E, _flat):
        ctx.save_for_backward(tokens)
        ctx.p = W_E
        return _flat.shadow_view(W_E)[tokens]

    @staticmethod
    def backward(ctx, g):
        (tokens,) = ctx.saved_tensors
        from ..engine import grad_hooks
        W_E = ctx.p
        slot = W_E.grad
        if slot is None:
            slot = W_E.grad = torch.zeros_like(W_E)
        slot.index_add_(0, tokens.reshape(-1), g.reshape(-1, g.shape[-1]).to(slot.dtype))
        grad_hooks.notify(W_E)
        return None, None, None


class _MirrorLinear(torch.autograd.Function):
    """``x @ W (+ b)`` for an arena weight ``W [K, N]``: both GEMMs read the bf16 mirror, and the weight
    gradient is one fp32-output GEMM accumulating straight into the arena's grad slot (``addmm`` with
    beta = 1) -- no bf16 ``dW`` tensor, no cast, no separate accumulate pass over the matrix."""

    @staticmethod
    def forward(ctx, x, W, b, _flat):
        Wm = _flat.shadow_view(W)
        lead = x.shape[:-1]
        x2 = x.reshape(-1, x.shape[-1])
        y = x2 @ Wm
        if b is not None:
            y = y + _flat.shadow_view(b)
        ctx.save_for_backward(x2)
        ctx.W, ctx.b, ctx.flat, ctx.lead = W, b, _flat, lead
        return y.view(*lead, y.shape[-1])

    @staticmethod
    def backward(ctx, gy):
        from ..engine import grad_hooks
        from .gemm_dispatch import _addmm_f32
        (x2,) = ctx.saved_tensors
        W, b, flat = ctx.W, ctx.b, ctx.flat
        g2 = gy.reshape(-1, gy.shape[-1]).to(x2.dtype)
        dx = None
        if ctx.needs_input_grad[0]:
            dx = (g2 @ flat.shadow_view(W).t()).view(*ctx.lead, W.shape[0])
        if W.requires_grad:
            slot = W.grad
            if slot is None:
                slot = W.grad = torch.zeros_like(W)
            _addmm_f32(slot, slot, x2.t(), g2)
            grad_hooks.notify(W)
        if b is not None and b.requires_grad:
            _accumulate(b, g2.float().sum(0))
        return dx, None, None, None


class TorchOps:
    name = "torch"
    fused = False

    def __init__(self, dtype: torch.dtype = torch.float32):
        self.dtype = dtype

    # -- helpers --------------------------------------------------------------
    def w(self, p: torch.Tensor) -> torch.Tensor:
        if p.dtype == self.dtype:
            return p
        if self.dtype == torch.bfloat16 and torch.is_grad_enabled():
            m = _arena_mirror(p)
            if m is not None:
                return _MirrorWeight.apply(p, m[0])
        elif self.dtype == torch.bfloat16:
            m = _arena_mirror(p)
            if m is not None:
                return m[1]
        return p.to(self.dtype)

    def lin(self, x, W, b=None):
        """``x @ W (+ b)``; arena weights on a GPU in bf16 take :class:`_MirrorLinear`."""
        if (self.dtype == torch.bfloat16 and W.dim() == 2 and W.dtype != self.dtype and x.is_cuda
                and torch.is_grad_enabled() and W.is_contiguous()):
            m = _arena_mirror(W)
            if m is not None and (b is None or (_arena_mirror(b) is not None and b.is_contiguous())):
                return _MirrorLinear.apply(x.to(self.dtype), W, b, m[0])
        y = x @ self.w(W)
        return y if b is None else y + self.w(b)

    # -- ops ------------------------------------------------------------------
    def embed(self, tokens, W_E):
        if self.dtype == torch.bfloat16 and W_E.dtype != self.dtype:
            m = _arena_mirror(W_E)
            if m is not None:
                if torch.is_grad_enabled():
                    return _MirrorEmbed.apply(tokens, W_E, m[0])
                return m[1][tokens]
        return self.w(W_E)[tokens]

    def pos_embed(self, batch: int, seq: int, W_pos, offset: int = 0):
        return self.w(W_pos)[offset:offset + seq].unsqueeze(0).expand(batch, seq, W_pos.shape[-1])

    def layer_norm(self, x, w: Optional[torch.Tensor], b: Optional[torch.Tensor], eps: float,
                   hook_scale=None, hook_normalized=None):
        x = x.to(self.dtype)
        x = x - x.mean(-1, keepdim=True)
        scale = (x.pow(2).mean(-1, keepdim=True) + eps).sqrt()
        if hook_scale is not None:
            scale = hook_scale(scale)
        y = x / scale
        if w is not None:
            y = y * self.w(w) + self.w(b)
        if hook_normalized is not None:
            y = hook_normalized(y)
        return y

    def rms_norm(self, x, w: Optional[torch.Tensor], eps: float, hook_scale=None, hook_normalized=None):
        """TL ``RMSNorm`` / ``RMSNormPre``: ``x / sqrt(mean(x^2) + eps) (* w)``."""
        x = x.to(self.dtype)
        scale = (x.pow(2).mean(-1, keepdim=True) + eps).sqrt()
        if hook_scale is not None:
            scale = hook_scale(scale)
        y = x / scale
        if w is not None:
            y = y * self.w(w)
        if hook_normalized is not None:
            y = hook_normalized(y)
        return y

    def rotary(self, x, cos, sin, rotary_dim: int, adjacent_pairs: bool = False, offset: int = 0):
        """Rotary position embedding of ``x [B, S, H, dh]`` on its first ``rotary_dim`` features
        (TL ``apply_rotary``; GPT-NeoX half-split pairs, or adjacent (even, odd) pairs)."""
        S = x.shape[1]
        c = cos[offset:offset + S].to(x.dtype)[None, :, None, :]
        s = sin[offset:offset + S].to(x.dtype)[None, :, None, :]
        xr, xp = x[..., :rotary_dim], x[..., rotary_dim:]
        if adjacent_pairs:
            x1, x2 = xr[..., 0::2], xr[..., 1::2]
            flipped = torch.stack([-x2, x1], dim=-1).flatten(-2)
        else:
            half = rotary_dim // 2
            flipped = torch.cat([-xr[..., half:], xr[..., :half]], dim=-1)
        out = xr * c + flipped * s
        return torch.cat([out, xp], dim=-1) if xp.shape[-1] else out

    def qkv(self, x, W_Q, W_K, W_V, b_Q, b_K, b_V):
        q = torch.einsum("bsd,hde->bshe", x, self.w(W_Q)) + self.w(b_Q)
        k = torch.einsum("bsd,hde->bshe", x, self.w(W_K)) + self.w(b_K)
        v = torch.einsum("bsd,hde->bshe", x, self.w(W_V)) + self.w(b_V)
        return q, k, v

    def attention(self, q, k, v, causal: bool, attn_scale: float, hook_scores=None, hook_pattern=None,
                  ignore: float = float("-inf")):
        scores = torch.einsum("bqhe,bkhe->bhqk", q, k) / attn_scale
        if causal:
            S = q.shape[1]
            mask = torch.ones(S, S, dtype=torch.bool, device=q.device).tril()
            scores = torch.where(mask, scores, torch.tensor(ignore, dtype=scores.dtype, device=scores.device))
        if hook_scores is not None:
            scores = hook_scores(scores)
        pattern = F.softmax(scores, dim=-1)
        pattern = torch.where(torch.isnan(pattern), torch.zeros_like(pattern), pattern)
        if hook_pattern is not None:
            pattern = hook_pattern(pattern)
        z = torch.einsum("bkhe,bhqk->bqhe", v, pattern)
        return z

    def o_proj(self, z, W_O, b_O):
        return torch.einsum("bshe,hed->bsd", z, self.w(W_O)) + self.w(b_O)

    def o_result(self, z, W_O):
        return torch.einsum("bshe,hed->bshd", z, self.w(W_O))

    def mlp_in(self, x, W_in, b_in, act: str, hook_pre=None):
        pre = self.lin(x, W_in, b_in)
        if hook_pre is not None:
            pre = hook_pre(pre)
        return pre, act_fn(act)(pre)

    def mlp_gated_in(self, x, W_gate, W_in, b_in, act: str, hook_pre=None, hook_pre_linear=None):
        """TL ``GatedMLP``: ``pre = x W_gate`` (hook_pre), ``pre_linear = x W_in + b_in``, ``post = act(pre) * pre_linear``."""
        pre = self.lin(x, W_gate)
        if hook_pre is not None:
            pre = hook_pre(pre)
        pre_linear = self.lin(x, W_in, b_in)
        if hook_pre_linear is not None:
            pre_linear = hook_pre_linear(pre_linear)
        return pre, act_fn(act)(pre) * pre_linear

    def mlp_out(self, post, W_out, b_out):
        return self.lin(post, W_out, b_out)

    def unembed(self, x, W_U, b_U):
        return self.lin(x, W_U, b_U)

    def unembed_argmax(self, x, W_U, b_U, chunk: int = 16384):
        """``argmax(x @ W_U + b_U, -1)`` with first-index tie-break, vocab-chunked (bounded memory)."""
        W, b = self.w(W_U), self.w(b_U)
        best_val = None
        best_idx = None
        for s in range(0, W.shape[1], chunk):
            logits = x @ W[:, s:s + chunk] + b[s:s + chunk]
            v, i = logits.max(dim=-1)
            i = i + s
            if best_val is None:
                best_val, best_idx = v, i
            else:
                upd = v > best_val
                best_val = torch.where(upd, v, best_val)
                best_idx = torch.where(upd, i, best_idx)
        return best_idx

    def residual(self, a, b):
        return a + b
