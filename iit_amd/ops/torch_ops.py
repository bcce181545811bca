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


class TorchOps:
    name = "torch"
    fused = False

    def __init__(self, dtype: torch.dtype = torch.float32):
        self.dtype = dtype

    # -- helpers --------------------------------------------------------------
    def w(self, p: torch.Tensor) -> torch.Tensor:
        return p if p.dtype == self.dtype else p.to(self.dtype)

    # -- ops ------------------------------------------------------------------
    def embed(self, tokens, W_E):
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
        pre = x @ self.w(W_in) + self.w(b_in)
        if hook_pre is not None:
            pre = hook_pre(pre)
        return pre, act_fn(act)(pre)

    def mlp_gated_in(self, x, W_gate, W_in, b_in, act: str, hook_pre=None, hook_pre_linear=None):
        """TL ``GatedMLP``: ``pre = x W_gate`` (hook_pre), ``pre_linear = x W_in + b_in``, ``post = act(pre) * pre_linear``."""
        pre = x @ self.w(W_gate)
        if hook_pre is not None:
            pre = hook_pre(pre)
        pre_linear = x @ self.w(W_in) + self.w(b_in)
        if hook_pre_linear is not None:
            pre_linear = hook_pre_linear(pre_linear)
        return pre, act_fn(act)(pre) * pre_linear

    def mlp_out(self, post, W_out, b_out):
        return post @ self.w(W_out) + self.w(b_out)

    def unembed(self, x, W_U, b_U):
        return x @ self.w(W_U) + self.w(b_U)

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
