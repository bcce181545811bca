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
        flat = getattr(p, "_iit_flat", None)
        slot = flat.bind_zero(p) if flat is not None and flat.owns(p) else torch.zeros_like(p)
        p.grad = slot
    if (g.dtype == torch.bfloat16 and slot.dtype == torch.float32 and slot.is_cuda and g.is_cuda
            and slot.shape == g.shape and slot.stride() == g.stride()
            and (slot.is_contiguous() or (slot.dim() == 4 and slot.is_contiguous(memory_format=torch.channels_last)))):
        # same memory order (e.g. a channels-last conv weight and its gradient): one HIP pass over the dense span,
        # fp32 += bf16 (the same math as cast + add, one launch instead of two)
        from . import hip_kernels as K
        if K.available():
            n = slot.numel()
            K.add_bf16(slot, n, slot, n, g, n, None, 1, n)
            grad_hooks.notify(p)
            return
    if g.dtype != slot.dtype and g.numel() <= (1 << 20):
        # small vectors (norm weights): cast + same-dtype add is two ~3 us launches; ROCm's mixed-dtype
        # add kernel takes ~50 us on a 4096-vector
        g = g.to(slot.dtype)
    slot.add_(g)
    grad_hooks.notify(p)


def _mm_bias(x2: torch.Tensor, wm: torch.Tensor, bm: Optional[torch.Tensor]) -> torch.Tensor:
    """``x2 @ wm (+ bm)`` as ONE library GEMM with the bias in its epilogue (``addmm`` with a 1-D bias) -- a separate
    broadcast add is a non-vectorised elementwise pass over the [T, N] output (~48 us per Llama-3-8B projection at
    S = 512, 5 per block and phase: 23 ms/step, profiles/llama3_8b_s512_step_breakdown_r4.txt)."""
    if bm is None:
        return x2 @ wm
    if bm.dim() == 1 and bm.dtype == wm.dtype and x2.dim() == 2:
        return torch.addmm(bm, x2, wm)
    return x2 @ wm + bm


def _bias_grad_accumulate(slot: torch.Tensor, g2: torch.Tensor) -> None:
    """fp32 ``slot`` += column sums of the ``[T, N]`` gradient ``g2`` (HIP column-sum kernel on the GPU)."""
    if g2.is_cuda and slot.is_contiguous() and slot.dtype == torch.float32 and g2.stride(-1) == 1:
        from . import hip_kernels as K
        K.colsum_accum(g2, g2.stride(0), slot, g2.shape[0], g2.shape[1])
    else:
        slot.add_(g2.float().sum(0))


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
        ctx.p, ctx.flat = W_E, _flat
        return _flat.shadow_view(W_E)[tokens]

    @staticmethod
    def backward(ctx, g):
        (tokens,) = ctx.saved_tensors
        from ..engine import grad_hooks
        W_E = ctx.p
        slot = W_E.grad
        if slot is None:
            slot = ctx.flat.bind_zero(W_E)
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
        y = _mm_bias(x2, Wm, _flat.shadow_view(b) if b is not None else None)
        ctx.save_for_backward(x2)
        ctx.W, ctx.b, ctx.flat, ctx.lead = W, b, _flat, lead
        return y.view(*lead, y.shape[-1])

    @staticmethod
    def backward(ctx, gy):
        from ..engine import grad_hooks
        (x2,) = ctx.saved_tensors
        W, b, flat = ctx.W, ctx.b, ctx.flat
        g2 = gy.reshape(-1, gy.shape[-1]).to(x2.dtype)
        dx = None
        if ctx.needs_input_grad[0]:
            dx = (g2 @ flat.shadow_view(W).t()).view(*ctx.lead, W.shape[0])
        bsum = None
        if b is not None and b.requires_grad:
            if b.grad is None:
                flat.bind_zero(b)
            bsum = b.grad if (b.grad.is_contiguous() and b.grad.dtype == torch.float32) else None
        if W.requires_grad:
            from .gemm_dispatch import wgrad_into
            # the bias gradient (colsum of g2) comes out of the weight-gradient GEMM (``bsum``)
            if flat.claim(W):  # lazily-zeroed slot: store (beta = 0), with its share of the fused clip norm
                wgrad_into(W.grad, x2, g2, store=True, params=(W,), bsum=bsum)
            else:
                slot = W.grad
                if slot is None:
                    slot = W.grad = torch.zeros_like(W)
                wgrad_into(slot, x2, g2, store=False, bsum=bsum)
            grad_hooks.notify(W)
        else:
            bsum = None
        if b is not None and b.requires_grad:
            if bsum is None:
                _bias_grad_accumulate(b.grad, g2)
            grad_hooks.notify(b)
        return dx, None, None, None


class _MirrorMat(torch.autograd.Function):
    """``y = x @ Wm (+ bm)`` for an arena matrix given as explicit 2-D views: ``wm`` / ``bm`` of the bf16
    mirror, ``gw`` / ``gb`` of the fp32 gradient arena.  The weight gradient is one fp32-output GEMM
    accumulating into ``gw`` (``addmm``, beta = 1); ``params`` are reported to the DP reducer.  Used for
    matrices whose TL shape is not 2-D: the packed ``W_Q|W_K|W_V`` group ``[d][(H + 2 H_kv) dh]`` and
    ``W_O [H, dh, d]`` as ``[H dh][d]``."""

    @staticmethod
    def forward(ctx, x, wm, bm, gw, gb, wparams, bparams, *leaves):
        lead = x.shape[:-1]
        x2 = x.reshape(-1, x.shape[-1])
        y = _mm_bias(x2, wm, bm)
        ctx.save_for_backward(x2)
        ctx.wm, ctx.gw, ctx.gb, ctx.lead, ctx.n_leaves = wm, gw, gb, lead, len(leaves)
        ctx.wparams, ctx.bparams = wparams, bparams
        return y.view(*lead, y.shape[-1])

    @staticmethod
    def backward(ctx, gy):
        from ..engine import grad_hooks
        (x2,) = ctx.saved_tensors
        g2 = gy.reshape(-1, gy.shape[-1]).to(x2.dtype)
        dx = None
        if ctx.needs_input_grad[0]:
            dx = (g2 @ ctx.wm.t()).view(*ctx.lead, ctx.wm.shape[0])
        if ctx.gb is not None:
            for b in ctx.bparams:
                if b.grad is None:
                    b._iit_flat.bind_zero(b)
        fused_b = ctx.gw is not None and ctx.gb is not None and ctx.gb.is_contiguous()
        if ctx.gw is not None:
            from .gemm_dispatch import wgrad_into
            flat = ctx.wparams[0]._iit_flat
            # a claimed (lazily-zeroed) slot is stored (beta = 0), else accumulated; the bias gradient (colsum of
            # g2) comes out of the same GEMM
            wgrad_into(ctx.gw, x2, g2, store=flat.claim(*ctx.wparams), params=ctx.wparams,
                       bsum=ctx.gb if fused_b else None)
        if ctx.gb is not None and not fused_b:
            _bias_grad_accumulate(ctx.gb, g2)
        for p in ctx.wparams + ctx.bparams:
            grad_hooks.notify(p)
        return (dx, None, None, None, None, None, None) + (None,) * ctx.n_leaves


class _MirrorMatResid(torch.autograd.Function):
    """``y = resid + x @ Wm (+ bm)``: :class:`_MirrorMat` with the residual add in the GEMM's epilogue (hipBLASLt
    ``addmm`` with beta = 1 reads ``resid`` as C) -- the pre-norm block's skip connection without a separate [T, d]
    elementwise pass.  ``resid``'s gradient is ``gy`` itself."""

    @staticmethod
    def forward(ctx, x, resid, wm, bm, gw, gb, wparams, bparams, *leaves):
        lead = x.shape[:-1]
        x2 = x.reshape(-1, x.shape[-1])
        r2 = resid.reshape(-1, resid.shape[-1]).to(wm.dtype)
        y = torch.addmm(r2, x2, wm)
        if bm is not None:
            y = y + bm
        ctx.save_for_backward(x2)
        ctx.wm, ctx.gw, ctx.gb, ctx.lead, ctx.n_leaves = wm, gw, gb, lead, len(leaves)
        ctx.wparams, ctx.bparams = wparams, bparams
        ctx.rdtype = resid.dtype
        return y.view(*lead, y.shape[-1])

    @staticmethod
    def backward(ctx, gy):
        dx = _MirrorMat.backward(ctx, gy)[0]
        dres = gy.to(ctx.rdtype) if ctx.needs_input_grad[1] else None
        return (dx, dres) + (None,) * (6 + ctx.n_leaves)


class _SplitQKV(torch.autograd.Function):
    """``q, k, v`` head views of the packed projection output ``y [..., (H + 2 H_kv) dh]``.  The backward
    concatenates their gradients into one ``[..., N]`` tensor with one launch; autograd's three slice backwards
    would each zero-fill a y-sized tensor, copy into it and add the three (~25 ms/step of fills, strided copies and
    adds on Llama-3-8B at S = 512, profiles/llama3_8b_s512_step_breakdown_r4.txt)."""

    @staticmethod
    def forward(ctx, y, H: int, Hkv: int, dh: int):
        lead = y.shape[:-1]
        ctx.lead, ctx.dims = lead, (H * dh, Hkv * dh, Hkv * dh)
        q = y[..., :H * dh].view(*lead, H, dh)
        k = y[..., H * dh:(H + Hkv) * dh].view(*lead, Hkv, dh)
        v = y[..., (H + Hkv) * dh:].view(*lead, Hkv, dh)
        ctx.dtype, ctx.device = y.dtype, y.device
        return q, k, v

    @staticmethod
    def backward(ctx, dq, dk, dv):
        parts = [torch.zeros(*ctx.lead, n, dtype=ctx.dtype, device=ctx.device) if g is None
                 else g.reshape(*ctx.lead, n).to(ctx.dtype) for g, n in zip((dq, dk, dv), ctx.dims)]
        return torch.cat(parts, -1), None, None, None


def _bound_to_arena(flat, p: torch.Tensor) -> bool:
    """``p.grad`` is the arena view at ``p``'s offset (so writing the arena is writing ``p.grad``)."""
    g = p.grad  # None: lazily zeroed (FlatParams.zero_grad) -- the backward claims / binds the slot itself
    return g is None or (g.data_ptr() == flat.grad.data_ptr() + flat.offset_of(p) * 4 and g.stride() == p.stride())


class TorchOps:
    name = "torch"
    fused = False

    # ops whose outputs IIT_EMULATE_BF16=act rounds to bf16 (the activations a bf16 engine stores between ops)
    _EMU_ACT_OPS = ("embed", "pos_embed", "layer_norm", "qkv", "attention", "o_proj", "mlp_in", "mlp_out", "unembed")

    def __init__(self, dtype: torch.dtype = torch.float32):
        self.dtype = dtype
        # precision study (scripts/iia_ceiling.py, profiles/iia_precision_r6.txt): an fp32 backend that rounds its
        # weights ("w") and/or its op outputs ("act") to bf16 -- forward values and, through the casts' autograd,
        # the activation gradients -- to find which bf16 rounding changes a training trajectory.  Off by default.
        import os
        emu = set(os.environ.get("IIT_EMULATE_BF16", "").split(",")) - {""} if dtype == torch.float32 else set()
        self.emu_w = "w" in emu
        if "act" in emu:
            for name in self._EMU_ACT_OPS:
                setattr(self, name, self._rounding(getattr(self, name)))

    @staticmethod
    def _rounding(fn):
        def rnd(t):
            if isinstance(t, torch.Tensor) and t.dtype == torch.float32:
                return t.to(torch.bfloat16).to(torch.float32)
            if isinstance(t, tuple):
                return tuple(rnd(u) for u in t)
            return t

        def wrapped(*args, **kwargs):
            return rnd(fn(*args, **kwargs))
        return wrapped

    # -- helpers --------------------------------------------------------------
    def w(self, p: torch.Tensor) -> torch.Tensor:
        if p.dtype == self.dtype:
            if getattr(self, "emu_w", False) and p.dtype == torch.float32:
                # bf16-rounded value, gradient straight through to the fp32 parameter
                return p + (p.detach().to(torch.bfloat16).to(torch.float32) - p.detach())
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

    def embed_spliced(self, tokens, W_E, index, src):
        """``embed`` with an interchange splice of ``hook_embed`` applied inside the gather (one HIP pass over the
        bf16 mirror, ``hip_ops.EmbedSpliceFn``), or None when not covered -- the caller then splices separately."""
        if self.dtype != torch.bfloat16 or W_E.dtype == self.dtype or not tokens.is_cuda:
            return None
        m = _arena_mirror(W_E)
        if m is None:
            return None
        from . import hip_ops
        if not hip_ops.llama_fused_ok(m[1]):
            return None
        return hip_ops.embed_spliced(tokens, W_E, m[0], index, src)

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
        if hook_scale is None and hook_normalized is None and self.dtype == torch.bfloat16 and x.is_cuda \
                and x.shape[-1] % 8 == 0 and x.shape[-1] <= 8192 and x.dtype in (torch.bfloat16, torch.float32) \
                and (w is None or (w.dtype == torch.float32 and w.is_contiguous())):
            import os
            if os.environ.get("IIT_LLAMA_FUSED", "1") != "0":
                from . import hip_ops
                return hip_ops.RMSNormFn.apply(x, w, eps)  # csrc/llama_ops.hip: one pass fwd, one + dw bwd
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
        if x.is_cuda and x.dtype == torch.bfloat16 and x.stride(-1) == 1 and cos.dtype == torch.float32 \
                and cos.is_contiguous() and sin.is_contiguous() and rotary_dim % 2 == 0:
            from . import hip_ops
            if hip_ops.llama_fused_ok(x):
                return hip_ops.RotaryFn.apply(x, cos, sin, rotary_dim, offset, adjacent_pairs)
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

    def _packed_qkv(self, x, W_Q, W_K, W_V, b_Q, b_K, b_V):
        """One GEMM over the packed arena group (see ``qkv_arena_groups``) on the bf16 mirror, or None."""
        if self.dtype != torch.bfloat16 or not x.is_cuda or W_Q.dim() != 3:
            return None
        m = _arena_mirror(W_Q)
        if m is None:
            return None
        flat = m[0]
        H, d, dh = W_Q.shape
        Hkv = W_K.shape[0]
        Ht = H + 2 * Hkv
        N = Ht * dh
        ws = (W_Q, W_K, W_V)
        if any(w.stride() != (dh, N, 1) or not flat.owns(w) for w in ws):
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
        grad = torch.is_grad_enabled() and all(w.requires_grad for w in ws)
        if grad and not all(_bound_to_arena(flat, p) for p in ws + (bs if packed_b else ())):
            return None
        sh = flat.shadow
        wm = sh.as_strided((d, N), (N, 1), off)
        bm = sh.as_strided((N,), (1,), boff) if packed_b else None
        xb = x.to(torch.bfloat16)
        if not grad:
            y = _mm_bias(xb.reshape(-1, d), wm, bm).view(*x.shape[:-1], N)
        else:
            gw = flat.grad.as_strided((d, N), (N, 1), off)
            gb = flat.grad.as_strided((N,), (1,), boff) if packed_b else None
            bp = bs if packed_b else ()
            y = _MirrorMat.apply(xb, wm, bm, gw, gb, ws, bp, *(ws + bp))
            return _SplitQKV.apply(y, H, Hkv, dh)
        lead = x.shape[:-1]
        q = y[..., :H * dh].view(*lead, H, dh)
        k = y[..., H * dh:(H + Hkv) * dh].view(*lead, Hkv, dh)
        v = y[..., (H + Hkv) * dh:].view(*lead, Hkv, dh)
        return q, k, v

    def qkv(self, x, W_Q, W_K, W_V, b_Q, b_K, b_V):
        packed = self._packed_qkv(x, W_Q, W_K, W_V, b_Q, b_K, b_V)
        if packed is not None:
            return packed
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
            # a python-scalar fill (no host->device tensor copy, so the op is capturable in a HIP graph)
            scores = scores.masked_fill(~mask, ignore)
        if hook_scores is not None:
            scores = hook_scores(scores)
        pattern = F.softmax(scores, dim=-1)
        pattern = torch.where(torch.isnan(pattern), torch.zeros_like(pattern), pattern)
        if hook_pattern is not None:
            pattern = hook_pattern(pattern)
        z = torch.einsum("bkhe,bhqk->bqhe", v, pattern)
        return z

    def o_proj(self, z, W_O, b_O):
        if self.dtype == torch.bfloat16 and z.is_cuda and W_O.is_contiguous():
            m = _arena_mirror(W_O)
            mb = _arena_mirror(b_O) if (b_O is not None and b_O.is_contiguous()) else None
            if m is not None and (b_O is None or mb is not None):
                flat = m[0]
                H, dh, d = W_O.shape
                wm = m[1].view(H * dh, d)
                grad = torch.is_grad_enabled() and W_O.requires_grad
                z2 = z.to(torch.bfloat16).reshape(*z.shape[:-2], H * dh)
                if not grad:
                    return _mm_bias(z2.reshape(-1, H * dh), wm, None if mb is None else mb[1]).view(
                        *z2.shape[:-1], d)
                if _bound_to_arena(flat, W_O) and (b_O is None or _bound_to_arena(flat, b_O)):
                    bp = () if b_O is None else (b_O,)
                    gw = flat.grad.as_strided((H * dh, d), (d, 1), flat.offset_of(W_O))
                    gb = None if b_O is None else flat.grad.as_strided((d,), (1,), flat.offset_of(b_O))
                    return _MirrorMat.apply(z2, wm, None if mb is None else mb[1], gw, gb, (W_O,), bp, W_O, *bp)
        return torch.einsum("bshe,hed->bsd", z, self.w(W_O)) + self.w(b_O)

    def o_result(self, z, W_O):
        return torch.einsum("bshe,hed->bshd", z, self.w(W_O))

    # -- residual epilogues (bf16 arena mirror on a GPU): the skip connection inside the projection GEMM --------
    @property
    def fuses_residual(self) -> bool:
        import os
        # opt-in until tests/test_llama_ops.py::test_llama_torch_backend_residual_epilogue_* has run on an MI355X
        return self.dtype == torch.bfloat16 and os.environ.get("IIT_TORCH_RESID_EPI", "0") == "1"

    def _mat_resid(self, x2, resid, W, b, wm, gw_shape):
        """``resid + x2 @ wm (+ b)`` for arena weight ``W`` viewed as the 2-D mirror ``wm``; None when the
        arena path does not apply (the caller adds the residual itself)."""
        m = _arena_mirror(W)
        mb = _arena_mirror(b) if (b is not None and b.is_contiguous()) else None
        if m is None or (b is not None and mb is None) or not x2.is_cuda:
            return None
        flat = m[0]
        if not torch.is_grad_enabled() or not W.requires_grad:
            r2 = resid.reshape(-1, resid.shape[-1]).to(torch.bfloat16)
            y = torch.addmm(r2, x2.reshape(-1, x2.shape[-1]), wm)
            if mb is not None:
                y = y + mb[1]
            return y.view(*resid.shape[:-1], y.shape[-1])
        if not (_bound_to_arena(flat, W) and (b is None or _bound_to_arena(flat, b))):
            return None
        bp = () if b is None else (b,)
        gw = flat.grad.as_strided(gw_shape, (gw_shape[1], 1), flat.offset_of(W))
        gb = None if b is None else flat.grad.as_strided((gw_shape[1],), (1,), flat.offset_of(b))
        return _MirrorMatResid.apply(x2, resid, wm, None if mb is None else mb[1], gw, gb, (W,), bp, W, *bp)

    def o_proj_residual(self, z, W_O, b_O, resid):
        if self.fuses_residual and z.is_cuda and W_O.is_contiguous():
            m = _arena_mirror(W_O)
            if m is not None:
                H, dh, d = W_O.shape
                out = self._mat_resid(z.to(torch.bfloat16).reshape(*z.shape[:-2], H * dh), resid, W_O, b_O,
                                      m[1].view(H * dh, d), (H * dh, d))
                if out is not None:
                    return out
        return self.residual(resid, self.o_proj(z, W_O, b_O))

    def mlp_out_residual(self, post, W_out, b_out, resid):
        if self.fuses_residual and post.is_cuda and W_out.dim() == 2 and W_out.is_contiguous():
            m = _arena_mirror(W_out)
            if m is not None:
                out = self._mat_resid(post.to(torch.bfloat16), resid, W_out, b_out, m[1], tuple(W_out.shape))
                if out is not None:
                    return out
        return self.residual(resid, self.mlp_out(post, W_out, b_out))

    def rms_norm_fork(self, x, w, eps):
        """``(RMSNorm(x), x_passthrough)`` -- the backward adds the skip gradient inside the norm kernel -- or None
        when the fused kernel does not apply."""
        if not (self.dtype == torch.bfloat16 and x.is_cuda and x.shape[-1] % 8 == 0 and x.shape[-1] <= 8192
                and x.dtype in (torch.bfloat16, torch.float32) and (w is None or (w.dtype == torch.float32
                                                                                   and w.is_contiguous()))):
            return None
        import os
        if os.environ.get("IIT_LLAMA_FUSED", "1") == "0" or os.environ.get("IIT_RMS_FORK", "0") != "1":
            return None  # (the fork is opt-in until validated on hardware, like the residual epilogue)
        from . import hip_ops
        return hip_ops.RMSNormForkFn.apply(x, w, eps)

    def mlp_in(self, x, W_in, b_in, act: str, hook_pre=None):
        pre = self.lin(x, W_in, b_in)
        if hook_pre is not None:
            pre = hook_pre(pre)
        return pre, act_fn(act)(pre)

    def mlp_gated_in(self, x, W_gate, W_in, b_in, act: str, hook_pre=None, hook_pre_linear=None, splice=None):
        """TL ``GatedMLP``: ``pre = x W_gate`` (hook_pre), ``pre_linear = x W_in + b_in``, ``post = act(pre) * pre_linear``.

        ``splice`` (a plan ``Splice`` of ``hook_post``, optional): returns ``(pre, post, spliced)``, where
        ``spliced`` says the splice was applied inside the SwiGLU kernel (the producer's epilogue); otherwise the
        caller applies it at the hook site."""
        pre = self.lin(x, W_gate)
        if act == "silu" and hook_pre is None and hook_pre_linear is None and pre.is_cuda \
                and pre.dtype == torch.bfloat16 and pre.shape[-1] % 8 == 0:
            from . import hip_ops
            if hip_ops.llama_fused_ok(pre):
                pre_linear = self.lin(x, W_in, b_in)
                if splice is not None:
                    post = hip_ops.swiglu_spliced(pre, pre_linear, splice.index, splice.src)
                    if post is not None:
                        return pre, post, True
                    return pre, hip_ops.SwiGLUFn.apply(pre, pre_linear), False
                return pre, hip_ops.SwiGLUFn.apply(pre, pre_linear)
        if hook_pre is not None:
            pre = hook_pre(pre)
        pre_linear = self.lin(x, W_in, b_in)
        if hook_pre_linear is not None:
            pre_linear = hook_pre_linear(pre_linear)
        if splice is not None:
            return pre, act_fn(act)(pre) * pre_linear, False
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
