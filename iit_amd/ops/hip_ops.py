"""HIP op backend: autograd Functions over the hand-written gfx950 kernels.

Numerics: bf16 activations / GEMM operands, fp32 accumulation, fp32 residual
stream, fp32 master weights and gradients.

Weights: :class:`ModelShadow` keeps one bf16 compute copy of every matrix in TL
layout (packed ``[d][3HD]`` for QKV, 16-byte aligned rows for ``W_U``); the forward
GEMM reads it as a k-major operand through ``ds_read_b64_tr_b16``, the
input-gradient GEMM as a k-contiguous operand, so no transposed copies exist.
One batched ``shadow_refresh`` launch re-derives them after each optimizer update.
GEMMs go through :mod:`iit_amd.ops.gemm_dispatch` (hand-written MFMA kernel with
the fused epilogue, or hipBLASLt when it measures faster for a plain product).

Gradients: weight/bias gradients are accumulated *inside* the backward GEMM
epilogues straight into ``param.grad`` (the flat fp32 arena when present) and the
Function returns ``None`` for them; :mod:`iit_amd.engine.grad_hooks` tells the
data-parallel reducer the gradient is final.

Interventions: ``attention(..., patch_heads, patch_src)`` splices source ``z``
for the listed heads inside the attention kernel; patched heads produce zero
q/k/v gradient (the spliced value is a constant), exactly like the reference's
clone + index-put hook.
"""
from __future__ import annotations

import math
import os
from typing import Optional, Sequence

import torch
from torch.autograd import Function

from ..engine import grad_hooks
from . import hip_kernels as K
from .gemm_dispatch import gemm, gemm_pair
from .torch_ops import TorchOps, act_fn

BF16 = torch.bfloat16
F32 = torch.float32


def _pad8(n: int) -> int:
    return (n + 7) // 8 * 8


def _grad_slot(p: Optional[torch.Tensor]) -> Optional[torch.Tensor]:
    """``p.grad`` ready to be accumulated into (an arena parameter's lazily-zeroed slot is zeroed now)."""
    if p is None or not p.requires_grad:
        return None
    g = p.grad
    if g is None:
        flat = getattr(p, "_iit_flat", None)
        if flat is not None and flat.owns(p):
            return flat.bind_zero(p)
        g = torch.zeros_like(p, memory_format=torch.contiguous_format)
        p.grad = g
    return g


def _settle_claim(choice, *ps) -> None:
    """The dispatcher served a claimed (fresh) gradient with "zero + accumulate": hand its slot back to the
    arena's bulk zero_grad memset (one launch for all such slots) instead of a memset per GEMM."""
    if choice is not None and choice.startswith("z+"):
        ps[0]._iit_flat.unclaim(*ps)


def _claim_store(*ps) -> bool:
    """True when the caller's single GEMM may *store* the complete gradient of ``ps`` (see FlatParams.claim);
    the caller then passes ``fresh=True`` so the dispatcher may also pick "zero + split-K accumulate"."""
    if any(p is None or not p.requires_grad for p in ps):
        return False
    flat = getattr(ps[0], "_iit_flat", None)
    if flat is None or not all(flat.owns(p) for p in ps):
        return False
    return flat.claim(*ps)


_FUSE_BIAS = os.environ.get("IIT_FUSED_BIAS_SUMS", "1") != "0"
# width cap of the fused bias sums (default: none; capping them below the vocabulary width measured 0.4 % slower,
# profiles/bench_r3s2p_bias_cap_ab.txt)
_FUSE_BIAS_MAX_N = int(os.environ.get("IIT_FUSED_BIAS_MAX_N", str(1 << 30)))


def _fused_bias(gb: Optional[torch.Tensor], N: int) -> Optional[torch.Tensor]:
    """``gb`` (a bias-gradient slot of ``N`` floats) when the layer's weight-gradient GEMM may add the bias gradient
    ``colsum(dY)`` into it itself (``gemm(..., bsum=gb)``: fused into the LDS-DMA kernel's main loop, so dY is not
    read again by a column-sum pass); None outside that case (no slot, a strided slot, deterministic mode, where the
    fp32 atomics of the fused sums would make the bias gradient run-to-run variable, or ``IIT_FUSED_BIAS_SUMS=0``)."""
    if gb is None or not _FUSE_BIAS or not gb.is_cuda or gb.dtype != F32 or not gb.is_contiguous() or \
            gb.numel() != N or N > _FUSE_BIAS_MAX_N:
        return None
    from .gemm_dispatch import deterministic
    return None if deterministic() else gb


def _norm_slots(store: bool, *ps) -> Optional[torch.Tensor]:
    """The fused-norm slots (``FlatParams.norm_cover``) for a GEMM that stores the complete gradient of ``ps``
    (``store``); registers the producer's capability either way (``FlatParams.norm_intent``)."""
    flat = getattr(ps[0], "_iit_flat", None)
    if flat is None:
        return None
    flat.norm_intent(*ps)
    return flat.norm_cover(*ps) if store else None


def _done(*params):
    for p in params:
        if p is not None and p.requires_grad:
            grad_hooks.notify(p)


class _BiasSums:
    """Bias-gradient column sums of one backward pass, batched.

    Each fused backward adds ``colsum(dY)`` into its bias gradient; as separate launches these are ~36 small
    kernels per backward (one per bias).  Here they are queued -- the bf16 / fp32 operands stay referenced, and
    no kernel writes them after their producer -- and summed by ONE launch per 32 biases at the end of the
    autograd backward pass (an engine final callback, so every ``backward()`` -- eager, graph-captured, a staged
    DP segment -- ends with its biases complete).  The biases are reported to the data-parallel reducer when
    their sums land.  ``IIT_DEFER_BIAS_SUMS=0`` restores one launch per bias."""

    def __init__(self):
        self.items, self.params, self.stream = [], [], None
        self.task = None  # autograd graph task whose final callback will flush the queue

    def add(self, x, ld, out, T, N, *params):
        if _DEFER_BIAS_SUMS and x.is_cuda and K.colsum_vec_ok(x, ld, out, N) and self._armed():
            self.items.append((x, ld, out, T, N))
            self.params.extend(params)
            return
        K.colsum_accum(x, ld, out, T, N)
        _done(*params)

    def _armed(self) -> bool:
        """True when this backward pass's final callback is queued.  The queue is keyed by the autograd graph
        task: a backward that raised after queueing (e.g. an aborted graph capture) never ran its callback, and
        its stale items -- tensors of the failed pass -- are dropped instead of being summed into a later one."""
        task = torch._C._current_graph_task_id()
        if task < 0:
            return False  # not inside an autograd backward pass: the sum runs immediately
        if task == self.task:
            return True
        self.reset()
        try:
            torch.autograd.Variable._execution_engine.queue_callback(self.flush)
        except RuntimeError:
            return False
        self.task = task
        self.stream = torch.cuda.current_stream()
        return True

    def reset(self) -> None:
        self.items, self.params, self.stream, self.task = [], [], None, None

    def flush(self) -> None:
        items, params, stream = self.items, self.params, self.stream
        self.reset()
        if not items:
            return
        with torch.cuda.stream(stream):
            K.colsum_multi(items)
        _done(*params)


_DEFER_BIAS_SUMS = os.environ.get("IIT_DEFER_BIAS_SUMS", "1") != "0"
_BIAS_SUMS = _BiasSums()


# ============================================================================ shadow weights
class ModelShadow:
    """bf16 compute copies of a HookedTransformer's matrices, in the layouts the GEMMs read.

    Layouts: QKV packed ``[d][3*H*dh]`` (column ``which*H*dh + h*dh + e``), ``W_O`` as
    ``[H*dh][d]``, ``W_in`` ``[d][d_mlp]``, ``W_out`` ``[d_mlp][d]``, ``W_U`` ``[d][Vp]``
    (rows padded to 8 columns).  Each copy serves both GEMMs of its weight: the
    forward reads it as a k-major B operand (tr16 transpose reads), the
    input-gradient GEMM as a k-contiguous B operand, so no transposed copies exist.

    Two modes:

    * **mirror** (training): the flat arena is already in these layouts
      (``HookedTransformer._iit_arena_groups``), so the copies are views of the
      arena's bf16 mirror, which the fused Adam kernel writes in its update pass;
      nothing is re-derived per step.
    * **copy** (no arena, e.g. evaluation of a freshly loaded model): private bf16
      buffers refreshed by one batched ``shadow_refresh`` launch when the weights change.
    """

    def __init__(self, model):
        self.model = model
        cfg = model.cfg
        self.dev = next(model.parameters()).device
        self.H, self.d, self.dh = cfg.n_heads, cfg.d_model, cfg.d_head
        self.HD = self.H * self.dh
        self.V = cfg.d_vocab_out
        self.Vp = _pad8(self.V)
        self.layers = []
        self.U = None
        self.biases = []  # per layer: packed bf16 [3HD] QKV bias (mirror mode) or None
        self.mode = None
        self._layout_sig = None
        self._value_sig = None
        self._descs = None
        self._n = 0
        self._frozen = []

    # ------------------------------------------------------------------ mirror mode
    def _mirror_layout_ok(self, flat) -> bool:
        m = self.model
        H, d, dh, HD = self.H, self.d, self.dh, self.HD
        for blk in m.blocks:
            a = blk.attn
            if a.W_Q.stride() != (dh, 3 * HD, 1):
                return False
            if a.W_K.data_ptr() != a.W_Q.data_ptr() + HD * 4 or a.W_V.data_ptr() != a.W_Q.data_ptr() + 2 * HD * 4:
                return False
            if not a.W_O.is_contiguous():
                return False
            if not m.cfg.attn_only and not (blk.mlp.W_in.is_contiguous() and blk.mlp.W_out.is_contiguous()):
                return False
        W_U = self._W_U()
        if W_U is not None and W_U.stride() != (self.Vp, 1):
            return False
        return all(flat.owns(p) or self._frozen_plain(p) for p in self._matrices())

    def _frozen_plain(self, p) -> bool:
        """A frozen (``requires_grad=False``) contiguous fp32 ``W_O`` / ``W_in`` / ``W_out``: outside the arena, so
        the mirror binds a bf16 copy of it instead (refreshed when the parameter's version changes)."""
        if p.requires_grad or p.dtype != F32 or not p.is_contiguous():
            return False
        return any(p is b.attn.W_O or (not self.model.cfg.attn_only and (p is b.mlp.W_in or p is b.mlp.W_out))
                   for b in self.model.blocks)

    def _W_U(self):
        """The unembedding matrix, or None for models with another head (BERT classifier)."""
        ue = getattr(self.model, "unembed", None)
        return None if ue is None else ue.W_U

    def _bind_mirror(self, flat):
        sh = flat.ensure_shadow()
        m = self.model
        d, HD = self.d, self.HD
        self.layers, self.biases = [], []
        self._frozen = []  # (fp32 parameter, its bf16 copy) for frozen matrices outside the arena

        def view(p, rows, cols):
            if flat.owns(p):
                return sh.as_strided((rows, cols), (cols, 1), flat.offset_of(p))
            c = torch.empty(rows, cols, dtype=BF16, device=self.dev)
            self._frozen.append((p, c))
            return c
        for blk in m.blocks:
            a = blk.attn
            L = {"qkv": sh.as_strided((d, 3 * HD), (3 * HD, 1), flat.offset_of(a.W_Q)), "o": view(a.W_O, HD, d)}
            if not m.cfg.attn_only:
                dm = m.cfg.d_mlp
                L["in"] = view(blk.mlp.W_in, d, dm)
                L["out"] = view(blk.mlp.W_out, dm, d)
            self.layers.append(L)
            packed_b = (a.b_Q.requires_grad and flat.owns(a.b_Q) and a.b_Q.is_contiguous()
                        and a.b_K.data_ptr() == a.b_Q.data_ptr() + HD * 4
                        and a.b_V.data_ptr() == a.b_Q.data_ptr() + 2 * HD * 4)
            self.biases.append(sh.as_strided((3 * HD,), (1,), flat.offset_of(a.b_Q)) if packed_b else None)
        W_U = self._W_U()
        self.U = None if W_U is None else sh.as_strided((d, self.Vp), (self.Vp, 1), flat.offset_of(W_U))
        self._descs = None

    # ------------------------------------------------------------------ copy mode
    def _alloc_copies(self):
        cfg = self.model.cfg
        d, HD = self.d, self.HD
        e = lambda *s: torch.empty(*s, dtype=BF16, device=self.dev)  # noqa: E731
        self.layers, self.biases = [], []
        for _ in self.model.blocks:
            L = {"qkv": e(d, 3 * HD), "o": e(HD, d)}
            if not cfg.attn_only:
                L.update({"in": e(d, cfg.d_mlp), "out": e(cfg.d_mlp, d)})
            self.layers.append(L)
            self.biases.append(None)
        self.U = torch.zeros(d, self.Vp, dtype=BF16, device=self.dev) if self._W_U() is not None else None

    def _entries(self):
        m, cfg = self.model, self.model.cfg
        H, d, dh, HD = self.H, self.d, self.dh, self.HD
        out = []
        for blk, L in zip(m.blocks, self.layers):
            a = blk.attn
            for which, W in enumerate((a.W_Q, a.W_K, a.W_V)):
                # [H][d][dh] -> columns which*HD + h*dh + j of the packed [d][3HD] copy
                out.append((W.data_ptr(), L["qkv"].data_ptr() + which * HD * 2, d, dh, 3 * HD, 0, H, d * dh, dh))
            out.append((a.W_O.data_ptr(), L["o"].data_ptr(), HD, d, d, 0))
            if not cfg.attn_only:
                mlp, dm = blk.mlp, cfg.d_mlp
                out.append((mlp.W_in.data_ptr(), L["in"].data_ptr(), d, dm, dm, 0))
                out.append((mlp.W_out.data_ptr(), L["out"].data_ptr(), dm, d, d, 0))
        W_U = self._W_U()
        if W_U is not None:
            # one single-row "head" per row of W_U: handles a padded (arena) row stride on the fp32 side
            out.append((W_U.data_ptr(), self.U.data_ptr(), 1, self.V, self.Vp, 0, d, W_U.stride(0), self.Vp))
        return out

    def _matrices(self):
        m = self.model
        ps = []
        for blk in m.blocks:
            a = blk.attn
            ps += [a.W_Q, a.W_K, a.W_V, a.W_O]
            if not m.cfg.attn_only:
                ps += [blk.mlp.W_in, blk.mlp.W_out]
        if self._W_U() is not None:
            ps.append(self._W_U())
        return ps

    # ------------------------------------------------------------------ per forward
    def ensure(self):
        m = self.model
        flat = getattr(m, "_flat_params", None)
        wv = getattr(m, "_iit_weights_version", 0)
        if flat is not None:
            layout = ("flat", id(flat), flat.data.data_ptr())
            if layout != self._layout_sig:
                self.mode = "mirror" if self._mirror_layout_ok(flat) else "copy"
                if self.mode == "mirror":
                    self._bind_mirror(flat)
                self._layout_sig = layout
                self._value_sig = None
            if self.mode != "mirror":
                join = getattr(m, "_param_join", None)  # the copies read every weight: no overlapped update
                if join is not None:
                    join()
            if self.mode == "mirror":
                pv = sum(p._version for p in flat.params)
                if flat.mirror_version != wv or pv != self._value_sig:
                    flat.refresh_shadow()
                    self._value_sig = pv
                if self._frozen:
                    fv = (wv, tuple(p._version for p, _ in self._frozen))
                    if fv != getattr(self, "_frozen_sig", None):
                        for p, c in self._frozen:
                            c.copy_(p.detach().view(c.shape))
                        self._frozen_sig = fv
                return
            value = (wv, flat.version)
        else:
            layout = tuple(p.data_ptr() for p in self._matrices())
            value = (wv, tuple(p._version for p in self._matrices()))
        if self.mode != "copy" or self._descs is None or layout != self._layout_sig:
            for p in self._matrices():
                if p.dtype != F32 or p.stride(-1) != 1 or (p is not self._W_U() and not p.is_contiguous()):
                    raise RuntimeError("HIP backend needs contiguous fp32 master weights (or the flat arena)")
            self.mode = "copy"
            self._alloc_copies()
            entries = self._entries()
            self._descs = K.make_shadow_descs(entries, self.dev)
            self._n = len(entries)
            self._layout_sig = layout
            self._value_sig = None
        if value != self._value_sig:
            K.shadow_refresh(self._descs, self._n)
            self._value_sig = value

    def mark_stale(self):
        self._value_sig = None


# ============================================================================ autograd functions
def _flat2(t: torch.Tensor) -> torch.Tensor:
    return t.reshape(-1, t.shape[-1])


def _aligned_rows(g: torch.Tensor, T: int, N: int) -> torch.Tensor:
    """[T, N] view of ``g`` whose row stride is a multiple of 8 elements (16-byte vector loads)."""
    if g.is_contiguous():
        g2 = g.reshape(T, N)
    elif g.stride(-1) == 1:
        g2 = g.reshape(-1, N)
    else:
        g2 = g.contiguous().reshape(T, N)
    if g2.stride(0) % 8 != 0 or g2.stride(1) != 1:
        padded = torch.zeros(T, _pad8(N), dtype=g2.dtype, device=g2.device)
        padded[:, :N] = g2
        g2 = padded[:, :N]
    return g2


# ---- cold-operand prefetch for the dual dX + dW launches (profiles/dual_l2_hypothesis_r6.txt): inside the step a
# pair's forward-saved activation X and its weight come from HBM (7-19 % over back-to-back timing).  Every op whose
# backward launches a pair registers (X, W) in forward order; the backward's pair then prefetches the operands of the
# pair that runs right after it -- the previous registration -- from extra workgroups of its own launch
# (csrc/gemm_dual.hip).  The list holds references, so a prefetched range is always live memory.
_PF_SEQ: list = []
_PF_ON = [True]  # set per forward by HipOps.begin_forward (the model's ``prefetch`` policy)


def _pf_register(ctx, x2, w):
    if _PF_ON[0] and any(ctx.needs_input_grad):
        ctx.pf_idx = len(_PF_SEQ)
        _PF_SEQ.append((x2, w))


def _pf_next(ctx):
    i = getattr(ctx, "pf_idx", 0) - 1
    return _PF_SEQ[i] if 0 <= i < len(_PF_SEQ) else None


class EmbedPosFn(Function):
    @staticmethod
    def forward(ctx, tokens, W_E, W_pos):
        ctx.set_materialize_grads(False)
        B, S = tokens.shape
        d = W_E.shape[1]
        tok = tokens.contiguous()
        out = torch.empty(B, S, d, dtype=F32, device=tokens.device)
        K.embed_pos_fwd(tok, W_E, W_pos, out, B, S, d)
        ctx.save_for_backward(tok)
        ctx.params = (W_E, W_pos)
        return out

    @staticmethod
    def backward(ctx, g):
        if g is None:
            return None, None, None
        (tok,) = ctx.saved_tensors
        W_E, W_pos = ctx.params
        B, S = tok.shape
        K.embed_pos_bwd(tok, g.contiguous(), _grad_slot(W_E), _grad_slot(W_pos), B, S, W_E.shape[1])
        _done(W_E, W_pos)
        return None, None, None


class LayerNormFn(Function):
    @staticmethod
    def forward(ctx, x, w, b, eps):
        ctx.set_materialize_grads(False)
        shape = x.shape
        d = shape[-1]
        x2 = _flat2(x.float().contiguous())
        T = x2.shape[0]
        y = torch.empty(T, d, dtype=BF16, device=x.device)
        mean = torch.empty(T, dtype=F32, device=x.device)
        rstd = torch.empty(T, dtype=F32, device=x.device)
        K.ln_fwd(x2, w, b, y, mean, rstd, T, d, eps)
        ctx.save_for_backward(x2, mean, rstd)
        ctx.params = (w, b)
        ctx.in_dtype = x.dtype
        return y.view(*shape[:-1], d)

    @staticmethod
    def backward(ctx, dy):
        if dy is None:
            return None, None, None, None
        x2, mean, rstd = ctx.saved_tensors
        w, b = ctx.params
        T, d = x2.shape
        dx = torch.empty(T, d, dtype=F32, device=x2.device)
        dx16 = torch.empty(T, d, dtype=BF16, device=x2.device) if ctx.in_dtype == F32 else None
        dw = _grad_slot(w) if w is not None else None
        db = _grad_slot(b) if b is not None else None
        K.ln_bwd(_flat2(dy.contiguous()), x2, mean, rstd, w, dx, dw, db, T, d, dx16=dx16)
        _done(w, b)
        dx = dx.view(*dy.shape[:-1], d)
        if dx16 is None:
            return dx.to(ctx.in_dtype), None, None, None
        _set_bf16_twin(dx, dx16)
        return dx, None, None, None


class LayerNormTwinFn(Function):
    """``(LN(x), fp32(LN(x)))`` from one kernel pass (``iit_ln_fwd_twin``): a post-norm block (BERT) feeds the bf16
    output to the next GEMM and the fp32 copy to the residual epilogue of the GEMM after it, which read a cast of
    the bf16 output before -- a [T, d] cast pass forward, and backward a cast of the residual gradient plus
    autograd's bf16 sum of the two gradients.  The backward takes both gradients and adds the fp32 one inside the
    LN-backward kernel (``dy2``)."""

    @staticmethod
    def forward(ctx, x, w, b, eps):
        ctx.set_materialize_grads(False)
        shape = x.shape
        d = shape[-1]
        x2 = _flat2(x.float().contiguous())
        T = x2.shape[0]
        # allocated in the output shape (the outputs are not views: a multi-output Function's views may not be
        # modified in place downstream)
        y = torch.empty(*shape[:-1], d, dtype=BF16, device=x.device)
        y32 = torch.empty(*shape[:-1], d, dtype=F32, device=x.device)
        mean = torch.empty(T, dtype=F32, device=x.device)
        rstd = torch.empty(T, dtype=F32, device=x.device)
        yf, y32f = y.view(T, d), y32.view(T, d)
        if not K.ln_fwd_twin(x2, w, b, yf, y32f, mean, rstd, T, d, eps):
            K.ln_fwd(x2, w, b, yf, mean, rstd, T, d, eps)
            y32f.copy_(yf)
        ctx.save_for_backward(x2, mean, rstd)
        ctx.params = (w, b)
        ctx.in_dtype = x.dtype
        return y, y32

    @staticmethod
    def backward(ctx, dy, dy32):
        if dy is None and dy32 is None:
            return None, None, None, None
        x2, mean, rstd = ctx.saved_tensors
        w, b = ctx.params
        T, d = x2.shape
        lead = (dy if dy is not None else dy32).shape[:-1]
        dx = torch.empty(T, d, dtype=F32, device=x2.device)
        dx16 = torch.empty(T, d, dtype=BF16, device=x2.device) if ctx.in_dtype == F32 else None
        dw = _grad_slot(w) if w is not None else None
        db = _grad_slot(b) if b is not None else None
        if dy is None:
            g, g2 = _flat2(dy32.float().contiguous()), None
        else:
            g = _flat2(dy.contiguous())
            g2 = None if dy32 is None else _flat2(dy32.float().contiguous())
        K.ln_bwd(g, x2, mean, rstd, w, dx, dw, db, T, d, dx16=dx16, dy2=g2)
        _done(w, b)
        dx = dx.view(*lead, d)
        if dx16 is None:
            return dx.to(ctx.in_dtype), None, None, None
        _set_bf16_twin(dx, dx16)
        return dx, None, None, None


def _f32_of(t: torch.Tensor) -> torch.Tensor:
    """The fp32 twin a :class:`LayerNormTwinFn` output carries (same storage and version as when it was produced),
    else ``t`` itself: consumers that want an fp32 residual pass the twin as their autograd input, so its gradient
    reaches the LN backward in fp32."""
    twin = getattr(t, "_iit_f32", None)
    if twin is not None and twin[0] == t.data_ptr() and twin[1] == t._version and twin[2].shape == t.shape:
        return twin[2]
    return t


def _set_bf16_twin(t: torch.Tensor, t16: torch.Tensor) -> None:
    """Attach a bf16 copy to an fp32 gradient: its producer wrote both in one pass, so the consuming
    backward GEMMs skip a separate cast.  Tensor attributes survive autograd hand-off when the gradient
    has a single consumer; when autograd sums several gradients the twin is simply absent."""
    t._iit_bf16 = (t.data_ptr(), t._version, t16)


def _bf16_of(t: torch.Tensor) -> torch.Tensor:
    if t.dtype == BF16:
        return t
    twin = getattr(t, "_iit_bf16", None)
    if twin is not None and twin[0] == t.data_ptr() and twin[1] == t._version and twin[2].numel() == t.numel():
        return twin[2].view(t.shape)
    return t.to(BF16)


def _xhat16(w, b, d: int) -> bool:
    """The LN backward reads the forward's bf16 output as xhat (norms without weight and bias: 2 B per element instead
    of the fp32 input).  Round 3 reverted it over a staged-backward mismatch that round 4 traced to the split-store GEMM
    candidate (profiles/split_store_removal_r4.txt); ``IIT_LN_XHAT16=0`` reads the fp32 input."""
    return w is None and b is None and d % 4 == 0 and d <= 4096 and os.environ.get("IIT_LN_XHAT16", "1") == "1"


def _ln_fork_bwd(ctx, dy, dpass):
    xs, mean, rstd = ctx.saved_tensors
    w, b = ctx.params
    T, d = xs.shape
    dres = None
    if dpass is not None:
        dres = _flat2(dpass.float().contiguous())
    dx = torch.empty(T, d, dtype=F32, device=xs.device)
    dx16 = torch.empty(T, d, dtype=BF16, device=xs.device) if ctx.in_dtype == F32 else None
    if xs.dtype == BF16:
        K.ln_bwd_xh16(_flat2(dy.contiguous()), xs, rstd, dx, T, d, dres=dres, dx16=dx16)
    else:
        dw = _grad_slot(w) if w is not None else None
        db = _grad_slot(b) if b is not None else None
        K.ln_bwd(_flat2(dy.contiguous()), xs, mean, rstd, w, dx, dw, db, T, d, dres=dres, dx16=dx16)
        _done(w, b)
    dx = dx.view(*dy.shape[:-1], d)
    if dx16 is None:
        return dx.to(ctx.in_dtype), None, None, None
    _set_bf16_twin(dx, dx16)
    return dx, None, None, None


class LayerNormForkFn(Function):
    """``(LN(x), x)``: the second output carries the residual stream past the norm, so the backward gets
    both gradients and sums them inside the LN-backward kernel (no separate autograd add over [T, d])."""

    @staticmethod
    def forward(ctx, x, w, b, eps):
        ctx.set_materialize_grads(False)
        shape = x.shape
        d = shape[-1]
        x2 = _flat2(x.float().contiguous())
        T = x2.shape[0]
        y = torch.empty(T, d, dtype=BF16, device=x.device)
        mean = torch.empty(T, dtype=F32, device=x.device)
        rstd = torch.empty(T, dtype=F32, device=x.device)
        K.ln_fwd(x2, w, b, y, mean, rstd, T, d, eps)
        ctx.save_for_backward(y if _xhat16(w, b, d) else x2, mean, rstd)
        ctx.params = (w, b)
        ctx.in_dtype = x.dtype
        return y.view(*shape[:-1], d), x.view_as(x)

    @staticmethod
    def backward(ctx, dy, dpass):
        if dy is None:
            return dpass, None, None, None
        return _ln_fork_bwd(ctx, dy, dpass)


def _packed3(a: Optional[torch.Tensor], b: Optional[torch.Tensor], c: Optional[torch.Tensor], n: int) -> bool:
    """``a|b|c`` are consecutive ``n``-column blocks of ONE row-major buffer (the arena QKV layout).  Three separate
    allocations that merely sit next to each other (the caching allocator hands out adjacent blocks) do not count:
    a kernel writing 3n columns from ``a`` would run past ``a``'s storage (IIT_CHECK_BOUNDS flagged it)."""
    if a is None or b is None or c is None:
        return False
    st = a.untyped_storage().data_ptr()
    if b.untyped_storage().data_ptr() != st or c.untyped_storage().data_ptr() != st:
        return False
    es = a.element_size()
    return b.data_ptr() == a.data_ptr() + n * es and c.data_ptr() == a.data_ptr() + 2 * n * es


class QKVFn(Function):
    """x [B,S,d] bf16 -> packed qkv [B,S,3,H,dh] bf16 (bias fused); weights from the packed [d][3HD] shadow.

    With the flat arena in kernel layout the weight gradient ``[d][3HD]`` is one plain
    accumulate-GEMM into the arena and the three bias gradients one column sum."""

    @staticmethod
    def forward(ctx, x, layer, bias_bf16, W_Q, W_K, W_V, b_Q, b_K, b_V):
        ctx.set_materialize_grads(False)
        B, S, d = x.shape
        H, dh = W_Q.shape[0], W_Q.shape[2]
        HD = H * dh
        x2 = _flat2(x.to(BF16).contiguous())
        T = x2.shape[0]
        out = torch.empty(B, S, 3, H, dh, dtype=BF16, device=x.device)
        gemm(x2, layer["qkv"], out, M=T, N=3 * HD, K=d, lda=d, ldb=3 * HD, ldc=3 * HD, mode=K.MODE_BKM,
             epi=K.EPI_BF16_BIAS3, bias0=b_Q, bias1=b_K, bias2=b_V, bias_cols=HD, blas_bias=bias_bf16)
        ctx.save_for_backward(x2)
        ctx.layer = layer
        ctx.params = (W_Q, W_K, W_V, b_Q, b_K, b_V)
        ctx.dims = (B, S, d, H, dh)
        _pf_register(ctx, x2, layer["qkv"])
        return out

    @staticmethod
    def backward(ctx, dqkv):
        if dqkv is None:
            return (None,) * 9
        (x2,) = ctx.saved_tensors
        W_Q, W_K, W_V, b_Q, b_K, b_V = ctx.params
        B, S, d, H, dh = ctx.dims
        HD = H * dh
        T = B * S
        g = dqkv.to(BF16).contiguous().view(T, 3 * HD)
        dx = torch.empty(T, d, dtype=BF16, device=g.device)
        xspec = dict(A=g, B=ctx.layer["qkv"], C=dx, M=T, N=d, K=3 * HD, lda=3 * HD, ldb=3 * HD, ldc=d, epi=K.EPI_BF16)
        store = W_Q.stride() == (dh, 3 * HD, 1) and _packed3(W_Q, W_K, W_V, HD) and \
            _claim_store(W_Q, W_K, W_V)
        if store:
            gq, gk, gv = W_Q.grad, W_K.grad, W_V.grad
        else:
            gq, gk, gv = _grad_slot(W_Q), _grad_slot(W_K), _grad_slot(W_V)
        gbs = [_grad_slot(bp) for bp in (b_Q, b_K, b_V)]
        packed_b = all(gb is not None for gb in gbs) and all(gb.is_contiguous() for gb in gbs) and _packed3(*gbs, HD)
        bs = None
        if gq is not None and gk is not None and gv is not None and gq.stride() == (dh, 3 * HD, 1) and \
                _packed3(gq, gk, gv, HD):
            if packed_b:  # b_Q | b_K | b_V gradients are one [3 HD] run: the GEMM adds colsum(dqkv) into it
                bs = _fused_bias(torch.as_strided(gbs[0], (3 * HD,), (1,)), 3 * HD)
            choice = gemm_pair(xspec, dict(A=x2, B=g, C=gq, M=d, N=3 * HD, K=T, lda=d, ldb=3 * HD, ldc=3 * HD,
                                           mode=K.MODE_AKM | K.MODE_BKM,
                                           epi=K.EPI_F32_STORE if store else K.EPI_F32_ACC, fresh=store, bsum=bs,
                                           gsq=_norm_slots(store, W_Q, W_K, W_V)), prefetch=_pf_next(ctx))
            if store:
                _settle_claim(choice, W_Q, W_K, W_V)
        else:
            gemm(**xspec)
            if gq is not None and gk is not None and gv is not None:
                gemm(x2, g, gq, C2=gk, C3=gv, M=d, N=3 * HD, K=T, lda=d, ldb=3 * HD, ldc=0,
                     mode=K.MODE_AKM | K.MODE_BKM, epi=K.EPI_F32_ACC_QKV, qkv=(dh, H, d))
        if all(gb is not None for gb in gbs):
            if bs is not None:
                _done(b_Q, b_K, b_V)  # summed by the weight-gradient GEMM
            elif packed_b:
                _BIAS_SUMS.add(g, 3 * HD, gbs[0], T, 3 * HD, b_Q, b_K, b_V)
            else:
                K.colsum3_accum(g, 3 * HD, gbs, T, HD)
                _done(b_Q, b_K, b_V)
        _done(W_Q, W_K, W_V)
        return (dx.view(B, S, d),) + (None,) * 8


class AttnFn(Function):
    """packed qkv [B,S,3,H,dh] -> z [B,S,H,dh]; heads in ``mask`` take ``zsrc`` (interchange splice)."""

    @staticmethod
    def forward(ctx, qkv, zsrc, mask, causal, scale):
        ctx.set_materialize_grads(False)
        B, S, _, H, dh = qkv.shape
        qkv = qkv.contiguous()
        z = torch.empty(B, S, H, dh, dtype=BF16, device=qkv.device)
        lse = torch.empty(B * H * S, dtype=F32, device=qkv.device)
        src = None
        if mask:
            src = zsrc.to(BF16).contiguous()
        K.attn_small_fwd(qkv, z, lse, src, mask, B, S, H, dh, 3 * H * dh, H * dh, H * dh, scale, causal)
        ctx.save_for_backward(qkv, lse)
        ctx.cfg = (mask, causal, scale)
        return z

    @staticmethod
    def backward(ctx, dz):
        if dz is None:
            return None, None, None, None, None
        qkv, lse = ctx.saved_tensors
        mask, causal, scale = ctx.cfg
        B, S, _, H, dh = qkv.shape
        dz = dz.to(BF16).contiguous()
        dqkv = torch.empty_like(qkv)
        K.attn_small_bwd(qkv, dz, lse, dqkv, mask, B, S, H, dh, 3 * H * dh, H * dh, scale, causal)
        return dqkv, None, None, None, None


def _flash_grads(ctx, dz, q, k, v, dq, dk, dv):
    z, lse = ctx.saved_tensors[-2:]
    mask, causal, scale = ctx.cfg
    B, S, Hq, _ = q.shape
    dz = dz.to(BF16)
    if dz.stride(-1) != 1 or dz.stride(1) % 8 or dz.stride(2) % 8:
        dz = dz.contiguous()
    dd = torch.empty(B, Hq, S, dtype=F32, device=q.device)
    K.flash_bwd(q, k, v, z, dz, lse, dd, dq, dk, dv, mask, scale, causal, spec=getattr(ctx, "spec", None))


class FlashPackedFn(Function):
    """Tiled MFMA attention (csrc/flash_attn.hip) over a packed qkv [B,S,3,H,dh] bf16 -> z [B,S,H,dh] bf16.
    Heads in ``mask`` take ``zsrc`` (interchange splice) and get zero q/k/v gradients."""

    @staticmethod
    def forward(ctx, qkv, zsrc, mask, causal, scale):
        ctx.set_materialize_grads(False)
        B, S, _, H, dh = qkv.shape
        q, k, v = qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2]
        z = torch.empty(B, S, H, dh, dtype=BF16, device=qkv.device)
        lse = torch.empty(B, H, S, dtype=F32, device=qkv.device)
        src = zsrc.to(BF16).contiguous() if mask else None
        K.flash_fwd(q, k, v, z, lse, src, mask, scale, causal)
        ctx.save_for_backward(qkv, z, lse)
        ctx.cfg = (mask, causal, scale)
        return z

    @staticmethod
    def backward(ctx, dz):
        if dz is None:
            return None, None, None, None, None
        qkv = ctx.saved_tensors[0]
        dqkv = torch.empty_like(qkv)
        _flash_grads(ctx, dz, qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2], dqkv[:, :, 0], dqkv[:, :, 1], dqkv[:, :, 2])
        return dqkv, None, None, None, None


class FlashFn(Function):
    """Tiled MFMA attention over separate q [B,S,Hq,dh] and grouped k/v [B,S,Hkv,dh] (bf16, GQA-native).  With
    ``spec`` / ``src``: an interchange splice of ``hook_z`` at any patch-spec index, applied by the kernel's output
    store; the backward kernels read dO with the spliced elements zeroed (no splice pass, no masked dO copy)."""

    @staticmethod
    def forward(ctx, q, k, v, causal, scale, src=None, spec=None):
        ctx.set_materialize_grads(False)
        B, S, Hq, dh = q.shape
        z = torch.empty(B, S, Hq, dh, dtype=BF16, device=q.device)
        lse = torch.empty(B, Hq, S, dtype=F32, device=q.device)
        K.flash_fwd(q, k, v, z, lse, src, 0, scale, causal, spec=spec)
        ctx.save_for_backward(q, k, v, z, lse)
        ctx.cfg = (0, causal, scale)
        ctx.spec = spec
        ctx.keep = src  # the spec's source pointer must outlive the launch
        return z

    @staticmethod
    def backward(ctx, dz):
        if dz is None:
            return None, None, None, None, None, None, None
        q, k, v = ctx.saved_tensors[:3]
        dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
        _flash_grads(ctx, dz, q, k, v, dq, dk, dv)
        return dq, dk, dv, None, None, None, None


def _flash_view(t: torch.Tensor) -> torch.Tensor:
    t = t.to(BF16)
    if t.stride(-1) != 1 or t.stride(1) % 8 or t.stride(2) % 8 or t.stride(0) % 8 or t.data_ptr() % 16:
        t = t.contiguous()
    return t


def flash_supported(q: torch.Tensor) -> bool:
    """The tiled kernel covers bf16-able [B,S,H,dh] inputs on the GPU with dh 64 / 128."""
    return q.is_cuda and q.shape[-1] in (64, 128) and os.environ.get("IIT_FLASH", "1") != "0"


def flash_attention(q, k, v, causal: bool, attn_scale: float) -> torch.Tensor:
    """softmax(q k^T / attn_scale) v for q [B,S,Hq,dh], k/v [B,S,Hkv,dh] (Hkv | Hq), never materialising [S,S]."""
    return FlashFn.apply(_flash_view(q), _flash_view(k), _flash_view(v), causal, 1.0 / attn_scale)


def flash_attention_spliced(q, k, v, causal: bool, attn_scale: float, index, src) -> Optional[torch.Tensor]:
    """:func:`flash_attention` whose output ``z`` [B,S,Hq,dh] takes ``src[index]`` at ``index`` inside the kernel's
    store (an interchange splice of ``hook_z``; SpliceFn's gradient: none through the spliced elements).  None when
    the patch-spec table cannot express the index or ``src`` does not broadcast to z (the caller splices
    separately); ``IIT_FLASH_SPLICE=0`` disables."""
    if os.environ.get("IIT_FLASH_SPLICE", "1") == "0":
        return None
    from .splice import patch_spec
    B, S, Hq, dh = q.shape
    src = src.to(device=q.device, dtype=BF16)
    spec = patch_spec(index, (B, S, Hq, dh), src)
    if spec is None or tuple(spec.dims[i][0] for i in range(4)) != (B, S, Hq, dh):
        return None
    return FlashFn.apply(_flash_view(q), _flash_view(k), _flash_view(v), causal, 1.0 / attn_scale, src, spec)


# ============================================================================ Llama-family fused elementwise ops
# (used by the torch op backend on the GPU: csrc/llama_ops.hip)
def _c16(t: torch.Tensor) -> torch.Tensor:
    t = t.contiguous()
    return t if t.data_ptr() % 16 == 0 else t.clone()


class RMSNormFn(Function):
    """``x * rsqrt(mean(x^2) + eps) * w`` -> bf16; ``w``'s gradient accumulates into its fp32 slot."""

    @staticmethod
    def forward(ctx, x, w, eps):
        ctx.set_materialize_grads(False)
        d = x.shape[-1]
        x2 = _c16(x.reshape(-1, d))
        T = x2.shape[0]
        y = torch.empty(T, d, dtype=BF16, device=x.device)
        rstd = torch.empty(T, dtype=F32, device=x.device)
        K.rms_fwd(x2, None if w is None else w.detach(), y, rstd, T, d, eps)
        ctx.save_for_backward(x2, rstd)
        ctx.w = w
        ctx.shape = x.shape
        return y.view(*x.shape[:-1], d)

    @staticmethod
    def backward(ctx, dy):
        if dy is None:
            return None, None, None
        x2, rstd = ctx.saved_tensors
        w = ctx.w
        T, d = x2.shape
        dx = torch.empty_like(x2)
        dw = _grad_slot(w) if w is not None else None
        K.rms_bwd(_c16(dy.to(BF16).reshape(T, d)), x2, rstd, None if w is None else w.detach(), dx, dw, T, d)
        _done(w)
        return dx.view(ctx.shape), None, None


class RMSNormForkFn(Function):
    """``(RMSNorm(x), x)``: the second output carries the residual stream past the norm; the backward sums both
    gradients inside the RMSNorm-backward kernel (the pre-norm block's skip connection, no autograd add)."""

    @staticmethod
    def forward(ctx, x, w, eps):
        ctx.set_materialize_grads(False)
        d = x.shape[-1]
        x2 = _c16(x.reshape(-1, d))
        T = x2.shape[0]
        y = torch.empty(T, d, dtype=BF16, device=x.device)
        rstd = torch.empty(T, dtype=F32, device=x.device)
        K.rms_fwd(x2, None if w is None else w.detach(), y, rstd, T, d, eps)
        ctx.save_for_backward(x2, rstd)
        ctx.w = w
        ctx.shape = x.shape
        return y.view(*x.shape[:-1], d), x.view_as(x)

    @staticmethod
    def backward(ctx, dy, dpass):
        if dy is None:
            return dpass, None, None
        x2, rstd = ctx.saved_tensors
        w = ctx.w
        T, d = x2.shape
        dx = torch.empty_like(x2)
        dres = None
        if dpass is not None:
            dres = _c16(dpass.to(x2.dtype).reshape(T, d))
        dw = _grad_slot(w) if w is not None else None
        K.rms_bwd(_c16(dy.to(BF16).reshape(T, d)), x2, rstd, None if w is None else w.detach(), dx, dw, T, d,
                  dres=dres)
        _done(w)
        return dx.view(ctx.shape), None, None


class RotaryFn(Function):
    @staticmethod
    def forward(ctx, x, cos, sin, rd, offset, adjacent):
        out = torch.empty(x.shape, dtype=BF16, device=x.device)
        K.rotary(x, out, cos, sin, rd, offset, adjacent, False)
        ctx.cfg = (cos, sin, rd, offset, adjacent)
        return out

    @staticmethod
    def backward(ctx, g):
        cos, sin, rd, offset, adjacent = ctx.cfg
        g = g.to(BF16)
        if g.stride(-1) != 1:
            g = g.contiguous()
        dx = torch.empty(g.shape, dtype=BF16, device=g.device)
        K.rotary(g, dx, cos, sin, rd, offset, adjacent, True)
        return dx, None, None, None, None, None


class SwiGLUFn(Function):
    """``silu(gate) * up`` (TL GatedMLP with act_fn silu), bf16."""

    @staticmethod
    def forward(ctx, gate, up):
        gate, up = _c16(gate.to(BF16)), _c16(up.to(BF16))
        post = torch.empty_like(gate)
        K.swiglu_fwd(gate, up, post)
        ctx.save_for_backward(gate, up)
        return post

    @staticmethod
    def backward(ctx, dpost):
        gate, up = ctx.saved_tensors
        dg, du = torch.empty_like(gate), torch.empty_like(up)
        K.swiglu_bwd(_c16(dpost.to(BF16)), gate, up, dg, du)
        return dg, du


class SwiGLUSpliceFn(Function):
    """:class:`SwiGLUFn` with an interchange splice of its output applied inside the kernel (``csrc/llama_ops.hip``
    ``swiglu_splice_*``): selected elements take ``src``'s value, their gate / up gradients are zero."""

    @staticmethod
    def forward(ctx, gate, up, src, spec):
        gate, up = _c16(gate.to(BF16)), _c16(up.to(BF16))
        post = torch.empty_like(gate)
        K.swiglu_splice_fwd(gate, up, post, src, spec.ptr)
        ctx.save_for_backward(gate, up)
        ctx.spec = spec
        return post

    @staticmethod
    def backward(ctx, dpost):
        gate, up = ctx.saved_tensors
        dg, du = torch.empty_like(gate), torch.empty_like(up)
        K.swiglu_splice_bwd(_c16(dpost.to(BF16)), gate, up, dg, du, ctx.spec.ptr)
        return dg, du, None, None


def swiglu_spliced(pre, pre_linear, index, src) -> Optional[torch.Tensor]:
    """``silu(pre) * pre_linear`` with ``out[index] = src[index]`` fused into the SwiGLU kernel, or None when the
    patch-spec table cannot express the index / the shapes do not fit (the caller splices separately)."""
    from .splice import patch_spec
    if os.environ.get("IIT_SWIGLU_SPLICE", "1") == "0" or pre.shape[-1] % 8 or pre.dtype != BF16:
        return None
    if src.dtype != BF16 or src.device != pre.device:
        src = src.to(device=pre.device, dtype=BF16)
    spec = patch_spec(index, tuple(pre.shape), src)
    if spec is None or spec.dims[3][0] % 8:
        return None
    return SwiGLUSpliceFn.apply(pre, pre_linear, src, spec)


class EmbedSpliceFn(Function):
    """``W_E[tokens]`` from the arena's bf16 mirror with an interchange splice of ``hook_embed`` applied in the gather
    (``csrc/llama_ops.hip`` ``embed_splice_*``): selected elements take ``src``'s value; the backward adds the other
    elements' gradient into W_E's fp32 grad slot (no dense ``[V, d]`` gradient, as ``TorchOps._MirrorEmbed``)."""

    @staticmethod
    def forward(ctx, tokens, W_E, flat, src, spec):
        tok = tokens.reshape(-1).to(torch.int64).contiguous()
        W16 = flat.shadow_view(W_E)
        out = torch.empty(*tokens.shape, W_E.shape[-1], dtype=BF16, device=W_E.device)
        K.embed_splice_fwd(tok, W16, out, src, spec.ptr)
        ctx.save_for_backward(tok)
        ctx.p, ctx.flat, ctx.spec = W_E, flat, spec
        return out

    @staticmethod
    def backward(ctx, g):
        (tok,) = ctx.saved_tensors
        from ..engine import grad_hooks
        W_E = ctx.p
        slot = W_E.grad
        if slot is None:
            slot = ctx.flat.bind_zero(W_E)
        g = g.reshape(-1, g.shape[-1])
        if g.dtype not in (BF16, torch.float32):
            g = g.float()
        K.embed_splice_bwd(tok, g.contiguous(), slot, ctx.spec.ptr)
        grad_hooks.notify(W_E)
        return None, None, None, None, None


def embed_spliced(tokens, W_E, flat, index, src) -> Optional[torch.Tensor]:
    """``W_E[tokens]`` (bf16 mirror) with ``out[index] = src[index]`` fused into the gather, or None when the
    patch-spec table cannot express the index / the shapes do not fit (the caller splices separately)."""
    from .splice import patch_spec
    d = W_E.shape[-1]
    if os.environ.get("IIT_EMBED_SPLICE", "1") == "0" or d % 8 or W_E.stride(-1) != 1 or W_E.stride(0) % 8:
        return None
    if src.dtype != BF16 or src.device != W_E.device:
        src = src.to(device=W_E.device, dtype=BF16)
    shape = tuple(tokens.shape) + (d,)
    spec = patch_spec(index, shape, src)
    if spec is None or spec.dims[3][0] % 8:
        return None
    return EmbedSpliceFn.apply(tokens, W_E, flat, src, spec)


def llama_fused_ok(x: torch.Tensor) -> bool:
    """The Llama-family fused kernels apply: a bf16 activation on the GPU (``IIT_LLAMA_FUSED=0`` disables)."""
    return x.is_cuda and x.dtype == BF16 and os.environ.get("IIT_LLAMA_FUSED", "1") != "0"


class LinearFn(Function):
    """y = x @ W + b, TL-layout master W [K, N] with bf16 shadow ``w`` (row stride ``ldw``).

    out kinds: ``bf16``, ``f32`` (store, padded row stride) or ``resid`` (fp32 ``resid + xW + b``).
    """

    @staticmethod
    def forward(ctx, x, W, b, w, ldw, resid, out_kind):
        ctx.set_materialize_grads(False)
        lead = x.shape[:-1]
        Kd = x.shape[-1]
        N = W.shape[-1]
        x2 = _flat2(x.to(BF16).contiguous())
        T = x2.shape[0]
        dev = x.device
        if out_kind == "bf16":
            out = torch.empty(T, N, dtype=BF16, device=dev)
            gemm(x2, w, out, M=T, N=N, K=Kd, lda=Kd, ldb=ldw, ldc=N, mode=K.MODE_BKM, epi=K.EPI_BF16, bias0=b)
            res = out.view(*lead, N)
        elif out_kind == "f32":
            Np = _pad8(N)
            out = torch.empty(T, Np, dtype=F32, device=dev)
            gemm(x2, w, out, M=T, N=N, K=Kd, lda=Kd, ldb=ldw, ldc=Np, mode=K.MODE_BKM, epi=K.EPI_F32_STORE, bias0=b)
            res = out[:, :N]
            res = res.unflatten(0, lead) if len(lead) != 1 else res
        else:
            r2 = _flat2(resid.float().contiguous())
            out = torch.empty(T, N, dtype=F32, device=dev)
            gemm(x2, w, out, M=T, N=N, K=Kd, lda=Kd, ldb=ldw, ldc=N, mode=K.MODE_BKM, epi=K.EPI_F32_RESID, bias0=b,
                 resid=r2, ldr=N)
            res = out.view(*lead, N)
        ctx.save_for_backward(x2)
        ctx.params = (W, b)
        ctx.w = w
        _pf_register(ctx, x2, w)
        ctx.ldw = ldw
        ctx.meta = (lead, Kd, N, out_kind, x.dtype)
        return res

    @staticmethod
    def backward(ctx, gy):
        if gy is None:
            return (None,) * 7
        (x2,) = ctx.saved_tensors
        W, b = ctx.params
        lead, Kd, N, out_kind, x_dtype = ctx.meta
        T = x2.shape[0]
        # one bf16 copy of an fp32 gradient (residual-stream outputs) serves both GEMMs and the bias sum;
        # the skip connection keeps the fp32 gradient
        gres = gy if out_kind == "resid" else None
        g16 = _bf16_of(gy)
        g2 = _aligned_rows(g16, T, N)
        ldg = g2.stride(0)
        dx = xspec = dxb = None
        if ctx.needs_input_grad[0]:
            amode = K.MODE_NN
            _, splits = K._tiling(T, Kd, N, True)
            if splits == 1:  # run below, paired with the weight gradient when it has one
                dxb = torch.empty(T, Kd, dtype=BF16, device=g2.device)
                xspec = dict(A=g2, B=ctx.w, C=dxb, M=T, N=Kd, K=N, lda=ldg, ldb=ctx.ldw, ldc=Kd, mode=amode,
                             epi=K.EPI_BF16)
            else:  # long reduction (unembed: K = vocab) -> split-K into fp32
                dxf = torch.zeros(T, Kd, dtype=F32, device=g2.device)
                gemm(g2, ctx.w, dxf, M=T, N=Kd, K=N, lda=ldg, ldb=ctx.ldw, ldc=Kd, mode=amode, epi=K.EPI_F32_ACC,
                     splits=splits)
                dx = dxf.to(x_dtype).view(*lead, Kd)
        store = _claim_store(W)
        gW = W.grad if store else _grad_slot(W)
        gb = _grad_slot(b)
        bs = _fused_bias(gb, N) if gW is not None else None
        if gW is not None:
            mode = K.MODE_AKM | K.MODE_BKM
            gW2 = gW.reshape(Kd, N) if gW.is_contiguous() else gW
            assert gW2.stride(-1) == 1 and gW2.dim() == 2, "weight gradient must have unit column stride"
            wspec = dict(A=x2, B=g2, C=gW2, M=Kd, N=N, K=T, lda=Kd, ldb=ldg, ldc=gW2.stride(0), mode=mode,
                         epi=K.EPI_F32_STORE if store else K.EPI_F32_ACC, fresh=store, bsum=bs,
                         gsq=_norm_slots(store, W))
            choice = gemm_pair(xspec, wspec, prefetch=_pf_next(ctx)) if xspec is not None else gemm(**wspec)
            if store:
                _settle_claim(choice, W)
        elif xspec is not None:
            gemm(**xspec)
        if dxb is not None:
            dx = (dxb if x_dtype == BF16 else dxb.to(x_dtype)).view(*lead, Kd)
        if gb is not None:
            if bs is not None:
                _done(b)  # summed by the weight-gradient GEMM
            else:
                _BIAS_SUMS.add(g2, ldg, gb, T, N, b)
        _done(W)
        return dx, None, None, None, None, gres, None


class MLPInFn(Function):
    """(pre, post) = (x @ W_in + b_in, gelu_new(pre)) in one GEMM epilogue."""

    @staticmethod
    def forward(ctx, x, W_in, b_in, w, erf=False):
        ctx.set_materialize_grads(False)
        ctx.erf = erf
        lead = x.shape[:-1]
        d = x.shape[-1]
        dm = W_in.shape[1]
        x2 = _flat2(x.to(BF16).contiguous())
        T = x2.shape[0]
        post = torch.empty(T, dm, dtype=BF16, device=x.device)
        pre = torch.empty(T, dm, dtype=BF16, device=x.device)
        gemm(x2, w, post, C2=pre, M=T, N=dm, K=d, lda=d, ldb=dm, ldc=dm, ldc2=dm, mode=K.MODE_BKM, epi=K.EPI_GELU_ERF if erf else K.EPI_GELU,
             bias0=b_in)
        ctx.save_for_backward(x2, pre)
        ctx.params = (W_in, b_in)
        ctx.w = w
        _pf_register(ctx, x2, w)
        ctx.meta = (lead, d, dm)
        return pre.view(*lead, dm), post.view(*lead, dm)

    @staticmethod
    def backward(ctx, gpre, gpost):
        if gpre is None and gpost is None:
            return None, None, None, None, None
        x2, pre = ctx.saved_tensors
        W_in, b_in = ctx.params
        lead, d, dm = ctx.meta
        T = x2.shape[0]
        if gpost is not None:
            dpre = torch.empty(T, dm, dtype=BF16, device=x2.device)
            K.dgelu(gpost.to(BF16).contiguous().view(T, dm), pre, dpre, erf=ctx.erf)
            zs = getattr(ctx, "zero_spec", None)
            if zs is not None:  # MLPInPairFn's in-op splice: the spliced post elements carry no gradient
                K.sparse_pair(dpre, T, dm, zs.ptr, 1)
            if gpre is not None:
                dpre = (dpre.float() + gpre.float().reshape(T, dm)).to(BF16)
        else:
            dpre = gpre.to(BF16).contiguous().view(T, dm)
        dx = torch.empty(T, d, dtype=BF16, device=x2.device)
        xspec = dict(A=dpre, B=ctx.w, C=dx, M=T, N=d, K=dm, lda=dm, ldb=dm, ldc=d, epi=K.EPI_BF16)
        store = W_in.is_contiguous() and _claim_store(W_in)
        gW = W_in.grad if store else _grad_slot(W_in)
        summed = _bias_sum_done(gpre if gpost is None else None, b_in)  # by MLPOutGeluFn's DGELU epilogue
        gb = None if summed else _grad_slot(b_in)
        bs = _fused_bias(gb, dm) if gW is not None else None
        if gW is not None:
            choice = gemm_pair(xspec, dict(A=x2, B=dpre, C=gW, M=d, N=dm, K=T, lda=d, ldb=dm, ldc=dm,
                                           mode=K.MODE_AKM | K.MODE_BKM,
                                           epi=K.EPI_F32_STORE if store else K.EPI_F32_ACC, fresh=store, bsum=bs,
                                           gsq=_norm_slots(store, W_in)), prefetch=_pf_next(ctx))
            if store:
                _settle_claim(choice, W_in)
        else:
            gemm(**xspec)
        if gb is not None and bs is None:
            _BIAS_SUMS.add(dpre, dm, gb, T, dm, b_in)
        else:
            _done(b_in)
        _done(W_in)
        return dx.view(*lead, d), None, None, None, None


def _bias_sum_done(g: Optional[torch.Tensor], b: Optional[torch.Tensor]) -> bool:
    """Whether ``g``'s producer already added its column sums into ``b``'s gradient (MLPOutGeluFn's fused
    epilogue); the tag is checked against the tensor's storage and version, like the bf16 twin."""
    tag = getattr(g, "_iit_bias_sum", None) if g is not None else None
    return tag is not None and b is not None and tag == (g.data_ptr(), g._version, id(b))


class MLPOutGeluFn(Function):
    """``resid + gelu(pre) @ W_out + b_out`` with the gradient taken w.r.t. ``pre`` (``post`` comes in as
    data: ``post = gelu(pre)`` from :class:`MLPInFn`'s epilogue, the block's only use of it; gelu_new, or the
    exact erf form with ``erf``).

    The backward's dX GEMM runs with the DGELU epilogue -- ``dpre = (g W_out^T) * gelu_new'(pre)`` in one pass --
    and, on the LDS-DMA kernel, reduces dpre into the b_in gradient in the same epilogue (tagged on dpre so
    MLPInFn skips its column sum).  Used only when neither ``hook_pre``, ``hook_post`` nor ``hook_mlp_out`` is
    live, so ``pre`` has no other consumer whose gradient autograd could add to the tagged tensor."""

    @staticmethod
    def forward(ctx, pre, post, W, b, w, ldw, resid, b_in, erf=False):
        ctx.set_materialize_grads(False)
        ctx.erf = erf
        lead = post.shape[:-1]
        Kd = post.shape[-1]
        N = W.shape[-1]
        x2 = _flat2(post)
        T = x2.shape[0]
        r2 = _flat2(resid.float().contiguous())
        out = torch.empty(T, N, dtype=F32, device=post.device)
        gemm(x2, w, out, M=T, N=N, K=Kd, lda=Kd, ldb=ldw, ldc=N, mode=K.MODE_BKM, epi=K.EPI_F32_RESID, bias0=b,
             resid=r2, ldr=N)
        ctx.save_for_backward(x2, _flat2(pre))
        ctx.params = (W, b, b_in)
        ctx.w = w
        _pf_register(ctx, x2, w)
        ctx.ldw = ldw
        ctx.meta = (lead, Kd, N)
        return out.view(*lead, N)

    @staticmethod
    def backward(ctx, gy):
        if gy is None:
            return (None,) * 9
        x2, pre2 = ctx.saved_tensors
        W, b, b_in = ctx.params
        lead, Kd, N = ctx.meta
        T = x2.shape[0]
        g16 = _bf16_of(gy)
        g2 = _aligned_rows(g16, T, N)
        ldg = g2.stride(0)
        dpre = xspec = gbi = None
        if ctx.needs_input_grad[0]:
            dpre = torch.empty(T, Kd, dtype=BF16, device=g2.device)
            gbi = _grad_slot(b_in)
            xspec = dict(A=g2, B=ctx.w, C=dpre, M=T, N=Kd, K=N, lda=ldg, ldb=ctx.ldw, ldc=Kd, mode=K.MODE_NN,
                         epi=K.EPI_DGELU_ERF if ctx.erf else K.EPI_DGELU, aux=pre2, ldc2=pre2.stride(0), colsum=gbi)
        store = _claim_store(W)
        gW = W.grad if store else _grad_slot(W)
        gb = _grad_slot(b)
        bs = _fused_bias(gb, N) if gW is not None else None
        if gW is not None:
            gW2 = gW.reshape(Kd, N) if gW.is_contiguous() else gW
            assert gW2.stride(-1) == 1 and gW2.dim() == 2, "weight gradient must have unit column stride"
            wspec = dict(A=x2, B=g2, C=gW2, M=Kd, N=N, K=T, lda=Kd, ldb=ldg, ldc=gW2.stride(0),
                         mode=K.MODE_AKM | K.MODE_BKM, epi=K.EPI_F32_STORE if store else K.EPI_F32_ACC, fresh=store,
                         bsum=bs, gsq=_norm_slots(store, W))
            choice = gemm_pair(xspec, wspec, prefetch=_pf_next(ctx)) if xspec is not None else gemm(**wspec)
            if store:
                _settle_claim(choice, W)
        elif xspec is not None:
            gemm(**xspec)
        if dpre is not None:
            dpre = dpre.view(*lead, Kd)
            if gbi is not None:
                dpre._iit_bias_sum = (dpre.data_ptr(), dpre._version, id(b_in))
        if gb is not None:
            if bs is not None:
                _done(b)  # summed by the weight-gradient GEMM
            else:
                _BIAS_SUMS.add(g2, ldg, gb, T, N, b)
        _done(W)
        return dpre, None, None, None, None, None, gy, None, None


class CrossEntropyFn(Function):
    """mean_r CE(logits[r], labels[r]) over fp32 logits with any row stride; fused fwd stats + bwd."""

    @staticmethod
    def forward(ctx, logits, labels):
        ctx.set_materialize_grads(False)
        R, V = logits.shape
        if logits.stride(1) != 1:
            logits = logits.contiguous()
        ld = logits.stride(0)
        loss = torch.empty(R, dtype=F32, device=logits.device)
        lse = torch.empty(R, dtype=F32, device=logits.device)
        lab = labels.contiguous()
        K.ce_fwd(logits, ld, lab, loss, lse, None, R, V)
        ctx.save_for_backward(logits, lab, lse)
        return loss.mean()

    @staticmethod
    def backward(ctx, g):
        if g is None:
            return None, None
        logits, lab, lse = ctx.saved_tensors
        R, V = logits.shape
        ld = logits.stride(0)
        ldo = _pad8(V)
        # fp32 (autograd casts a gradient to its input's dtype anyway) plus, in the same pass, the bf16 twin with
        # the same padded row stride that the unembed backward GEMMs read
        buf = torch.empty(R, ldo, dtype=F32, device=logits.device)
        buf16 = torch.empty(R, ldo, dtype=BF16, device=logits.device)
        gs = g.reshape(1).float().contiguous()
        K.ce_bwd(logits, ld, lab, lse, gs, 1.0 / R, buf, ldo, R, V, out16=buf16)
        res = buf[:, :V]
        _set_bf16_twin(res, buf16[:, :V])
        return res, None


def cross_entropy(logits: torch.Tensor, labels: torch.Tensor) -> torch.Tensor:
    return CrossEntropyFn.apply(logits.float(), labels)


# ============================================================================ paired (source + base) rows
# One launch per op over the rows of BOTH runs of an interchange intervention: the base run (rows [0, B), with
# autograd) and the no-grad source run (rows [B, 2B)) share every weight, so up to the deepest splice site the two
# forwards are one M = 2T batch (the reference runs them as two forwards,
# /root/reference/iit/model_pairs/base_model_pair.py:80-98).  Each paired Function computes over the full rows,
# returns the base rows as its (differentiable) output, appends the full result to ``box`` for the source side
# and saves only base-row slices for the backward -- the backward is the unpaired op's, unchanged, so source rows
# cost no backward work and produce no gradient (the reference's source run is under no_grad).


class Paired:
    """An activation of a paired forward: ``full`` [2B, ...] (rows [0, B) base, [B, 2B) source) and ``base``, the
    autograd-visible tensor holding the values of ``full[:B]`` (a view of it, or a passthrough of such a view)."""

    __slots__ = ("base", "full", "f32")

    def __init__(self, base: torch.Tensor, full: torch.Tensor, f32=None):
        # f32: (base32, full32) fp32 twins of a bf16 LN output (LayerNormPairTwinFn) for residual consumers
        self.base, self.full, self.f32 = base, full, f32

    def resid_operands(self):
        """(autograd base, fp32 full) for a residual epilogue: the fp32 twins when present (no cast pass; the base
        twin's gradient reaches the LN backward in fp32), else the bf16 base and a cast of ``full``."""
        if self.f32 is not None:
            return self.f32
        return self.base, self.full.float().contiguous()

    @property
    def nb(self) -> int:
        return self.base.shape[0]

    @property
    def src(self) -> torch.Tensor:
        return self.full[self.nb:]


class EmbedPosPairFn(EmbedPosFn):
    @staticmethod
    def forward(ctx, tokens, W_E, W_pos, tokens_full, box):
        ctx.set_materialize_grads(False)
        B2, S = tokens_full.shape
        d = W_E.shape[1]
        B = tokens.shape[0]
        out = torch.empty(B2, S, d, dtype=F32, device=tokens.device)
        K.embed_pos_fwd(tokens_full, W_E, W_pos, out, B2, S, d)
        ctx.save_for_backward(tokens_full[:B])
        ctx.params = (W_E, W_pos)
        box.append(out)
        return out[:B]

    @staticmethod
    def backward(ctx, g):
        return EmbedPosFn.backward(ctx, g) + (None, None)


class LayerNormForkPairFn(LayerNormForkFn):
    @staticmethod
    def forward(ctx, x, w, b, eps, x_full, box):
        ctx.set_materialize_grads(False)
        d = x.shape[-1]
        B = x.shape[0]
        x2 = _flat2(x_full)
        T2 = x2.shape[0]
        T = T2 * B // x_full.shape[0]
        y = torch.empty(T2, d, dtype=BF16, device=x.device)
        mean = torch.empty(T2, dtype=F32, device=x.device)
        rstd = torch.empty(T2, dtype=F32, device=x.device)
        K.ln_fwd(x2, w, b, y, mean, rstd, T2, d, eps)
        ctx.save_for_backward(y[:T] if _xhat16(w, b, d) else x2[:T], mean[:T], rstd[:T])
        ctx.params = (w, b)
        ctx.in_dtype = x.dtype
        yf = y.view(*x_full.shape[:-1], d)
        box.append(yf)
        return yf[:B], x.view_as(x)

    @staticmethod
    def backward(ctx, dy, dpass):
        return LayerNormForkFn.backward(ctx, dy, dpass) + (None, None)


class LayerNormPairTwinFn(Function):
    """:class:`LayerNormPairFn` (no position splice) that also writes the fp32 twin of both row sets in the same
    pass (``iit_ln_fwd_twin``) -- :class:`LayerNormTwinFn` for the paired forward: outputs (base bf16, base fp32),
    ``box`` gets (full bf16, full fp32); the backward adds the fp32 output's gradient inside the LN backward."""

    @staticmethod
    def forward(ctx, x, w, b, eps, x_full, box):
        ctx.set_materialize_grads(False)
        d = x.shape[-1]
        B = x.shape[0]
        x2 = _flat2(x_full)
        T2 = x2.shape[0]
        T = T2 * B // x_full.shape[0]
        y = torch.empty(T2, d, dtype=BF16, device=x.device)
        y32 = torch.empty(T2, d, dtype=F32, device=x.device)
        mean = torch.empty(T2, dtype=F32, device=x.device)
        rstd = torch.empty(T2, dtype=F32, device=x.device)
        if not K.ln_fwd_twin(x2, w, b, y, y32, mean, rstd, T2, d, eps):
            K.ln_fwd(x2, w, b, y, mean, rstd, T2, d, eps)
            y32.copy_(y)
        ctx.save_for_backward(x2[:T], mean[:T], rstd[:T])
        ctx.params = (w, b)
        ctx.in_dtype = x.dtype
        yf = y.view(*x_full.shape[:-1], d)
        yf32 = y32.view(*x_full.shape[:-1], d)
        box.append((yf, yf32))
        return yf[:B], yf32[:B]

    @staticmethod
    def backward(ctx, dy, dy32):
        return LayerNormTwinFn.backward(ctx, dy, dy32) + (None, None)


class LayerNormPairFn(LayerNormFn):
    """LN of both row sets (a post-LN block's residual output, BERT): bf16 ``Paired``; backward = LayerNormFn's on
    the base rows."""

    @staticmethod
    def forward(ctx, x, w, b, eps, x_full, box, pos_mask=0):
        ctx.set_materialize_grads(False)
        d = x.shape[-1]
        B = x.shape[0]
        x2 = _flat2(x_full)
        T2 = x2.shape[0]
        T = T2 * B // x_full.shape[0]
        y = torch.empty(T2, d, dtype=BF16, device=x.device)
        mean = torch.empty(T2, dtype=F32, device=x.device)
        rstd = torch.empty(T2, dtype=F32, device=x.device)
        S = x.shape[1] if x.dim() == 3 else 1
        if pos_mask:  # whole-position splice of the base rows from the source rows, inside the LN kernel
            K.ln_fwd_sel(x2, w, b, y, mean, rstd, T2, d, eps, pos_mask, S, T)
        else:
            K.ln_fwd(x2, w, b, y, mean, rstd, T2, d, eps)
        ctx.save_for_backward(x2[:T], mean[:T], rstd[:T])
        ctx.params = (w, b)
        ctx.in_dtype = x.dtype
        ctx.sel = (pos_mask, S)
        yf = y.view(*x_full.shape[:-1], d)
        box.append(yf)
        return yf[:B]

    @staticmethod
    def backward(ctx, dy):
        pos_mask, S = ctx.sel
        if not pos_mask:
            return LayerNormFn.backward(ctx, dy) + (None, None, None)
        if dy is None:
            return (None,) * 7
        x2, mean, rstd = ctx.saved_tensors
        w, b = ctx.params
        T, d = x2.shape
        dx = torch.empty(T, d, dtype=F32, device=x2.device)
        dx16 = torch.empty(T, d, dtype=BF16, device=x2.device) if ctx.in_dtype == F32 else None
        dw = _grad_slot(w) if w is not None else None
        db = _grad_slot(b) if b is not None else None
        K.ln_bwd_sel(_flat2(dy.contiguous()), x2, mean, rstd, w, dx, dw, db, T, d, pos_mask, S, dx16=dx16)
        _done(w, b)
        dx = dx.view(*dy.shape[:-1], d)
        if dx16 is None:
            return (dx.to(ctx.in_dtype),) + (None,) * 6
        _set_bf16_twin(dx, dx16)
        return (dx,) + (None,) * 6


class QKVPairFn(QKVFn):
    @staticmethod
    def forward(ctx, x, layer, bias_bf16, W_Q, W_K, W_V, b_Q, b_K, b_V, x_full, box):
        ctx.set_materialize_grads(False)
        B, S, d = x.shape
        B2 = x_full.shape[0]
        H, dh = W_Q.shape[0], W_Q.shape[2]
        HD = H * dh
        x2 = _flat2(x_full)
        T2 = x2.shape[0]
        out = torch.empty(B2, S, 3, H, dh, dtype=BF16, device=x.device)
        gemm(x2, layer["qkv"], out, M=T2, N=3 * HD, K=d, lda=d, ldb=3 * HD, ldc=3 * HD, mode=K.MODE_BKM,
             epi=K.EPI_BF16_BIAS3, bias0=b_Q, bias1=b_K, bias2=b_V, bias_cols=HD, blas_bias=bias_bf16)
        ctx.save_for_backward(x2[:B * S])
        ctx.layer = layer
        ctx.params = (W_Q, W_K, W_V, b_Q, b_K, b_V)
        ctx.dims = (B, S, d, H, dh)
        _pf_register(ctx, x2[:B * S], layer["qkv"])
        box.append(out)
        return out[:B]

    @staticmethod
    def backward(ctx, dqkv):
        return QKVFn.backward(ctx, dqkv) + (None, None)


class AttnPairFn(AttnFn):
    """Paired attention; heads in ``mask`` (an interchange splice of those heads of ``hook_z``) are computed once, by
    the source rows, and stored into the base rows too -- the base rows of those heads carry no gradient."""

    @staticmethod
    def forward(ctx, qkv, causal, scale, mask, qkv_full, box):
        ctx.set_materialize_grads(False)
        B = qkv.shape[0]
        B2, S, _, H, dh = qkv_full.shape
        z = torch.empty(B2, S, H, dh, dtype=BF16, device=qkv.device)
        lse = torch.empty(B2 * H * S, dtype=F32, device=qkv.device)
        if mask:
            K.attn_pair_fwd(qkv_full, z, lse, B2, S, H, dh, 3 * H * dh, H * dh, scale, causal, pair_seqs=B,
                            pair_mask=mask)
        else:
            K.attn_small_fwd(qkv_full, z, lse, None, 0, B2, S, H, dh, 3 * H * dh, H * dh, H * dh, scale, causal)
        ctx.save_for_backward(qkv_full[:B], lse[:B * H * S])  # lse rows are (batch, head)-major
        ctx.cfg = (mask, causal, scale)
        box.append(z)
        return z[:B]

    @staticmethod
    def backward(ctx, dz):
        g = AttnFn.backward(ctx, dz)
        return (g[0], None, None, None, None, None)


class AttnPairSpecFn(Function):
    """Paired attention with a general interchange splice of ``hook_z`` (any patch-spec index over the base rows'
    ``[B, S, H, dh]`` z: positions, head lists, feature ranges) applied in the attention kernel's store -- the source
    rows' selected elements are written into the base rows -- and the gradient mask in its backward (SURVEY K04 /
    K10: the z-epilogue patch point with per-head and per-position masks)."""

    @staticmethod
    def forward(ctx, qkv, causal, scale, spec, qkv_full, box):
        ctx.set_materialize_grads(False)
        B = qkv.shape[0]
        B2, S, _, H, dh = qkv_full.shape
        z = torch.empty(B2, S, H, dh, dtype=BF16, device=qkv.device)
        lse = torch.empty(B2 * H * S, dtype=F32, device=qkv.device)
        K.attn_pair_fwd_spec(qkv_full, z, lse, B2, S, H, dh, 3 * H * dh, H * dh, scale, causal, B, spec.ptr)
        ctx.save_for_backward(qkv_full[:B], lse[:B * H * S])
        ctx.cfg = (spec, causal, scale)
        box.append(z)
        return z[:B]

    @staticmethod
    def backward(ctx, dz):
        if dz is None:
            return None, None, None, None, None, None
        qkv, lse = ctx.saved_tensors
        spec, causal, scale = ctx.cfg
        B, S, _, H, dh = qkv.shape
        qkv = qkv.contiguous()
        dz = dz.to(BF16).contiguous()
        dqkv = torch.empty_like(qkv)
        K.attn_bwd_spec(qkv, dz, lse, dqkv, B, S, H, dh, 3 * H * dh, H * dh, scale, causal, spec.ptr)
        return dqkv, None, None, None, None, None


class LinearPairFn(LinearFn):
    """bf16 out or fp32 ``resid + xW + b`` out (``resid_full`` paired with the input rows)."""

    @staticmethod
    def forward(ctx, x, W, b, w, ldw, resid, out_kind, x_full, resid_full, box):
        ctx.set_materialize_grads(False)
        B = x.shape[0]
        lead = x.shape[:-1]
        Kd = x.shape[-1]
        N = W.shape[-1]
        x2 = _flat2(x_full)
        T2 = x2.shape[0]
        T = T2 * B // x_full.shape[0]
        if out_kind == "bf16":
            out = torch.empty(T2, N, dtype=BF16, device=x.device)
            gemm(x2, w, out, M=T2, N=N, K=Kd, lda=Kd, ldb=ldw, ldc=N, mode=K.MODE_BKM, epi=K.EPI_BF16, bias0=b)
        else:
            r2 = _flat2(resid_full)
            out = torch.empty(T2, N, dtype=F32, device=x.device)
            gemm(x2, w, out, M=T2, N=N, K=Kd, lda=Kd, ldb=ldw, ldc=N, mode=K.MODE_BKM, epi=K.EPI_F32_RESID, bias0=b,
                 resid=r2, ldr=N)
        ctx.save_for_backward(x2[:T])
        ctx.params = (W, b)
        ctx.w = w
        _pf_register(ctx, x2[:T], w)
        ctx.ldw = ldw
        ctx.meta = (lead, Kd, N, out_kind, x.dtype)
        of = out.view(*x_full.shape[:-1], N)
        box.append(of)
        return of[:B]

    @staticmethod
    def backward(ctx, gy):
        return LinearFn.backward(ctx, gy) + (None, None, None)


class MLPInPairFn(MLPInFn):
    """Paired W_in GEMM (+ gelu epilogue) over base and source rows.  ``spec`` (a PatchSpec over the base rows'
    ``mlp.hook_post`` [B, S, d_mlp], optional): the interchange splice of that site inside this op -- right after the
    GEMM the selected elements of the source half are copied into the base half in place (one thread per selected
    element, not a pass over the activation), and the backward zeroes the same elements of its dpre (the spliced
    values are constants).  ``pre`` keeps the base rows' own values, which the masked dgelu never reads."""

    @staticmethod
    def forward(ctx, x, W_in, b_in, w, erf, x_full, spec, box):
        ctx.set_materialize_grads(False)
        ctx.erf = erf
        ctx.zero_spec = spec
        B = x.shape[0]
        lead = x.shape[:-1]
        d = x.shape[-1]
        dm = W_in.shape[1]
        x2 = _flat2(x_full)
        T2 = x2.shape[0]
        T = T2 * B // x_full.shape[0]
        post = torch.empty(T2, dm, dtype=BF16, device=x.device)
        pre = torch.empty(T2, dm, dtype=BF16, device=x.device)
        gemm(x2, w, post, C2=pre, M=T2, N=dm, K=d, lda=d, ldb=dm, ldc=dm, ldc2=dm, mode=K.MODE_BKM,
             epi=K.EPI_GELU_ERF if erf else K.EPI_GELU, bias0=b_in)
        if spec is not None:
            K.sparse_pair(post, T, dm, spec.ptr, 0)
        ctx.save_for_backward(x2[:T], pre[:T])
        ctx.params = (W_in, b_in)
        ctx.w = w
        _pf_register(ctx, x2[:T], w)
        ctx.meta = (lead, d, dm)
        pf, qf = pre.view(*x_full.shape[:-1], dm), post.view(*x_full.shape[:-1], dm)
        box.append((pf, qf))
        return pf[:B], qf[:B]

    @staticmethod
    def backward(ctx, gpre, gpost):
        return MLPInFn.backward(ctx, gpre, gpost) + (None, None, None)


class MLPOutGeluPairFn(MLPOutGeluFn):
    @staticmethod
    def forward(ctx, pre, post, W, b, w, ldw, resid, b_in, erf, post_full, resid_full, box):
        ctx.set_materialize_grads(False)
        ctx.erf = erf
        B = post.shape[0]
        lead = post.shape[:-1]
        Kd = post.shape[-1]
        N = W.shape[-1]
        x2 = _flat2(post_full)
        T2 = x2.shape[0]
        T = T2 * B // post_full.shape[0]
        r2 = _flat2(resid_full)
        out = torch.empty(T2, N, dtype=F32, device=post.device)
        gemm(x2, w, out, M=T2, N=N, K=Kd, lda=Kd, ldb=ldw, ldc=N, mode=K.MODE_BKM, epi=K.EPI_F32_RESID, bias0=b,
             resid=r2, ldr=N)
        ctx.save_for_backward(x2[:T], _flat2(pre))
        ctx.params = (W, b, b_in)
        ctx.w = w
        _pf_register(ctx, x2[:T], w)
        ctx.ldw = ldw
        ctx.meta = (lead, Kd, N)
        of = out.view(*post_full.shape[:-1], N)
        box.append(of)
        return of[:B]

    @staticmethod
    def backward(ctx, gy):
        return MLPOutGeluFn.backward(ctx, gy) + (None, None, None)


class PairSpliceFn(Function):
    """Splice at a paired site: ``out_full[:B] = base`` with ``index`` taken from the source rows at the same
    positions, ``out_full[B:] = source`` -- one launch of the patch-spec kernel over a leading (base, source) axis.
    Gradient: the base gradient with the spliced elements zeroed (exactly :class:`iit_amd.ops.splice.SpliceFn`)."""

    @staticmethod
    def forward(ctx, act, act_full, spec_pair, spec_base, box):
        out = torch.empty_like(act_full)
        B = act.shape[0]
        K.splice(act_full, act_full[B:], out, act_full.numel(), spec_pair.ptr, act_full.dtype == F32, 0)
        ctx.spec = spec_base
        box.append(out)
        return out[:B]

    @staticmethod
    def backward(ctx, g):
        if g is None:
            return None, None, None, None, None
        g = g.contiguous()
        out = torch.empty_like(g)
        K.splice(g, None, out, g.numel(), ctx.spec.ptr, g.dtype == F32, 1)
        return out, None, None, None, None


def _one(fn, *args):
    box = []
    out = fn.apply(*args, box)
    return out, box[0]


# ============================================================================ op backend
class HipOps(TorchOps):
    name = "hip"
    fused = True

    def __init__(self, model):
        super().__init__(BF16)
        self.model = model
        self.shadow = ModelShadow(model)
        # dual-pair cold-operand prefetch (IIT_DUAL_PREFETCH=auto|0|1): auto = on for the decoder (GPT-2 headline step
        # 15.58-15.65 -> 15.43-15.49 ms) and off for the post-LN encoder, where it measured slower (MQNLI 12.14 -> 12.31 ms,
        # profiles/dual_l2_hypothesis_r6.txt)
        pol = os.environ.get("IIT_DUAL_PREFETCH", "auto")
        self.prefetch = pol == "1" or (pol == "auto" and type(model).__name__ != "HookedEncoder")
        self._layer_of = {}
        for i, blk in enumerate(model.blocks):
            self._layer_of[id(blk.attn.W_Q)] = i
            self._layer_of[id(blk.attn.W_O)] = i
            if not model.cfg.attn_only:
                self._layer_of[id(blk.mlp.W_in)] = i
                self._layer_of[id(blk.mlp.W_out)] = i

    def begin_forward(self):
        self.shadow.ensure()
        _PF_SEQ.clear()  # a new forward: the prefetch order restarts (the references of the last one are dropped)
        _PF_ON[0] = self.prefetch

    def _L(self, p):
        return self.shadow.layers[self._layer_of[id(p)]]

    # -- residual stream ------------------------------------------------------------
    def embed(self, tokens, W_E):
        return W_E[tokens]

    def pos_embed(self, batch, seq, W_pos, offset: int = 0):
        return W_pos[offset:offset + seq].unsqueeze(0).expand(batch, seq, W_pos.shape[-1])

    def embed_pos(self, tokens, W_E, W_pos):
        return EmbedPosFn.apply(tokens, W_E, W_pos)

    def residual(self, a, b):
        return a.float() + b.float()

    def w(self, p: torch.Tensor) -> torch.Tensor:
        """Small parameters used outside the fused kernels (BERT token types, pooler, classifier)."""
        return p.to(BF16)

    def layer_norm(self, x, w, b, eps):
        return LayerNormFn.apply(x, w, b, eps)

    def layer_norm_twin(self, x, w, b, eps):
        """``layer_norm`` whose bf16 output carries an fp32 twin for residual consumers (:class:`LayerNormTwinFn`;
        ``IIT_LN_TWIN=0`` disables)."""
        if os.environ.get("IIT_LN_TWIN", "1") == "0":
            return LayerNormFn.apply(x, w, b, eps)
        y, y32 = LayerNormTwinFn.apply(x, w, b, eps)
        y._iit_f32 = (y.data_ptr(), y._version, y32)
        return y

    def layer_norm_fork(self, x, w, b, eps):
        """``(LN(x), x_passthrough)``; use the passthrough for the skip connection."""
        return LayerNormForkFn.apply(x, w, b, eps)

    # -- attention -------------------------------------------------------------------
    def qkv(self, x, W_Q, W_K, W_V, b_Q, b_K, b_V):
        i = self._layer_of[id(W_Q)]
        packed = QKVFn.apply(x, self.shadow.layers[i], self.shadow.biases[i], W_Q, W_K, W_V, b_Q, b_K, b_V)
        q, k, v = packed[:, :, 0], packed[:, :, 1], packed[:, :, 2]
        q._iit_packed = k._iit_packed = v._iit_packed = packed
        return q, k, v

    def attention(self, q, k, v, causal, attn_scale, patch_heads: Optional[Sequence[int]] = None, patch_src=None,
                  hook_scores=None, hook_pattern=None, ignore=float("-inf")):
        S, dh = q.shape[1], q.shape[-1]
        if S > 16 and flash_supported(q):
            packed = getattr(q, "_iit_packed", None)
            if packed is not None and getattr(k, "_iit_packed", None) is packed and \
                    getattr(v, "_iit_packed", None) is packed and packed.is_contiguous():
                return FlashPackedFn.apply(packed, patch_src, K.heads_to_mask(patch_heads), causal, 1.0 / attn_scale)
            z = flash_attention(q, k, v, causal, attn_scale)
            if patch_heads:
                z = z.clone()
                z[:, :, list(patch_heads)] = patch_src[:, :, list(patch_heads)].to(z.dtype)
            return z
        if S > 64 or dh > 128:
            z = TorchOps.attention(self, q, k, v, causal, attn_scale)
            if patch_heads:
                z = z.clone()
                z[:, :, list(patch_heads)] = patch_src[:, :, list(patch_heads)].to(z.dtype)
            return z
        packed = getattr(q, "_iit_packed", None)
        if packed is None or getattr(k, "_iit_packed", None) is not packed or getattr(v, "_iit_packed", None) is not packed:
            packed = torch.stack([q, k, v], dim=2).to(BF16)
        mask = K.heads_to_mask(patch_heads)
        return AttnFn.apply(packed, patch_src, mask, causal, 1.0 / attn_scale)

    def o_proj(self, z, W_O, b_O):
        B, S, H, dh = z.shape
        return LinearFn.apply(z.reshape(B, S, H * dh), W_O, b_O, self._L(W_O)["o"], W_O.shape[-1], None, "bf16")

    def o_proj_residual(self, z, W_O, b_O, resid):
        resid = _f32_of(resid)
        B, S, H, dh = z.shape
        return LinearFn.apply(z.reshape(B, S, H * dh), W_O, b_O, self._L(W_O)["o"], W_O.shape[-1], resid, "resid")

    def o_result(self, z, W_O):
        return torch.einsum("bshe,hed->bshd", z.to(BF16), W_O.to(BF16))

    # -- MLP ---------------------------------------------------------------------------
    def mlp_in(self, x, W_in, b_in, act: str, hook_pre=None):
        w = self._L(W_in)["in"]
        if hook_pre is None and act in ("gelu_new", "gelu_fast", "gelu_pytorch_tanh", "gelu"):
            return MLPInFn.apply(x, W_in, b_in, w, act == "gelu")
        pre = LinearFn.apply(x, W_in, b_in, w, W_in.shape[1], None, "bf16")
        if hook_pre is not None:
            pre = hook_pre(pre)
        return pre, act_fn(act)(pre)

    def mlp_gelu_residual(self, x, W_in, b_in, W_out, b_out, resid, erf: bool = False):
        """``resid + gelu(x W_in + b_in) W_out + b_out`` (gelu_new, or the exact erf GELU) for a block whose MLP
        sites are all dead: the backward forms dpre in the dX GEMM's epilogue (see :class:`MLPOutGeluFn`).
        Without autograd (evaluation sweeps, source captures) the W_in epilogue stores only ``post``: no
        pre-activation is kept for a backward, half the epilogue's writes."""
        resid = _f32_of(resid)
        if not torch.is_grad_enabled():
            lead, d, dm, N = x.shape[:-1], x.shape[-1], W_in.shape[1], W_out.shape[1]
            x2 = _flat2(x.to(BF16).contiguous())
            T = x2.shape[0]
            post = torch.empty(T, dm, dtype=BF16, device=x.device)
            gemm(x2, self._L(W_in)["in"], post, C2=None, M=T, N=dm, K=d, lda=d, ldb=dm, ldc=dm, ldc2=dm,
                 mode=K.MODE_BKM, epi=K.EPI_GELU_ERF if erf else K.EPI_GELU, bias0=b_in)
            r2 = _flat2(resid.float().contiguous())
            out = torch.empty(T, N, dtype=F32, device=x.device)
            gemm(post, self._L(W_out)["out"], out, M=T, N=N, K=dm, lda=dm, ldb=W_out.shape[1], ldc=N,
                 mode=K.MODE_BKM, epi=K.EPI_F32_RESID, bias0=b_out, resid=r2, ldr=N)
            return out.view(*lead, N)
        pre, post = MLPInFn.apply(x, W_in, b_in, self._L(W_in)["in"], erf)
        return MLPOutGeluFn.apply(pre, post.detach(), W_out, b_out, self._L(W_out)["out"], W_out.shape[1], resid,
                                  b_in, erf)

    def mlp_out(self, post, W_out, b_out):
        return LinearFn.apply(post, W_out, b_out, self._L(W_out)["out"], W_out.shape[1], None, "bf16")

    def mlp_out_residual(self, post, W_out, b_out, resid):
        resid = _f32_of(resid)
        return LinearFn.apply(post, W_out, b_out, self._L(W_out)["out"], W_out.shape[1], resid, "resid")

    # -- unembed -------------------------------------------------------------------------
    def unembed(self, x, W_U, b_U):
        sh = self.shadow
        return LinearFn.apply(x, W_U, b_U, sh.U, sh.Vp, None, "f32")

    def unembed_argmax(self, x, W_U, b_U, chunk: int = 8192):
        sh = self.shadow
        lead = x.shape[:-1]
        d = x.shape[-1]
        x2 = _flat2(x.to(BF16).contiguous())
        T = x2.shape[0]
        V = W_U.shape[1]
        buf = torch.empty(T, chunk, dtype=F32, device=x.device)
        best_v = best_i = None
        for s in range(0, V, chunk):
            n = min(chunk, V - s)
            gemm(x2, sh.U[:, s:], buf, M=T, N=n, K=d, lda=d, ldb=sh.Vp, ldc=chunk, mode=K.MODE_BKM,
                 epi=K.EPI_F32_STORE, bias0=b_U[s:s + n])
            v, i = buf[:, :n].max(dim=-1)
            i = i + s
            if best_v is None:
                best_v, best_i = v, i
            else:
                upd = v > best_v
                best_v = torch.where(upd, v, best_v)
                best_i = torch.where(upd, i, best_i)
        return best_i.view(*lead)


    # -- paired (source + base) rows: see Paired ----------------------------------------------------------------
    supports_pairs = True

    def pair_embed_pos(self, tokens, src_tokens, W_E, W_pos) -> Paired:
        full_tok = torch.cat([tokens, src_tokens]).contiguous()
        out, full = _one(EmbedPosPairFn, tokens, W_E, W_pos, full_tok)
        return Paired(out, full)

    def pair_layer_norm_fork(self, p: Paired, w, b, eps):
        """(LN of both row sets, residual passthrough): ``(Paired normed, Paired resid)``."""
        box = []
        y, x_pass = LayerNormForkPairFn.apply(p.base, w, b, eps, p.full.float().contiguous(), box)
        return Paired(y, box[0]), Paired(x_pass, p.full)

    def pair_layer_norm(self, p: Paired, w, b, eps, pos_mask: int = 0, twin: bool = False) -> Paired:
        """LN of both row sets (no residual passthrough: post-LN blocks).  ``pos_mask``: the base rows at these
        positions take the source rows' output -- an interchange splice of whole positions of the LN output done
        by the LN kernel itself (and masked out of its backward), no separate splice pass."""
        box = []
        if twin and not pos_mask and w is not None and os.environ.get("IIT_LN_TWIN", "1") != "0":
            y, y32 = LayerNormPairTwinFn.apply(p.base, w, b, eps, p.full.float().contiguous(), box)
            yf, yf32 = box[0]
            y._iit_f32 = (y.data_ptr(), y._version, y32)  # (the unpaired blocks after the pairing ends)
            return Paired(y, yf, (y32, yf32))
        y = LayerNormPairFn.apply(p.base, w, b, eps, p.full.float().contiguous(), box, int(pos_mask))
        return Paired(y, box[0])

    @staticmethod
    def position_mask(index, shape) -> int:
        """The bit mask of positions when ``index`` selects whole positions (every batch row, every feature) of a
        ``[B, S, d]`` hook with S <= 64, else 0."""
        if len(shape) != 3 or shape[1] > 64:
            return 0
        ranges = index.to_ranges(tuple(shape))
        if ranges is None or ranges[0] != [(0, shape[0])] or ranges[2] != [(0, shape[2])]:
            return 0
        m = 0
        for lo, hi in ranges[1]:
            for s_ in range(lo, hi):
                m |= 1 << s_
        return m

    def pair_qkv(self, p: Paired, W_Q, W_K, W_V, b_Q, b_K, b_V) -> Paired:
        i = self._layer_of[id(W_Q)]
        out, full = _one(QKVPairFn, p.base, self.shadow.layers[i], self.shadow.biases[i], W_Q, W_K, W_V, b_Q, b_K,
                         b_V, p.full)
        return Paired(out, full)

    def pair_attention(self, p: Paired, causal: bool, attn_scale: float, heads: Optional[Sequence[int]] = None
                       ) -> Paired:
        """Attention over paired rows; ``heads``: the base rows of these heads take the source rows' z."""
        out, full = _one(AttnPairFn, p.base, causal, 1.0 / attn_scale, K.heads_to_mask(heads) if heads else 0,
                         p.full)
        return Paired(out, full)

    def pair_attention_spliced(self, p: Paired, causal: bool, attn_scale: float, index) -> Optional[Paired]:
        """Attention over paired rows with ``hook_z[index]`` of the base rows taken from the source rows inside the
        kernel (``AttnPairSpecFn``); None when the patch-spec table cannot express ``index``
        (``IIT_ATTN_SPLICE=0`` disables: the caller splices with a separate pass)."""
        from .splice import patch_spec
        if os.environ.get("IIT_ATTN_SPLICE", "1") == "0":
            return None
        B2, S, _, H, dh = p.full.shape
        B = p.base.shape[0]
        spec = patch_spec(index, (B, S, H, dh))
        if spec is None or [d[0] for d in spec.dims] != [B, S, H, dh]:
            return None
        out, full = _one(AttnPairSpecFn, p.base, causal, 1.0 / attn_scale, spec, p.full)
        return Paired(out, full)

    def attention_dual(self, q, causal: bool, attn_scale: float) -> torch.Tensor:
        """No-grad attention of the packed qkv behind ``q`` (``qkv`` output) into BOTH halves of a [2B, S, H, dh]
        tensor: the z of a whole-layer ``hook_z`` splice, whose base rows are the source rows."""
        packed = q._iit_packed
        B, S, _, H, dh = packed.shape
        zf = torch.empty(2 * B, S, H, dh, dtype=BF16, device=packed.device)
        K.attn_pair_fwd(packed, zf[B:], None, B, S, H, dh, 3 * H * dh, H * dh, 1.0 / attn_scale, causal, z2=zf[:B])
        return zf

    def pair_heads_ok(self, S: int, dh: int) -> bool:
        return K.attn_pair_ok(S, dh)

    def pair_o_proj_residual(self, z: Paired, W_O, b_O, resid: Paired) -> Paired:
        B2, S, H, dh = z.full.shape
        B = z.base.shape[0]
        rb, rf = resid.resid_operands()
        out, full = _one(LinearPairFn, z.base.reshape(B, S, H * dh), W_O, b_O, self._L(W_O)["o"], W_O.shape[-1],
                         rb, "resid", z.full.reshape(B2, S, H * dh), rf)
        return Paired(out, full)

    def pair_mlp_in(self, x: Paired, W_in, b_in, erf: bool = False, index=None):
        """Paired W_in + gelu.  ``index`` (optional): an ``mlp.hook_post`` splice applied inside the op
        (``MLPInPairFn``); returns None when the patch-spec table cannot express it (``IIT_MLP_SPLICE=0``
        disables) -- the caller then splices with a separate pass."""
        spec = None
        if index is not None:
            from .splice import patch_spec
            B, S = x.base.shape[0], x.base.shape[1]
            spec = patch_spec(index, (B, S, W_in.shape[1])) if os.environ.get("IIT_MLP_SPLICE", "1") != "0" else None
            if spec is None:
                return None
        (pre, post), (pf, qf) = _one(MLPInPairFn, x.base, W_in, b_in, self._L(W_in)["in"], erf, x.full, spec)
        return Paired(pre, pf), Paired(post, qf)

    def pair_mlp_out_residual(self, post: Paired, W_out, b_out, resid: Paired) -> Paired:
        rb, rf = resid.resid_operands()
        out, full = _one(LinearPairFn, post.base, W_out, b_out, self._L(W_out)["out"], W_out.shape[1], rb,
                         "resid", post.full, rf)
        return Paired(out, full)

    def pair_mlp_gelu_residual(self, x: Paired, W_in, b_in, W_out, b_out, resid: Paired, erf: bool = False):
        pre, post = self.pair_mlp_in(x, W_in, b_in, erf)
        rb, rf = resid.resid_operands()
        out, full = _one(MLPOutGeluPairFn, pre.base, post.base.detach(), W_out, b_out, self._L(W_out)["out"],
                         W_out.shape[1], rb, b_in, erf, post.full, rf)
        return Paired(out, full)

    def pair_splice(self, p: Paired, index) -> Optional[Paired]:
        """Base rows take the source rows' values at ``index`` (None when the range table cannot express it)."""
        if not p.full.is_contiguous():
            return None
        specs = pair_specs(index, tuple(p.base.shape))
        if specs is None:
            return None
        out, full = _one(PairSpliceFn, p.base, p.full, specs[0], specs[1])
        return Paired(out, full)


def pair_specs(index, shape):
    """(paired spec, base spec) of ``index`` on a hook of base shape ``shape`` whose paired activation is the
    contiguous [2B, ...] tensor: the paired spec selects ``index`` inside rows [0, B) and reads the source from rows
    [B, 2B) at the same positions (a whole-batch index merges the (base | source) axis into the batch axis: rows
    [0, B) of 2B), or None when the kernel's 4-dimensional range table cannot express it."""
    from . import splice as _sp
    key = ("pair",) + tuple(shape)
    cache = getattr(index, "_iit_specs", None)
    if cache is not None and key in cache:
        return cache[key]
    ranges = index.to_ranges(tuple(shape))
    base_spec = _sp.patch_spec(index, tuple(shape))
    out = None
    if ranges is not None and base_spec is not None:
        B = shape[0]
        rest = list(shape[1:])
        row = 1
        for n in rest:
            row *= n
        cstr = []  # contiguous strides of the trailing dims
        acc = 1
        for n in reversed(rest):
            cstr.insert(0, acc)
            acc *= n
        if ranges[0] == [(0, B)]:
            dims = _sp._collapse((2 * B,) + tuple(rest), [[(0, B)]] + ranges[1:], [row] + cstr)
        else:
            dims = _sp._collapse((2, B) + tuple(rest), [[(0, 1)]] + ranges, [0, row] + cstr)
        if dims is not None:
            out = (_sp.PatchSpec(dims), base_spec)
    if cache is None:
        cache = index._iit_specs = {}
    cache[key] = out
    return out


def get_hip_ops(model) -> HipOps:
    K.lib()  # strict: fail loudly if the kernel library is unavailable
    ops = getattr(model, "_iit_hip_ops", None)
    if ops is None:
        ops = HipOps(model)
        model._iit_hip_ops = ops
    return ops
