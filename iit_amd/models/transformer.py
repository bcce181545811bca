"""TransformerLens-compatible hooked transformer, built natively for MI355X.

Replaces the reference's external ``transformer_lens.HookedTransformer``
(SURVEY.md §2.1 X1, §2.6): identical hook names and shapes, parameter names and
layouts (``W_Q [H,d,dh]``, ``W_O [H,dh,d]``, ``W_in [d,d_mlp]``...), named-parameter
order, ``mask``/``IGNORE`` buffers, GPT-2 init and ``cfg.to_dict()`` keys, so
checkpoints written by ``torch.save(model.state_dict())`` load in both.

Execution is plan-driven instead of closure-driven:

* every hook site calls ``_Run.site`` which applies the active ``RunPlan``
  (capture / splice / StopGrad scale) and then the user ``HookPoint``;
* hook sites nobody listens to are never materialised when the fused HIP op
  backend is active (``iit_amd.ops.hip_ops``): LN, QKV, attention, MLP and the
  residual adds run as fused kernels, and splices of ``attn.hook_z`` (whole or
  per head) / ``mlp.hook_post`` happen *inside* those kernels (or skip the dead
  producer entirely for whole-tensor splices);
* a capture-only plan stops the forward right after its last captured hook;
* ``logits_at=-1`` (or a plan with ``logits="last"``) computes the unembed only
  for the last position (all IOI losses only read ``[:, -1]``).

Parameters are always fp32 masters; ``cfg.dtype`` selects the compute dtype
(fp32 = reference parity mode, bf16 = MI355X fast mode).
"""
from __future__ import annotations

import math
import os
from typing import List, Optional, Union

import torch
from torch import nn

from ..engine.plan import RunPlan, Splice, scale_site as _scale_site, zero_grad_site as _zero_grad_site
from ..hooks.hook_points import HookedRootModule, HookPoint
from ..ops import select_ops
from ..ops.torch_ops import TorchOps
from .config import HookedTransformerConfig, make_config


def _hip_ops():
    from ..ops import hip_ops
    return hip_ops


def _flash_ok(q: torch.Tensor) -> bool:
    return q.is_cuda and q.dtype == torch.bfloat16 and _hip_ops().flash_supported(q)


class _StopForward(Exception):
    pass


class _Run:
    """Per-forward execution state: the plan plus the active op backend."""

    __slots__ = ("plan", "ops", "remaining")

    def __init__(self, plan: Optional[RunPlan], ops):
        self.plan = plan
        self.ops = ops
        self.remaining = None
        if plan is not None and plan.logits == "none" and plan.truncate and plan.capture:
            self.remaining = set(plan.capture)

    def live(self, hp: HookPoint) -> bool:
        return hp.is_live or (self.plan is not None and self.plan.touches(hp.name))

    def whole_splice(self, name: str):
        if self.plan is None:
            return None
        spl = self.plan.splice.get(name)
        if spl and len(spl) == 1 and spl[0].whole:
            return spl[0]
        return None

    def site(self, hp: HookPoint, x: torch.Tensor, spliced: bool = False) -> torch.Tensor:
        plan = self.plan
        name = hp.name
        if plan is not None:
            if not spliced and name in plan.splice:
                for s in plan.splice[name]:
                    x = s.apply(x)
            if name in plan.scale:
                x = _scale_site(x, plan.scale[name])
            if name in plan.zero_grad and isinstance(x, torch.Tensor) and x.requires_grad:
                x = _zero_grad_site(x, plan.zero_grad[name])
        x = hp(x)
        if plan is not None and name in plan.capture:
            plan.cache[name] = x.detach()
            if self.remaining is not None:
                self.remaining.discard(name)
                if not self.remaining:
                    raise _StopForward()
        return x


# ---------------------------------------------------------------------------- modules
class Embed(nn.Module):
    def __init__(self, cfg: HookedTransformerConfig):
        super().__init__()
        self.W_E = nn.Parameter(torch.empty(cfg.d_vocab, cfg.d_model))


class PosEmbed(nn.Module):
    def __init__(self, cfg: HookedTransformerConfig):
        super().__init__()
        self.W_pos = nn.Parameter(torch.empty(cfg.n_ctx, cfg.d_model))


class Unembed(nn.Module):
    def __init__(self, cfg: HookedTransformerConfig):
        super().__init__()
        self.W_U = nn.Parameter(torch.empty(cfg.d_model, cfg.d_vocab_out))
        self.b_U = nn.Parameter(torch.zeros(cfg.d_vocab_out))


class LayerNormSite(nn.Module):
    """``LN`` (affine) / ``LNPre`` (no params) or ``RMS`` (weight only) / ``RMSPre`` with TL hook names."""

    def __init__(self, cfg: HookedTransformerConfig, affine: bool, rms: bool = False):
        super().__init__()
        self.eps = cfg.eps
        self.rms = rms
        self.w = nn.Parameter(torch.ones(cfg.d_model)) if affine else None
        self.b = nn.Parameter(torch.zeros(cfg.d_model)) if (affine and not rms) else None
        self.hook_scale = HookPoint()
        self.hook_normalized = HookPoint()

    @staticmethod
    def make(cfg: HookedTransformerConfig, kind: Optional[str]) -> Optional["LayerNormSite"]:
        if kind is None:
            return None
        if kind not in ("LN", "LNPre", "RMS", "RMSPre"):
            raise NotImplementedError(f"normalization_type {kind}")
        return LayerNormSite(cfg, affine=kind in ("LN", "RMS"), rms=kind in ("RMS", "RMSPre"))

    def run(self, x, run: _Run, twin: bool = False):
        """``twin``: the output will also be a residual operand (post-norm blocks): the fused backend then returns
        it with an fp32 twin (``HipOps.layer_norm_twin``)."""
        live = run.live(self.hook_scale) or run.live(self.hook_normalized)
        if self.rms:
            hs = (lambda t: run.site(self.hook_scale, t)) if live else None
            hn = (lambda t: run.site(self.hook_normalized, t)) if live else None
            return TorchOps.rms_norm(run.ops, x, self.w, self.eps, hook_scale=hs, hook_normalized=hn)
        if live or not run.ops.fused:
            return TorchOps.layer_norm(
                run.ops, x, self.w, self.b, self.eps,
                hook_scale=lambda t: run.site(self.hook_scale, t),
                hook_normalized=lambda t: run.site(self.hook_normalized, t),
            )
        if twin and self.w is not None and hasattr(run.ops, "layer_norm_twin"):
            return run.ops.layer_norm_twin(x, self.w, self.b, self.eps)
        return run.ops.layer_norm(x, self.w, self.b, self.eps)


def rotary_tables(cfg: HookedTransformerConfig):
    """TL rotary sin/cos ``[n_ctx, rotary_dim]`` (angles repeated per pair layout)."""
    rd = cfg.rotary_dim or cfg.d_head
    pos = torch.arange(cfg.n_ctx, dtype=torch.float64)
    freq = cfg.rotary_base ** (-torch.arange(0, rd, 2, dtype=torch.float64) / rd)
    ang = pos[:, None] * freq[None, :]
    ang = ang.repeat_interleave(2, dim=-1) if cfg.rotary_adjacent_pairs else torch.cat([ang, ang], dim=-1)
    return ang.sin().float(), ang.cos().float()


class Attention(nn.Module):
    def __init__(self, cfg: HookedTransformerConfig, layer: int):
        super().__init__()
        H, d, dh = cfg.n_heads, cfg.d_model, cfg.d_head
        self.cfg = cfg
        self.layer = layer
        n_kv = cfg.n_key_value_heads or H
        self.n_kv = n_kv
        self.gqa = n_kv != H  # grouped-query attention (TL ``_W_K`` / ``_W_V`` naming)
        self.W_Q = nn.Parameter(torch.empty(H, d, dh))
        if self.gqa:
            if H % n_kv:
                raise ValueError("n_heads must be a multiple of n_key_value_heads")
            self._W_K = nn.Parameter(torch.empty(n_kv, d, dh))
            self._W_V = nn.Parameter(torch.empty(n_kv, d, dh))
        else:
            self.W_K = nn.Parameter(torch.empty(H, d, dh))
            self.W_V = nn.Parameter(torch.empty(H, d, dh))
        self.W_O = nn.Parameter(torch.empty(H, dh, d))
        self.b_Q = nn.Parameter(torch.zeros(H, dh))
        if self.gqa:
            self._b_K = nn.Parameter(torch.zeros(n_kv, dh))
            self._b_V = nn.Parameter(torch.zeros(n_kv, dh))
        else:
            self.b_K = nn.Parameter(torch.zeros(H, dh))
            self.b_V = nn.Parameter(torch.zeros(H, dh))
        self.b_O = nn.Parameter(torch.zeros(d))
        self.rotary = cfg.positional_embedding_type == "rotary"
        if self.rotary:
            self.rotary_dim = cfg.rotary_dim or dh
            sin, cos = rotary_tables(cfg)
            self.register_buffer("rotary_sin", sin)
            self.register_buffer("rotary_cos", cos)
            self.hook_rot_q = HookPoint()
            self.hook_rot_k = HookPoint()
        causal = torch.tril(torch.ones(cfg.n_ctx, cfg.n_ctx, dtype=torch.bool))
        self.register_buffer("mask", causal)
        self.register_buffer("IGNORE", torch.tensor(float("-inf")))
        self.attn_scale = math.sqrt(dh) if cfg.use_attn_scale else 1.0
        if cfg.scale_attn_by_inverse_layer_idx:
            self.attn_scale *= layer + 1
        self.hook_k = HookPoint()
        self.hook_q = HookPoint()
        self.hook_v = HookPoint()
        self.hook_z = HookPoint()
        self.hook_attn_scores = HookPoint()
        self.hook_pattern = HookPoint()
        self.hook_result = HookPoint()

    # grouped-query attention: TL exposes the expanded per-query-head views
    def _kv(self, name: str):
        p = self._parameters.get(name)
        if p is not None:
            return p
        kv = self._parameters.get("_" + name)
        if kv is None:  # (during registration) -> AttributeError keeps hasattr() honest
            raise AttributeError(name)
        return kv.repeat_interleave(self.cfg.n_heads // self.n_kv, dim=0)

    W_K = property(lambda self: self._kv("W_K"))
    W_V = property(lambda self: self._kv("W_V"))
    b_K = property(lambda self: self._kv("b_K"))
    b_V = property(lambda self: self._kv("b_V"))

    def kv_params(self):
        """(W_K, W_V, b_K, b_V) as stored (kv heads for GQA)."""
        if self.gqa:
            return self._W_K, self._W_V, self._b_K, self._b_V
        return self.W_K, self.W_V, self.b_K, self.b_V

    def inner_live(self, run: _Run) -> bool:
        return any(run.live(h) for h in (self.hook_q, self.hook_k, self.hook_v, self.hook_attn_scores,
                                         self.hook_pattern))

    def compute_z(self, x, run: _Run):
        ops = run.ops
        Wk, Wv, bk, bv = self.kv_params()
        q, k, v = ops.qkv(x, self.W_Q, Wk, Wv, self.b_Q, bk, bv)
        q = run.site(self.hook_q, q)
        k = run.site(self.hook_k, k)
        v = run.site(self.hook_v, v)
        if self.rotary:
            q = run.site(self.hook_rot_q, TorchOps.rotary(ops, q, self.rotary_cos, self.rotary_sin, self.rotary_dim,
                                                          self.cfg.rotary_adjacent_pairs))
            k = run.site(self.hook_rot_k, TorchOps.rotary(ops, k, self.rotary_cos, self.rotary_sin, self.rotary_dim,
                                                          self.cfg.rotary_adjacent_pairs))
        causal = self.cfg.attention_dir == "causal"
        if not ops.fused and q.shape[1] > 16 and _flash_ok(q) and \
                not (run.live(self.hook_attn_scores) or run.live(self.hook_pattern)):
            # torch op backend on the GPU (Llama family): tiled MFMA attention, GQA-native (no k/v expansion); a
            # single interchange splice of hook_z is applied by the kernel's output store (no splice pass; the
            # site's scale / gradient mask / hook still run after it, as after SpliceFn)
            z_spl = run.plan.splice.get(self.hook_z.name) if run.plan is not None else None
            if z_spl and len(z_spl) == 1 and not z_spl[0].whole:
                z = _hip_ops().flash_attention_spliced(q, k, v, causal, self.attn_scale, z_spl[0].index,
                                                       z_spl[0].src)
                if z is not None:
                    return z, True
            return _hip_ops().flash_attention(q, k, v, causal, self.attn_scale), False
        if self.gqa:
            rep = self.cfg.n_heads // self.n_kv
            k = k.repeat_interleave(rep, dim=2)
            v = v.repeat_interleave(rep, dim=2)
        z_spl = run.plan.splice.get(self.hook_z.name) if run.plan is not None else None
        if ops.fused and not (run.live(self.hook_attn_scores) or run.live(self.hook_pattern)):
            heads = z_spl[0].head_mask(self.cfg.n_heads) if (z_spl and len(z_spl) == 1) else None
            if heads is not None:
                z = ops.attention(q, k, v, causal, self.attn_scale, patch_heads=heads, patch_src=z_spl[0].src)
                return z, True
            return ops.attention(q, k, v, causal, self.attn_scale), False
        z = TorchOps.attention(
            ops, q, k, v, causal, self.attn_scale,
            hook_scores=lambda t: run.site(self.hook_attn_scores, t),
            hook_pattern=lambda t: run.site(self.hook_pattern, t),
            ignore=self.ignore_value(),
        )
        return z, False

    def ignore_value(self) -> float:
        """The masked-score fill (the ``IGNORE`` buffer) as a host float, read once: a device read inside a
        graph-captured phase is a synchronising copy, which capture forbids.  ``load_state_dict`` re-reads it."""
        v = self.__dict__.get("_ignore_f")
        if v is None:
            v = self.__dict__["_ignore_f"] = float(self.IGNORE)
        return v

    def _load_from_state_dict(self, *args, **kwargs):
        self.__dict__.pop("_ignore_f", None)
        return super()._load_from_state_dict(*args, **kwargs)


class MLP(nn.Module):
    def __init__(self, cfg: HookedTransformerConfig):
        super().__init__()
        self.cfg = cfg
        self.gated = cfg.gated_mlp
        self.W_in = nn.Parameter(torch.empty(cfg.d_model, cfg.d_mlp))
        if self.gated:  # TL GatedMLP (SwiGLU with act_fn="silu")
            self.W_gate = nn.Parameter(torch.empty(cfg.d_model, cfg.d_mlp))
        self.b_in = nn.Parameter(torch.zeros(cfg.d_mlp))
        self.W_out = nn.Parameter(torch.empty(cfg.d_mlp, cfg.d_model))
        self.b_out = nn.Parameter(torch.zeros(cfg.d_model))
        self.hook_pre = HookPoint()
        if self.gated:
            self.hook_pre_linear = HookPoint()
        self.hook_post = HookPoint()


class TransformerBlock(nn.Module):
    def __init__(self, cfg: HookedTransformerConfig, layer: int):
        super().__init__()
        self.cfg = cfg
        self.layer = layer
        self.ln1 = LayerNormSite.make(cfg, cfg.normalization_type)
        if not cfg.attn_only:
            self.ln2 = LayerNormSite.make(cfg, cfg.normalization_type)
        self.attn = Attention(cfg, layer)
        if not cfg.attn_only:
            self.mlp = MLP(cfg)
        self.hook_attn_in = HookPoint()
        self.hook_q_input = HookPoint()
        self.hook_k_input = HookPoint()
        self.hook_v_input = HookPoint()
        self.hook_mlp_in = HookPoint()
        self.hook_attn_out = HookPoint()
        self.hook_mlp_out = HookPoint()
        self.hook_resid_pre = HookPoint()
        if not cfg.attn_only:
            self.hook_resid_mid = HookPoint()
        self.hook_resid_post = HookPoint()

    def _norm(self, ln, x, run):
        if ln is None:
            return x.to(run.ops.dtype)
        return ln.run(x, run)

    def _norm_fork(self, ln, x, run):
        """(normed x, residual to carry forward): fused backends return a passthrough of ``x`` whose
        gradient the LN (or RMSNorm) backward kernel adds in (one pass instead of norm-bwd + autograd's sum)."""
        if ln is None or run.live(ln.hook_scale) or run.live(ln.hook_normalized) or not x.requires_grad:
            return self._norm(ln, x, run), x
        if ln.rms:
            fork = getattr(run.ops, "rms_norm_fork", None)
            out = fork(x, ln.w, ln.eps) if fork is not None else None
            return out if out is not None else (self._norm(ln, x, run), x)
        fork = getattr(run.ops, "layer_norm_fork", None)
        if fork is None:
            return self._norm(ln, x, run), x
        return fork(x, ln.w, ln.b, ln.eps)

    def last_position_ok(self, run: _Run) -> bool:
        """Whether this (final) block may compute only the last position after attention: nothing observes
        or rewrites a later site of the block at other positions (the logits read position -1 only)."""
        if self.cfg.use_attn_result:
            return False
        sites = [self.hook_attn_out, self.hook_resid_post, self.hook_mlp_out]
        if not self.cfg.attn_only:
            sites += [self.hook_resid_mid, self.hook_mlp_in, self.mlp.hook_pre, self.mlp.hook_post]
            if self.mlp.gated:
                sites.append(self.mlp.hook_pre_linear)
            if self.ln2 is not None:
                sites += [self.ln2.hook_scale, self.ln2.hook_normalized]
        return not any(run.live(h) for h in sites)

    def forward(self, resid: torch.Tensor, run: _Run, last_only: bool = False) -> torch.Tensor:
        """``last_only``: after attention (which still sees every position's keys / values) continue with the
        last position only -- ``[B, 1, d]`` out.  Exact for a loss that reads the last position's logits: the
        other positions of the final block's W_O / LN2 / MLP never reach it (their gradients are zero)."""
        ops = run.ops
        attn = self.attn
        resid = run.site(self.hook_resid_pre, resid)

        # ---- attention -----------------------------------------------------------
        spl = run.whole_splice(attn.hook_z.name)
        ln1_live = self.ln1 is not None and (run.live(self.ln1.hook_scale) or run.live(self.ln1.hook_normalized))
        if spl is not None and not attn.inner_live(run) and not ln1_live:
            z = run.site(attn.hook_z, spl.src.to(ops.dtype), spliced=True)
        else:
            x, resid = self._norm_fork(self.ln1, resid, run)
            z, spliced = attn.compute_z(x, run)
            z = run.site(attn.hook_z, z, spliced=spliced)
        if last_only:
            z, resid = z[:, -1:].contiguous(), resid[:, -1:].contiguous()
        attn_out_live = run.live(self.hook_attn_out) or self.cfg.use_attn_result
        if self.cfg.use_attn_result:
            result = run.site(attn.hook_result, ops.o_result(z, attn.W_O))
            attn_out = result.sum(-2) + ops.w(attn.b_O)
            attn_out = run.site(self.hook_attn_out, attn_out)
            resid_mid_pre = ops.residual(resid, attn_out)
        elif attn_out_live or not (ops.fused or getattr(ops, "fuses_residual", False)):
            attn_out = run.site(self.hook_attn_out, ops.o_proj(z, attn.W_O, attn.b_O))
            resid_mid_pre = ops.residual(resid, attn_out)
        else:
            resid_mid_pre = ops.o_proj_residual(z, attn.W_O, attn.b_O, resid)

        if self.cfg.attn_only:
            return run.site(self.hook_resid_post, resid_mid_pre)
        resid_mid = run.site(self.hook_resid_mid, resid_mid_pre)

        # ---- MLP -----------------------------------------------------------------
        mlp = self.mlp
        spl = run.whole_splice(mlp.hook_post.name)
        ln2_live = self.ln2 is not None and (run.live(self.ln2.hook_scale) or run.live(self.ln2.hook_normalized))
        pre_lin_live = mlp.gated and run.live(mlp.hook_pre_linear)
        if spl is not None and not run.live(mlp.hook_pre) and not ln2_live and not pre_lin_live:
            post = run.site(mlp.hook_post, spl.src.to(ops.dtype), spliced=True)
        elif (not mlp.gated and getattr(ops, "mlp_gelu_residual", None) is not None
              and self.cfg.act_fn in ("gelu_new", "gelu_fast", "gelu_pytorch_tanh")
              and not (ln2_live or run.live(mlp.hook_pre) or run.live(mlp.hook_post) or run.live(self.hook_mlp_out))):
            # no MLP site observed: one fused op whose backward forms dpre in the dX GEMM epilogue
            x, resid_mid = self._norm_fork(self.ln2, resid_mid, run)
            resid_post = ops.mlp_gelu_residual(x, mlp.W_in, mlp.b_in, mlp.W_out, mlp.b_out, resid_mid)
            return run.site(self.hook_resid_post, resid_post)
        else:
            x, resid_mid = self._norm_fork(self.ln2, resid_mid, run)
            pre_hook = (lambda t: run.site(mlp.hook_pre, t)) if run.live(mlp.hook_pre) else None
            spliced = False
            if mlp.gated:
                lin_hook = (lambda t: run.site(mlp.hook_pre_linear, t)) if run.live(mlp.hook_pre_linear) else None
                pspl = run.plan.splice.get(mlp.hook_post.name) if run.plan is not None else None
                if pspl and len(pspl) == 1 and not pspl[0].whole and pre_hook is None and lin_hook is None:
                    # the hook_post splice inside the SwiGLU kernel (the producer), not a separate pass
                    _, post, spliced = TorchOps.mlp_gated_in(ops, x, mlp.W_gate, mlp.W_in, mlp.b_in,
                                                             self.cfg.act_fn, splice=pspl[0])
                else:
                    _, post = TorchOps.mlp_gated_in(ops, x, mlp.W_gate, mlp.W_in, mlp.b_in, self.cfg.act_fn,
                                                    hook_pre=pre_hook, hook_pre_linear=lin_hook)
            else:
                _, post = ops.mlp_in(x, mlp.W_in, mlp.b_in, self.cfg.act_fn, hook_pre=pre_hook)
            post = run.site(mlp.hook_post, post, spliced=spliced)
        if run.live(self.hook_mlp_out) or not (ops.fused or getattr(ops, "fuses_residual", False)):
            mlp_out = run.site(self.hook_mlp_out, ops.mlp_out(post, mlp.W_out, mlp.b_out))
            resid_post = ops.residual(resid_mid, mlp_out)
        else:
            resid_post = ops.mlp_out_residual(post, mlp.W_out, mlp.b_out, resid_mid)
        return run.site(self.hook_resid_post, resid_post)


    # ------------------------------------------------------------------ paired source + base rows
    def paired_ok(self, run: _Run) -> bool:
        """Whether this block can run as part of a paired forward (the fused HIP path, no live hook inside)."""
        cfg = self.cfg
        if cfg.use_attn_result or self.attn.rotary or self.attn.gqa:
            return False
        if self.ln1 is None or self.ln1.rms or (not cfg.attn_only and (self.ln2 is None or self.ln2.rms)):
            return False
        if not cfg.attn_only and (self.mlp.gated or cfg.act_fn not in ("gelu_new", "gelu_fast", "gelu_pytorch_tanh")):
            return False
        return True

    def forward_paired(self, p, run: _Run, sites, stop_after: str, captures, last_only: bool = False):
        """One block over paired rows (``ops.hip_ops.Paired``: base rows with autograd, source rows without).

        ``sites``: hook name -> list of TorchIndex spliced from source into base (only ``attn.hook_z`` and
        ``mlp.hook_post`` occur); their source values go to ``captures``.  When the block holds ``stop_after`` (the
        deepest site) the pairing ends right after it and the rest of the block runs on the base rows only.
        Returns ``(resid, still_paired)``."""
        ops = run.ops
        attn = self.attn
        zname = attn.hook_z.name
        zs = sites.get(zname)
        causal = self.cfg.attention_dir == "causal"
        S, H, dh = p.full.shape[1], self.cfg.n_heads, self.cfg.d_head
        mirror = ops.pair_heads_ok(S, dh) and H <= 64
        if zs is not None and any(ix.is_everything() for ix in zs):
            # the base z is the source z: the base attention is dead, compute the source rows only
            with torch.no_grad():
                x = ops.layer_norm(p.src, self.ln1.w, self.ln1.b, self.ln1.eps)
                q, k, v = ops.qkv(x, attn.W_Q, attn.W_K, attn.W_V, attn.b_Q, attn.b_K, attn.b_V)
                if mirror:  # stored into both halves by the attention kernel itself
                    zf = ops.attention_dual(q, causal, attn.attn_scale)
                else:
                    z_src = ops.attention(q, k, v, causal, attn.attn_scale)
                    zf = torch.cat([z_src, z_src])
            z = _hip_ops().Paired(zf[:p.nb], zf)
            resid = p
        else:
            x, resid = ops.pair_layer_norm_fork(p, self.ln1.w, self.ln1.b, self.ln1.eps)
            qkv = ops.pair_qkv(x, attn.W_Q, attn.W_K, attn.W_V, attn.b_Q, attn.b_K, attn.b_V)
            heads, rest = None, list(zs or ())
            z = None
            if mirror and len(rest) == 1:
                heads = Splice(rest[0], None).head_mask(H)
                if heads is not None:
                    rest = []  # head splice inside the attention kernel
                else:  # any other patch-spec index (positions, features, ...) in the kernel's z store
                    z = ops.pair_attention_spliced(qkv, causal, attn.attn_scale, rest[0])
                    if z is not None:
                        rest = []
            if z is None:
                z = ops.pair_attention(qkv, causal, attn.attn_scale, heads=heads)
            for ix in rest:
                z = ops.pair_splice(z, ix)
        if zs is not None:
            captures[zname] = z.src
        if zname == stop_after:
            return self._finish_after_attn(z.base, resid.base, run, last_only), False
        resid_mid = ops.pair_o_proj_residual(z, attn.W_O, attn.b_O, resid)
        if self.cfg.attn_only:
            return resid_mid, True
        mlp = self.mlp
        pname = mlp.hook_post.name
        ps = sites.get(pname)
        erf = False  # gelu_new family only (paired_ok)
        if ps is None:
            x, resid2 = ops.pair_layer_norm_fork(resid_mid, self.ln2.w, self.ln2.b, self.ln2.eps)
            return ops.pair_mlp_gelu_residual(x, mlp.W_in, mlp.b_in, mlp.W_out, mlp.b_out, resid2, erf=erf), True
        if any(ix.is_everything() for ix in ps):
            with torch.no_grad():
                x = ops.layer_norm(resid_mid.src, self.ln2.w, self.ln2.b, self.ln2.eps)
                _, post_src = ops.mlp_in(x, mlp.W_in, mlp.b_in, self.cfg.act_fn)
            qf = torch.cat([post_src, post_src])
            post = _hip_ops().Paired(qf[:post_src.shape[0]], qf)
            resid2 = resid_mid
        else:
            x, resid2 = ops.pair_layer_norm_fork(resid_mid, self.ln2.w, self.ln2.b, self.ln2.eps)
            done = ops.pair_mlp_in(x, mlp.W_in, mlp.b_in, erf=erf, index=ps[0]) if len(ps) == 1 else None
            if done is not None:  # the splice inside the producing op (sparse copy + masked dpre)
                _, post = done
            else:
                _, post = ops.pair_mlp_in(x, mlp.W_in, mlp.b_in, erf=erf)
                for ix in ps:
                    post = ops.pair_splice(post, ix)
        captures[pname] = post.src
        if pname == stop_after:
            return ops.mlp_out_residual(post.base, mlp.W_out, mlp.b_out, resid2.base), False
        return ops.pair_mlp_out_residual(post, mlp.W_out, mlp.b_out, resid2), True

    # ------------------------------------------------------------------ paired rows, torch op backend (Llama family)
    def paired_torch_ok(self, ops) -> bool:
        """Whether this block can run in a paired forward on the torch op backend (``ops.torch_pairs``): bf16 on the
        GPU, RMSNorm, (rotary / GQA) flash attention, SiLU-gated MLP, no attention-result hook."""
        cfg = self.cfg
        if getattr(ops, "fused", True) or ops.dtype != torch.bfloat16 or cfg.use_attn_result:
            return False
        if self.ln1 is None or not self.ln1.rms or self.ln1.w is None or cfg.d_head not in (64, 128):
            return False
        if cfg.d_model % 8 or (not cfg.attn_only and cfg.d_mlp % 8) or not _hip_ops().flash_supported(
                self.attn.W_Q):
            return False
        if not cfg.attn_only and (self.ln2 is None or not self.ln2.rms or self.ln2.w is None or not self.mlp.gated
                                  or cfg.act_fn != "silu"):
            return False
        return True

    def forward_paired_torch(self, p, run: _Run, sites, stop_after: str, captures):
        """:meth:`forward_paired` for the torch op backend (RMSNorm / rotary / GQA flash attention / SwiGLU) with the
        paired Functions of :mod:`iit_amd.ops.torch_pairs`; sites ``attn.hook_z`` / ``mlp.hook_post``.  Returns
        ``(resid, still_paired)``, or None when an arena layout the paired ops need does not hold (the caller then
        drops the partial paired run -- nothing was accumulated -- and falls back to two forwards)."""
        from ..ops import torch_pairs as tp
        ops = run.ops
        attn = self.attn
        zname = attn.hook_z.name
        zs = sites.get(zname)
        x = tp.pair_rms(p, self.ln1.w, self.ln1.eps)
        Wk, Wv, bk, bv = attn.kv_params()
        qkv = tp.pair_qkv(x, attn.W_Q, Wk, Wv, attn.b_Q, bk, bv)
        if qkv is None:
            return None
        q, k, v = qkv
        if attn.rotary:
            q = tp.pair_rotary(q, attn.rotary_cos, attn.rotary_sin, attn.rotary_dim, self.cfg.rotary_adjacent_pairs)
            k = tp.pair_rotary(k, attn.rotary_cos, attn.rotary_sin, attn.rotary_dim, self.cfg.rotary_adjacent_pairs)
        z = tp.pair_flash(q, k, v, self.cfg.attention_dir == "causal", attn.attn_scale)
        for ix in zs or ():
            z = tp.pair_splice(z, ix)
        if zs is not None:
            captures[zname] = z.src
        if zname == stop_after:
            return self._finish_after_attn_torch(z.base, p.base, run), False
        attn_out = tp.pair_o_proj(z, attn.W_O, attn.b_O)
        if attn_out is None:
            return None
        resid_mid = tp.pair_add(p, attn_out)
        if self.cfg.attn_only:
            return resid_mid, True
        mlp = self.mlp
        x = tp.pair_rms(resid_mid, self.ln2.w, self.ln2.eps)
        gate = tp.pair_linear(x, mlp.W_gate)
        up = tp.pair_linear(x, mlp.W_in, mlp.b_in)
        if gate is None or up is None:
            return None
        post = tp.pair_swiglu(gate, up)
        pname = mlp.hook_post.name
        ps = sites.get(pname)
        for ix in ps or ():
            post = tp.pair_splice(post, ix)
        if ps is not None:
            captures[pname] = post.src
        if pname == stop_after:
            return ops.residual(resid_mid.base, ops.mlp_out(post.base, mlp.W_out, mlp.b_out)), False
        out = tp.pair_linear(post, mlp.W_out, mlp.b_out)
        if out is None:
            return None
        return tp.pair_add(resid_mid, out), True

    def _finish_after_attn_torch(self, z, resid, run: _Run):
        """The rest of a (torch-backend) block on base rows, after a paired attention section."""
        ops = run.ops
        attn = self.attn
        resid_mid = ops.residual(resid, ops.o_proj(z, attn.W_O, attn.b_O))
        if self.cfg.attn_only:
            return resid_mid
        mlp = self.mlp
        x = self.ln2.run(resid_mid, run)
        _, post = TorchOps.mlp_gated_in(ops, x, mlp.W_gate, mlp.W_in, mlp.b_in, self.cfg.act_fn)
        return ops.residual(resid_mid, ops.mlp_out(post, mlp.W_out, mlp.b_out))

    def _finish_after_attn(self, z, resid, run: _Run, last_only: bool):
        """The rest of the block (O projection + MLP) on base rows, after a paired attention section."""
        ops = run.ops
        attn = self.attn
        if last_only:
            z, resid = z[:, -1:].contiguous(), resid[:, -1:].contiguous()
        resid_mid = ops.o_proj_residual(z, attn.W_O, attn.b_O, resid)
        if self.cfg.attn_only:
            return resid_mid
        mlp = self.mlp
        x, resid_mid = self._norm_fork(self.ln2, resid_mid, run)
        return ops.mlp_gelu_residual(x, mlp.W_in, mlp.b_in, mlp.W_out, mlp.b_out, resid_mid)


def qkv_arena_groups(blocks, cfg):
    """Arena groups packing each block's ``W_Q|W_K|W_V`` into one ``[d_model][(H + 2*H_kv)*d_head]`` matrix
    (query heads, then key heads, then value heads; column ``head*dh + e``) and ``b_Q|b_K|b_V`` into
    ``[H + 2*H_kv][dh]`` (see ``HookedTransformer._iit_arena_groups``).  Without grouped-query heads this is the
    ``[d][3][H][dh]`` layout the HIP backend's fused QKV GEMM reads; with them (Llama: ``_W_K`` / ``_W_V`` hold
    the ``H_kv`` heads) the torch backend's packed projection (``TorchOps.qkv``) runs one GEMM per block."""
    H, d, dh = cfg.n_heads, cfg.d_model, cfg.d_head
    groups = []
    for blk in blocks:
        a = blk.attn
        Hkv = a.n_kv
        Wq = a.W_Q
        Wk, Wv = (a._W_K, a._W_V) if a.gqa else (a.W_K, a.W_V)
        bq = a.b_Q
        bk, bv = (a._b_K, a._b_V) if a.gqa else (a.b_K, a.b_V)
        if Wq.shape != (H, d, dh) or Wk.shape != (Hkv, d, dh) or Wv.shape != (Hkv, d, dh):
            continue
        Ht = H + 2 * Hkv

        def w_view(c0, n):
            return lambda buf: buf.view(d, Ht, dh)[:, c0:c0 + n].permute(1, 0, 2)

        def b_view(c0, n):
            return lambda buf: buf.view(Ht, dh)[c0:c0 + n]

        spans = ((0, H), (H, Hkv), (H + Hkv, Hkv))
        groups.append((d * Ht * dh, [(w, w_view(*sp)) for w, sp in zip((Wq, Wk, Wv), spans)]))
        groups.append((Ht * dh, [(b, b_view(*sp)) for b, sp in zip((bq, bk, bv), spans)]))
    return groups


class HookedTransformer(HookedRootModule):
    def __init__(self, cfg: Union[HookedTransformerConfig, dict], tokenizer=None, move_to_device: bool = True,
                 default_padding_side: str = "right"):
        super().__init__()
        self.cfg = make_config(cfg)
        cfg = self.cfg
        self.tokenizer = tokenizer
        self.embed = Embed(cfg)
        self.hook_embed = HookPoint()
        self.rotary = cfg.positional_embedding_type == "rotary"
        if cfg.positional_embedding_type not in ("standard", "rotary"):
            raise NotImplementedError(f"positional_embedding_type {cfg.positional_embedding_type}")
        if not self.rotary:
            self.pos_embed = PosEmbed(cfg)
            self.hook_pos_embed = HookPoint()
        self.blocks = nn.ModuleList([TransformerBlock(cfg, l) for l in range(cfg.n_layers)])
        final = cfg.normalization_type
        if cfg.final_rms and final in ("LN", "LNPre"):
            final = "RMS" if final == "LN" else "RMSPre"
        self.ln_final = LayerNormSite.make(cfg, final)
        self.unembed = Unembed(cfg)
        self.op_backend: Optional[str] = None  # None = auto (see iit_amd.ops.select_ops)
        if cfg.init_weights:
            self.init_weights()
        if move_to_device and cfg.device is not None:
            self.to(cfg.device)
        self.setup()

    # ------------------------------------------------------------------ init
    def init_weights(self) -> None:
        """GPT-2 init (TL ``_init_weights_gpt2``): N(0, initializer_range) for every ``W_*``."""
        for name, p in self.named_parameters():
            if "W_" in name:
                nn.init.normal_(p, std=self.cfg.initializer_range)

    def load_state_dict(self, state_dict, strict: bool = True, assign: bool = False):
        res = super().load_state_dict(state_dict, strict=strict, assign=assign)
        self.mark_weights_changed()
        return res

    def mark_weights_changed(self) -> None:
        """Invalidate derived bf16 compute copies after an out-of-band weight update."""
        self._iit_weights_version = getattr(self, "_iit_weights_version", 0) + 1

    def _iit_arena_groups(self):
        """GEMM-operand layout of the flat parameter arena (see :mod:`iit_amd.engine.flat`).

        * per block, ``W_Q|W_K|W_V`` interleave into one ``[d_model][3*H*d_head]``
          matrix (column ``which*H*dh + h*dh + e``) and ``b_Q|b_K|b_V`` into ``[3][H][dh]``:
          the fused QKV projection, its input gradient and its weight gradient are
          then single plain GEMMs on the arena (or its bf16 mirror) with no
          repacking pass;
        * ``W_U`` gets rows padded to a multiple of 8 columns (16-byte aligned
          k-major B operand for the unembed GEMM).
        Parameters keep their TL shapes; only their strides differ from contiguous.
        """
        cfg = self.cfg
        d = cfg.d_model
        groups = qkv_arena_groups(self.blocks, cfg)
        V = cfg.d_vocab_out
        Vp = (V + 7) // 8 * 8
        if Vp != V:
            groups.append((d * Vp, [(self.unembed.W_U, lambda buf: buf.view(d, Vp)[:, :V])]))
        return groups

    # ------------------------------------------------------------------ backend
    def set_op_backend(self, backend: Optional[str]) -> "HookedTransformer":
        self.op_backend = backend
        return self

    def ops(self):
        return select_ops(self, self.op_backend)

    # ------------------------------------------------------------------ forward
    def _embed(self, tokens: torch.Tensor, run: _Run) -> torch.Tensor:
        ops = run.ops
        B, S = tokens.shape
        if self.rotary:  # positions enter through the rotary q/k rotation
            spl = run.plan.splice.get(self.hook_embed.name) if run.plan is not None else None
            e = None
            if spl and len(spl) == 1 and not spl[0].whole and hasattr(ops, "embed_spliced"):
                # a single interchange splice of hook_embed applied by the gather itself (no splice pass; the
                # site's scale / gradient mask / hook still run after it)
                e = ops.embed_spliced(tokens, self.embed.W_E, spl[0].index, spl[0].src)
            e = run.site(self.hook_embed, e, spliced=True) if e is not None else \
                run.site(self.hook_embed, ops.embed(tokens, self.embed.W_E))
            return e.to(torch.float32 if ops.fused else ops.dtype)
        if ops.fused and not (run.live(self.hook_embed) or run.live(self.hook_pos_embed)):
            return ops.embed_pos(tokens, self.embed.W_E, self.pos_embed.W_pos)
        e = run.site(self.hook_embed, ops.embed(tokens, self.embed.W_E))
        p = run.site(self.hook_pos_embed, ops.pos_embed(B, S, self.pos_embed.W_pos))
        return ops.residual(e, p)

    def forward(self, input, return_type: Optional[str] = "logits", loss_per_token: bool = False,
                prepend_bos: Optional[bool] = None, stop_at_layer: Optional[int] = None,
                past_kv_cache=None, *, plan: Optional[RunPlan] = None, logits_at: Optional[int] = None,
                start_at_layer: Optional[int] = None):
        """TL semantics; ``start_at_layer`` (TL's keyword): ``input`` is the residual stream entering that block
        ([B, S, d]) and the embedding and earlier blocks are skipped (evaluation sweeps resume a cached base run
        at each spliced node's layer, :func:`iit_amd.utils.eval_ablations._resample_scores`)."""
        if start_at_layer is not None:
            tokens = input
        else:
            tokens = self.to_tokens(input, prepend_bos=prepend_bos) if isinstance(input, (str, list)) else input
            if tokens.dim() == 1:
                tokens = tokens.unsqueeze(0)
            if tokens.device != self.embed.W_E.device:
                tokens = tokens.to(self.embed.W_E.device)
        run = _Run(plan, self.ops())
        begin = getattr(run.ops, "begin_forward", None)
        if begin is not None:
            begin()
        gate = self.__dict__.get("_param_gate")  # ZeRO-1 deferred all-gather (parallel/zero.py attach_gates)
        try:
            if gate is not None:
                gate(None)
            first = 0 if start_at_layer is None else int(start_at_layer)
            resid = self._embed(tokens, run) if start_at_layer is None else input
            n_blocks = len(self.blocks) if stop_at_layer is None else stop_at_layer
            cuts = self.__dict__.get("_grad_cuts") if torch.is_grad_enabled() else None
            want = plan.logits if plan is not None else ("last" if logits_at == -1 else "full")
            # last-position logits: the final block continues past attention at position -1 only
            last_only = (want == "last" and stop_at_layer is None and return_type is not None
                         and len(self.blocks) > 0 and getattr(self, "last_position_final_block", True)
                         and tokens.shape[1] > 1 and self.blocks[-1].last_position_ok(run))
            for li, block in enumerate(self.blocks[:n_blocks]):
                if li < first:
                    continue
                if cuts and li in cuts and resid.requires_grad:
                    # staged backward (engine.graphs): the backward stops here and resumes as its own segment
                    leaf = resid.detach().requires_grad_(True)
                    self._cut_log.append((li, resid, leaf))
                    resid = leaf
                if gate is not None:
                    gate(li)
                resid = block(resid, run, last_only=last_only and li == len(self.blocks) - 1)
            if stop_at_layer is not None:
                return resid
            if plan is not None and plan.logits == "none":
                return None
            if return_type is None:
                return None
            if want == "last":
                resid = resid[:, -1]  # [B, d]: only the position every IOI loss reads
            x = resid if self.ln_final is None else self.ln_final.run(resid, run)
            if want == "argmax":
                return run.ops.unembed_argmax(x, self.unembed.W_U, self.unembed.b_U)
            logits = run.ops.unembed(x, self.unembed.W_U, self.unembed.b_U)
            if return_type == "logits":
                return logits
            loss = lm_cross_entropy_loss(logits.float(), tokens, per_token=loss_per_token)
            if return_type == "loss":
                return loss
            if return_type == "both":
                return logits, loss
            raise ValueError(f"invalid return_type {return_type}")
        except _StopForward:
            return None

    # ------------------------------------------------------------------ helpers
    supports_run_plan = True
    # forward / run_paired call ``_param_gate(None)`` before the first weight read and ``_param_gate(li)`` before
    # block li (ZeRO-1's all-gather overlapped with the forward, iit_amd/parallel/zero.py)
    supports_param_gate = True

    def run_capture(self, tokens: torch.Tensor, names, truncate: bool = True, base_plan: Optional[RunPlan] = None):
        """Source run of an interchange intervention: no grad, capture ``names`` only, stop early."""
        plan = RunPlan.capture_only(list(names), truncate=truncate)
        if base_plan is not None:
            plan = base_plan.merged(plan)
        with torch.no_grad():
            self.forward(tokens, plan=plan)
        return plan.cache

    def run_paired(self, tokens: torch.Tensor, src_tokens: torch.Tensor, sites, logits: str = "full"):
        """Interchange intervention with the source run folded into the base forward.

        ``sites``: ``{hook name: [TorchIndex, ...]}`` spliced from the source run into the base run, as
        ``ll_source_cache`` + ``ll_intervened_forward`` do with two forwards
        (/root/reference/iit/model_pairs/base_model_pair.py:80-98).  Up to the deepest site both runs go through
        every kernel as one batch of 2B rows (``ops.hip_ops.Paired``): the source rows carry no autograd state (the
        reference's source run is under no_grad) and the base rows are exactly the unpaired intervened forward's.
        Returns ``(output, {site: source activation})``, or None when the configuration is not covered (fused HIP
        backend, S <= 64 (short-sequence attention kernels), LN models, sites on ``attn.hook_z`` / ``mlp.hook_post``, no live user
        hook) -- the caller then runs the two forwards.  ``IIT_PAIRED=0`` disables it."""
        import os
        if os.environ.get("IIT_PAIRED", "1") == "0" or not sites:
            return None
        ops = self.ops()
        cfg = self.cfg
        if self._torch_pairs_ok(ops, tokens, src_tokens):
            return self._run_paired_torch(tokens, src_tokens, sites, logits)
        if not getattr(ops, "supports_pairs", False) or self.rotary or cfg.final_rms:
            return None
        # S <= 16: the MFMA attention kernel (in-kernel head mirroring); 16 < S <= 64: the short-sequence kernel,
        # head splices then go through the paired patch-spec splice
        if tokens.dim() != 2 or tokens.shape != src_tokens.shape or tokens.shape[1] > 64 or tokens.shape[1] < 1:
            return None
        if any(hp.is_live for hp in self.hook_dict.values()):
            return None
        B, S = tokens.shape
        order = []
        for name, idxs in sites.items():
            parts = name.split(".")
            if len(parts) != 4 or parts[0] != "blocks" or (parts[2], parts[3]) not in (("attn", "hook_z"),
                                                                                        ("mlp", "hook_post")):
                return None
            li = int(parts[1])
            if parts[2] == "mlp" and cfg.attn_only:
                return None
            shape = (B, S, cfg.n_heads, cfg.d_head) if parts[2] == "attn" else (B, S, cfg.d_mlp)
            for ix in idxs:
                if not ix.is_everything() and _hip_ops().pair_specs(ix, shape) is None:
                    return None
            order.append((li, 0 if parts[2] == "attn" else 1, name))
        deepest = max(order)
        if not all(blk.paired_ok(None) for blk in self.blocks[:deepest[0] + 1]):
            return None
        tokens = tokens.to(self.embed.W_E.device)
        src_tokens = src_tokens.to(self.embed.W_E.device)
        run = _Run(RunPlan(logits=logits), ops)
        gate = self.__dict__.get("_param_gate")
        if gate is not None:
            gate(None)
        ops.begin_forward()
        n = len(self.blocks)
        final_mlp_site = not cfg.attn_only and self.blocks[-1].mlp.hook_post.name in sites
        last_only = (logits == "last" and n > 0 and S > 1 and getattr(self, "last_position_final_block", True)
                     and self.blocks[-1].last_position_ok(run) and not final_mlp_site)
        captures = {}
        resid = ops.pair_embed_pos(tokens, src_tokens, self.embed.W_E, self.pos_embed.W_pos)
        paired = True
        cuts = self.__dict__.get("_grad_cuts") if torch.is_grad_enabled() else None
        for li, block in enumerate(self.blocks):
            lo = last_only and li == n - 1
            base = resid.base if paired else resid
            if cuts and li in cuts and base.requires_grad:
                # staged backward (engine.staged): the backward stops here and resumes as its own segment; the
                # source rows carry no autograd state, so only the base rows are cut
                leaf = base.detach().requires_grad_(True)
                self._cut_log.append((li, base, leaf))
                resid = _hip_ops().Paired(leaf, resid.full) if paired else leaf
            if gate is not None:
                gate(li)
            if paired:
                resid, paired = block.forward_paired(resid, run, sites, deepest[2], captures, last_only=lo)
            else:
                resid = block(resid, run, last_only=lo)
        if paired:  # (cannot happen: the deepest site ends the pairing) -- keep the base rows
            resid = resid.base
        if logits == "none":
            return None, captures
        if logits == "last":
            resid = resid[:, -1]
        x = resid if self.ln_final is None else self.ln_final.run(resid, run)
        if logits == "argmax":
            return ops.unembed_argmax(x, self.unembed.W_U, self.unembed.b_U), captures
        return ops.unembed(x, self.unembed.W_U, self.unembed.b_U), captures

    def _torch_pairs_ok(self, ops, tokens, src_tokens) -> bool:
        """The torch-backend paired forward applies: bf16 torch ops on the GPU, the Llama block family
        (:meth:`TransformerBlock.paired_torch_ok`), flash-attention sequence lengths, no live user hook."""
        if getattr(ops, "fused", True) or ops.dtype != torch.bfloat16 or not self.embed.W_E.is_cuda:
            return False
        # opt-in (IIT_PAIRED_TORCH=1): at Llama-3-8B / S = 512 every projection is already an 8192-row GEMM and the
        # paired forward measured 0.9-3.5 % slower than the two forwards, with ~10 GB more peak memory
        # (profiles/llama3_8b_paired_r6.txt)
        if self.cfg.positional_embedding_type != "rotary" or os.environ.get("IIT_PAIRED_TORCH", "0") != "1":
            return False
        if tokens.dim() != 2 or tokens.shape != src_tokens.shape or tokens.shape[1] <= 16:
            return False
        if any(hp.is_live for hp in self.hook_dict.values()):
            return False
        return all(blk.paired_torch_ok(ops) for blk in self.blocks)

    def _run_paired_torch(self, tokens, src_tokens, sites, logits: str):
        """:meth:`run_paired` on the torch op backend (Llama family, ``ops.torch_pairs``): sites ``hook_embed``,
        ``blocks.L.attn.hook_z`` and ``blocks.L.mlp.hook_post``; the pairing ends after the deepest site."""
        from ..ops import torch_pairs as tp
        cfg = self.cfg
        B, S = tokens.shape
        order = []
        for name, idxs in sites.items():
            parts = name.split(".")
            if name == "hook_embed":
                order.append((-1, 0, name))
                shape = (B, S, cfg.d_model)
            elif len(parts) == 4 and parts[0] == "blocks" and (parts[2], parts[3]) in (("attn", "hook_z"),
                                                                                          ("mlp", "hook_post")):
                if parts[2] == "mlp" and cfg.attn_only:
                    return None
                order.append((int(parts[1]), 0 if parts[2] == "attn" else 1, name))
                shape = (B, S, cfg.n_heads, cfg.d_head) if parts[2] == "attn" else (B, S, cfg.d_mlp)
            else:
                return None
            for ix in idxs:
                if not ix.is_everything() and _hip_ops().pair_specs(ix, shape) is None:
                    return None
        deepest = max(order)
        tokens = tokens.to(self.embed.W_E.device)
        src_tokens = src_tokens.to(self.embed.W_E.device)
        ops = self.ops()
        run = _Run(RunPlan(logits=logits), ops)
        gate = self.__dict__.get("_param_gate")
        if gate is not None:
            gate(None)
        begin = getattr(ops, "begin_forward", None)
        if begin is not None:
            begin()
        captures = {}
        resid = tp.pair_embed(tokens, src_tokens, self.embed.W_E)
        if resid is None:
            return None
        for ix in sites.get("hook_embed", ()):
            resid = tp.pair_splice(resid, ix)
            if resid is None:
                return None
        if "hook_embed" in sites:
            captures["hook_embed"] = resid.src
        paired = deepest[2] != "hook_embed"
        if not paired:
            resid = resid.base
        cuts = self.__dict__.get("_grad_cuts") if torch.is_grad_enabled() else None
        for li, block in enumerate(self.blocks):
            base = resid.base if paired else resid
            if cuts and li in cuts and base.requires_grad:
                leaf = base.detach().requires_grad_(True)
                self._cut_log.append((li, base, leaf))
                resid = _hip_ops().Paired(leaf, resid.full) if paired else leaf
            if gate is not None:
                gate(li)
            if paired:
                res = block.forward_paired_torch(resid, run, sites, deepest[2], captures)
                if res is None:
                    return None
                resid, paired = res
            else:
                resid = block(resid, run)
        if paired:
            resid = resid.base
        if logits == "none":
            return None, captures
        if logits == "last":
            resid = resid[:, -1]
        x = resid if self.ln_final is None else self.ln_final.run(resid, run)
        if logits == "argmax":
            return ops.unembed_argmax(x, self.unembed.W_U, self.unembed.b_U), captures
        return ops.unembed(x, self.unembed.W_U, self.unembed.b_U), captures

    def to_tokens(self, input, prepend_bos: Optional[bool] = None):
        if self.tokenizer is None:
            raise ValueError("to_tokens requires a tokenizer")
        bos = self.cfg.default_prepend_bos if prepend_bos is None else prepend_bos
        texts = [input] if isinstance(input, str) else list(input)
        rows = [([self.tokenizer.bos_token_id] if bos else []) + self.tokenizer.encode(t) for t in texts]
        width = max(len(r) for r in rows)
        pad = self.tokenizer.pad_token_id if self.tokenizer.pad_token_id is not None else 0
        rows = [r + [pad] * (width - len(r)) for r in rows]
        return torch.tensor(rows, dtype=torch.long, device=self.embed.W_E.device)

    @property
    def W_E(self):
        return self.embed.W_E

    @property
    def W_U(self):
        return self.unembed.W_U

    @property
    def W_pos(self):
        if self.rotary:
            raise AttributeError("rotary models have no W_pos")
        return self.pos_embed.W_pos


def lm_cross_entropy_loss(logits: torch.Tensor, tokens: torch.Tensor, per_token: bool = False):
    logp = torch.log_softmax(logits, dim=-1)
    picked = logp[:, :-1].gather(-1, tokens[:, 1:, None])[..., 0]
    return -picked if per_token else -picked.mean()
