"""BERT-style hooked encoder (the MQNLI LL model of ``BASELINE.json`` config 4).

TransformerLens ``HookedEncoder`` names and layouts (``embed.embed.W_E``,
``embed.pos_embed.W_pos``, ``embed.token_type_embed.W_token_type``, ``embed.ln``,
``blocks.L.attn.W_Q [H, d, dh]`` ..., post-LN blocks with ``ln1`` after attention and
``ln2`` after the MLP, ``mlm_head`` + ``unembed``), plus an optional sequence-
classification head on the first ([CLS]) position with HF BERT semantics
(``pooler.W``/``pooler.b`` dense + tanh, ``classifier.W``/``classifier.b``) -- the
head MQNLI's 3-way entailment label is read from.

Every hook site goes through the same plan executor as the decoder
(:class:`iit_amd.models.transformer._Run`), so the native intervention engine
(capture-only truncated source runs, splices, StopGrad scaling) works unchanged.
Compute goes through :func:`iit_amd.ops.select_ops`: on an MI355X in bf16 the HIP backend
(packed-QKV GEMM into the flat arena's bf16 mirror, fused small-S attention with the
in-kernel head splice, W_O / W_out GEMMs with the residual add in the epilogue, affine
LayerNorm kernels); anywhere else the fp32 :class:`~iit_amd.ops.torch_ops.TorchOps` oracle.
A key-padding ``attention_mask`` or a live attention-internal hook takes the
TorchOps-semantics path for that block.

``from_hf_bert`` converts an in-memory HF ``BertForSequenceClassification`` /
``BertForMaskedLM`` / ``BertModel`` (random-init or local weights; nothing is
downloaded).
"""
from __future__ import annotations

import math
from typing import Dict, Optional, Union

import torch
import torch.nn.functional as F
from torch import nn

from ..engine.plan import RunPlan
from ..hooks.hook_points import HookedRootModule, HookPoint
from ..ops import select_ops
from .config import HookedTransformerConfig, make_config
from .transformer import MLP, Attention, LayerNormSite, _Run, _StopForward, qkv_arena_groups


def bert_config_dict(size: str = "bert-base", **overrides):
    presets = {
        "bert-base": dict(n_layers=12, d_model=768, n_heads=12, d_head=64, d_mlp=3072, d_vocab=30522, n_ctx=512),
        "bert-tiny": dict(n_layers=2, d_model=64, n_heads=4, d_head=16, d_mlp=128, d_vocab=128, n_ctx=64),
    }
    cfg = dict(presets[size])
    cfg.update(act_fn="gelu", normalization_type="LN", attention_dir="bidirectional", eps=1e-12,
               original_architecture="BertForMaskedLM", model_name=size, initializer_range=0.02)
    cfg.update(overrides)
    return HookedTransformerConfig.from_dict(cfg).to_dict()


class BertEmbed(nn.Module):
    def __init__(self, cfg: HookedTransformerConfig, n_token_types: int = 2):
        super().__init__()
        self.embed = nn.Module()
        self.embed.W_E = nn.Parameter(torch.empty(cfg.d_vocab, cfg.d_model))
        self.pos_embed = nn.Module()
        self.pos_embed.W_pos = nn.Parameter(torch.empty(cfg.n_ctx, cfg.d_model))
        self.token_type_embed = nn.Module()
        self.token_type_embed.W_token_type = nn.Parameter(torch.empty(n_token_types, cfg.d_model))
        self.ln = LayerNormSite(cfg, affine=True)
        self.hook_embed = HookPoint()
        self.hook_pos_embed = HookPoint()
        self.hook_token_type_embed = HookPoint()


class BertBlock(nn.Module):
    """Post-LN encoder block: ``x = ln1(x + attn(x)); x = ln2(x + mlp(x))``."""

    def __init__(self, cfg: HookedTransformerConfig, layer: int):
        super().__init__()
        self.cfg = cfg
        self.attn = Attention(cfg, layer)
        self.ln1 = LayerNormSite(cfg, affine=True)
        self.mlp = MLP(cfg)
        self.ln2 = LayerNormSite(cfg, affine=True)
        self.hook_attn_out = HookPoint()
        self.hook_mlp_in = HookPoint()
        self.hook_mlp_out = HookPoint()
        self.hook_resid_pre = HookPoint()
        self.hook_resid_mid = HookPoint()
        self.hook_resid_post = HookPoint()
        self.hook_normalized_resid_post = HookPoint()

    def _fused_ok(self, run: _Run, key_mask) -> bool:
        attn = self.attn
        return (run.ops.fused and key_mask is None and not any(
            run.live(h) for h in (self.hook_attn_out, attn.hook_attn_scores, attn.hook_pattern, attn.hook_q,
                                  attn.hook_k, attn.hook_v, self.hook_mlp_out)))

    def forward(self, resid, run: _Run, key_mask: Optional[torch.Tensor]):
        ops, attn = run.ops, self.attn
        resid = run.site(self.hook_resid_pre, resid)
        if self._fused_ok(run, key_mask):
            # HIP path: packed-QKV GEMM -> fused attention (in-kernel head splice) -> W_O GEMM with the fp32
            # residual add in its epilogue -> LN -> W_in GEMM -> W_out GEMM + residual -> LN
            z, spliced = attn.compute_z(resid, run)
            z = run.site(attn.hook_z, z, spliced=spliced)
            resid_mid = run.site(self.hook_resid_mid, ops.o_proj_residual(z, attn.W_O, attn.b_O, resid))
            # (post-norm: both LN outputs are also residual operands -- fp32 twins, LayerNormTwinFn)
            x = run.site(self.hook_mlp_in, self.ln1.run(resid_mid, run, twin=True))
            mlp = self.mlp
            if (getattr(ops, "mlp_gelu_residual", None) is not None and self.cfg.act_fn in ("gelu", "gelu_new")
                    and not (run.live(mlp.hook_pre) or run.live(mlp.hook_post))):
                # no MLP site observed: dpre formed in the backward's dX GEMM epilogue (HipOps.mlp_gelu_residual)
                resid_post = ops.mlp_gelu_residual(x, mlp.W_in, mlp.b_in, mlp.W_out, mlp.b_out, x,
                                                   erf=self.cfg.act_fn == "gelu")
                resid_post = run.site(self.hook_resid_post, resid_post)
                return run.site(self.hook_normalized_resid_post, self.ln2.run(resid_post, run, twin=True))
            pre_hook = (lambda t: run.site(self.mlp.hook_pre, t)) if run.live(self.mlp.hook_pre) else None
            _, post = ops.mlp_in(x, self.mlp.W_in, self.mlp.b_in, self.cfg.act_fn, hook_pre=pre_hook)
            post = run.site(self.mlp.hook_post, post)
            resid_post = run.site(self.hook_resid_post, ops.mlp_out_residual(post, self.mlp.W_out, self.mlp.b_out, x))
            return run.site(self.hook_normalized_resid_post, self.ln2.run(resid_post, run, twin=True))
        q, k, v = ops.qkv(resid, attn.W_Q, attn.W_K, attn.W_V, attn.b_Q, attn.b_K, attn.b_V)
        q, k, v = run.site(attn.hook_q, q), run.site(attn.hook_k, k), run.site(attn.hook_v, v)
        scores = torch.einsum("bqhe,bkhe->bhqk", q, k) / attn.attn_scale
        if key_mask is not None:
            scores = scores.masked_fill(~key_mask[:, None, None, :], float("-inf"))
        scores = run.site(attn.hook_attn_scores, scores)
        pattern = run.site(attn.hook_pattern, torch.softmax(scores.float(), dim=-1).to(scores.dtype))
        z = run.site(attn.hook_z, torch.einsum("bkhe,bhqk->bqhe", v, pattern))
        attn_out = run.site(self.hook_attn_out, ops.o_proj(z, attn.W_O, attn.b_O))
        resid_mid = run.site(self.hook_resid_mid, resid + attn_out)
        x = self.ln1.run(resid_mid, run)
        x = run.site(self.hook_mlp_in, x)
        pre_hook = (lambda t: run.site(self.mlp.hook_pre, t)) if run.live(self.mlp.hook_pre) else None
        _, post = ops.mlp_in(x, self.mlp.W_in, self.mlp.b_in, self.cfg.act_fn, hook_pre=pre_hook)
        post = run.site(self.mlp.hook_post, post)
        mlp_out = run.site(self.hook_mlp_out, ops.mlp_out(post, self.mlp.W_out, self.mlp.b_out))
        resid_post = run.site(self.hook_resid_post, x + mlp_out)
        return run.site(self.hook_normalized_resid_post, self.ln2.run(resid_post, run))


    # ------------------------------------------------------------------ paired source + base rows
    def paired_ok(self) -> bool:
        a = self.attn
        return not (a.rotary or a.gqa or self.cfg.use_attn_result) and self.cfg.act_fn in ("gelu", "gelu_new")

    def forward_paired(self, p, run: _Run, sites, stop_after: str, captures):
        """The fused block over paired rows (``ops.hip_ops.Paired``: base rows with autograd, source rows without),
        as :meth:`iit_amd.models.transformer.TransformerBlock.forward_paired` does for the decoder.  Sites:
        ``attn.hook_z`` (whole / heads in the attention kernel, other indices by the paired patch-spec splice),
        ``mlp.hook_post`` and ``hook_normalized_resid_post`` (the paired splice); their source values go to
        ``captures``.  Pairing ends after ``stop_after`` (the rest of the block runs on the base rows).  Returns
        ``(x, still_paired)``."""
        from .transformer import _hip_ops
        from ..engine.plan import Splice
        ops, attn, mlp = run.ops, self.attn, self.mlp
        S, H, dh = p.full.shape[1], self.cfg.n_heads, self.cfg.d_head
        erf = self.cfg.act_fn == "gelu"
        zname = attn.hook_z.name
        zs = sites.get(zname)
        qkv = ops.pair_qkv(p, attn.W_Q, attn.W_K, attn.W_V, attn.b_Q, attn.b_K, attn.b_V)
        heads, rest = None, list(zs or ())
        if ops.pair_heads_ok(S, dh) and H <= 64 and len(rest) == 1:
            heads = Splice(rest[0], None).head_mask(H)
            if heads is not None:
                rest = []
        z = ops.pair_attention(qkv, False, attn.attn_scale, heads=heads)
        for ix in rest:
            z = ops.pair_splice(z, ix)
        if zs is not None:
            captures[zname] = z.src
        if zname == stop_after:
            resid_mid = ops.o_proj_residual(z.base, attn.W_O, attn.b_O, p.base)
            x = self.ln1.run(resid_mid, run)
            resid_post = ops.mlp_gelu_residual(x, mlp.W_in, mlp.b_in, mlp.W_out, mlp.b_out, x, erf=erf)
            return self.ln2.run(resid_post, run), False
        resid_mid = ops.pair_o_proj_residual(z, attn.W_O, attn.b_O, p)
        x = ops.pair_layer_norm(resid_mid, self.ln1.w, self.ln1.b, self.ln1.eps, twin=True)
        pname = mlp.hook_post.name
        ps = sites.get(pname)
        if ps is None:
            resid_post = ops.pair_mlp_gelu_residual(x, mlp.W_in, mlp.b_in, mlp.W_out, mlp.b_out, x, erf=erf)
        else:
            _, post = ops.pair_mlp_in(x, mlp.W_in, mlp.b_in, erf=erf)
            for ix in ps:
                post = ops.pair_splice(post, ix)
            captures[pname] = post.src
            if pname == stop_after:
                resid_post = ops.mlp_out_residual(post.base, mlp.W_out, mlp.b_out, x.base)
                return self.ln2.run(resid_post, run), False
            resid_post = ops.pair_mlp_out_residual(post, mlp.W_out, mlp.b_out, x)
        nname = self.hook_normalized_resid_post.name
        idxs = list(sites.get(nname, ()))
        shape = tuple(p.base.shape[:2]) + (self.cfg.d_model,)
        masks = [ops.position_mask(ix, shape) for ix in idxs]
        mask = 0
        if idxs and all(masks):  # whole positions: spliced inside the LN kernel (no splice pass, fwd or bwd)
            for m in masks:
                mask |= m
            idxs = []
        out = ops.pair_layer_norm(resid_post, self.ln2.w, self.ln2.b, self.ln2.eps, pos_mask=mask, twin=True)
        for ix in idxs:
            out = ops.pair_splice(out, ix)
        if nname in sites:
            captures[nname] = out.src
            if nname == stop_after:
                return out.base, False
        return out, True


_BERT_PAIRED_DEFAULT = "1"  # validated on MI355X in round 4 (tests/test_hip_model.py, MQNLI 12,296 -> 20,032 pairs/s with the embedding fixes)


class HookedEncoder(HookedRootModule):
    """BERT encoder; ``n_classes`` adds the [CLS] pooler + classifier head (forward then returns ``[B, C]``)."""

    supports_run_plan = True

    def __init__(self, cfg: Union[HookedTransformerConfig, dict], n_classes: Optional[int] = None,
                 move_to_device: bool = True):
        super().__init__()
        self.cfg = make_config(cfg)
        cfg = self.cfg
        self.embed = BertEmbed(cfg)
        self.hook_full_embed = HookPoint()
        self.blocks = nn.ModuleList([BertBlock(cfg, l) for l in range(cfg.n_layers)])
        self.n_classes = n_classes
        self.op_backend: Optional[str] = None  # None = auto (iit_amd.ops.select_ops: HIP on a GPU in bf16)
        self.sep_token_id: Optional[int] = None  # set -> token types derived from [SEP] when not given
        if n_classes:
            self.pooler = nn.Module()
            self.pooler.W = nn.Parameter(torch.empty(cfg.d_model, cfg.d_model))
            self.pooler.b = nn.Parameter(torch.zeros(cfg.d_model))
            self.classifier = nn.Module()
            self.classifier.W = nn.Parameter(torch.empty(cfg.d_model, n_classes))
            self.classifier.b = nn.Parameter(torch.zeros(n_classes))
            self.hook_pooled = HookPoint()
        else:
            self.mlm_head = nn.Module()
            self.mlm_head.W = nn.Parameter(torch.empty(cfg.d_model, cfg.d_model))
            self.mlm_head.b = nn.Parameter(torch.zeros(cfg.d_model))
            self.mlm_head.ln = LayerNormSite(cfg, affine=True)
            self.unembed = nn.Module()
            self.unembed.W_U = nn.Parameter(torch.empty(cfg.d_model, cfg.d_vocab_out))
            self.unembed.b_U = nn.Parameter(torch.zeros(cfg.d_vocab_out))
        for name, p in self.named_parameters():
            if name.endswith((".W_E", ".W_pos", ".W_token_type")) or ".W_" in name or name.endswith(".W"):
                nn.init.normal_(p, std=cfg.initializer_range)
        if move_to_device and cfg.device is not None:
            self.to(cfg.device)
        self.setup()

    def mark_weights_changed(self) -> None:
        self._iit_weights_version = getattr(self, "_iit_weights_version", 0) + 1

    def _iit_arena_groups(self):
        """Packed-QKV arena layout, as for the decoder (``transformer.qkv_arena_groups``)."""
        return qkv_arena_groups(self.blocks, self.cfg)

    def set_op_backend(self, backend: Optional[str]) -> "HookedEncoder":
        self.op_backend = backend
        return self

    def ops(self):
        return select_ops(self, self.op_backend)

    def forward(self, input, token_type_ids: Optional[torch.Tensor] = None,
                attention_mask: Optional[torch.Tensor] = None, *, plan: Optional[RunPlan] = None,
                return_type: Optional[str] = "logits"):
        tokens = input
        if tokens.dim() == 1:
            tokens = tokens.unsqueeze(0)
        dev = self.embed.embed.W_E.device
        tokens = tokens.to(dev)
        run = _Run(plan, self.ops())
        ops = run.ops
        begin = getattr(ops, "begin_forward", None)
        if begin is not None:
            begin()
        B, S = tokens.shape
        if token_type_ids is None:
            sep = getattr(self, "sep_token_id", None)
            if sep is None:
                token_type_ids = torch.zeros_like(tokens)
            else:  # segment B starts after the first [SEP] (BERT sentence-pair convention)
                is_sep = (tokens == sep).long()
                token_type_ids = ((is_sep.cumsum(-1) - is_sep) > 0).long()
        key_mask = None if attention_mask is None else attention_mask.to(dev).bool()
        try:
            t = run.site(self.embed.hook_token_type_embed, self._token_type_embed(ops, token_type_ids))
            x = self.embed.ln.run(self._embed_pos(tokens, run) + t, run)
            x = run.site(self.hook_full_embed, x)
            for blk in self.blocks:
                x = blk(x, run, key_mask)
            if plan is not None and plan.logits == "none" or return_type is None:
                return None
            if self.n_classes:
                pooled = torch.tanh(x[:, 0] @ ops.w(self.pooler.W) + ops.w(self.pooler.b))
                pooled = run.site(self.hook_pooled, pooled)
                return pooled @ ops.w(self.classifier.W) + ops.w(self.classifier.b)
            h = F.gelu(x @ ops.w(self.mlm_head.W) + ops.w(self.mlm_head.b))
            h = self.mlm_head.ln.run(h, run)
            return h @ ops.w(self.unembed.W_U) + ops.w(self.unembed.b_U)
        except _StopForward:
            return None

    _PAIR_SITES = ("attn.hook_z", "mlp.hook_post", "hook_normalized_resid_post")

    def _token_types(self, tokens):
        sep = getattr(self, "sep_token_id", None)
        if sep is None:
            return torch.zeros_like(tokens)
        is_sep = (tokens == sep).long()
        return ((is_sep.cumsum(-1) - is_sep) > 0).long()

    def _token_type_embed(self, ops, types: torch.Tensor) -> torch.Tensor:
        """Rows of the (2-row) token-type table per position.  As a one-hot GEMM against the fp32 table rather than a
        gather: the gather's backward (an index_put accumulating B*S rows into 2) ran 3.0 ms per phase on MI355X
        (profiles/mqnli_step_breakdown_r4.txt); this backward is one [n x B*S] x [B*S x d] product."""
        W = self.embed.token_type_embed.W_token_type
        n = W.shape[0]
        if n <= 8:
            return F.one_hot(types, n).to(W.dtype) @ W
        return ops.w(W)[types]

    def _embed_pos(self, tokens, run: _Run):
        """Token + position embeddings.  On the fused backend with neither hook observed: one kernel each way
        (``EmbedPosFn``: the backward is the scatter-add kernel, not a gather's index_put backward -- 0.63 ms per
        phase for BERT-base's W_E on MI355X, profiles/mqnli_step_breakdown_r4.txt)."""
        ops = run.ops
        emb = self.embed
        B, S = tokens.shape
        if getattr(ops, "fused", False) and not (run.live(emb.hook_embed) or run.live(emb.hook_pos_embed)):
            return ops.embed_pos(tokens, emb.embed.W_E, emb.pos_embed.W_pos)
        e = run.site(emb.hook_embed, ops.embed(tokens, emb.embed.W_E))
        p = run.site(emb.hook_pos_embed, ops.pos_embed(B, S, emb.pos_embed.W_pos))
        return e + p

    def _embed_ln(self, tokens, run: _Run):
        ops = run.ops
        t = self._token_type_embed(ops, self._token_types(tokens))
        return self.embed.ln.run(self._embed_pos(tokens, run) + t, run)

    def run_paired(self, tokens: torch.Tensor, src_tokens: torch.Tensor, sites, logits: str = "full"):
        """Interchange intervention with the source run folded into the base forward: one pass of 2B rows
        (source rows without autograd) through every block up to the deepest site, which splices inside the
        paired kernels (the decoder's :meth:`iit_amd.models.transformer.HookedTransformer.run_paired`; reference
        ``do_intervention``, /root/reference/iit/model_pairs/base_model_pair.py:80-98).  Sites: ``attn.hook_z``,
        ``mlp.hook_post`` and ``hook_normalized_resid_post`` of any block (MQNLI's position sites).  Returns
        ``(output, {site: source activation})`` or None when not covered (then two forwards run)."""
        import os
        if os.environ.get("IIT_PAIRED", "1") == "0" or not sites:
            return None
        if os.environ.get("IIT_BERT_PAIRED", _BERT_PAIRED_DEFAULT) != "1":  # IIT_BERT_PAIRED=0: two forwards
            return None
        ops = self.ops()
        if not getattr(ops, "supports_pairs", False) or getattr(ops, "pair_layer_norm", None) is None:
            return None
        if tokens.dim() != 2 or tokens.shape != src_tokens.shape or tokens.shape[1] > 64:
            return None
        if any(hp.is_live for hp in self.hook_dict.values()):
            return None
        B, S = tokens.shape
        cfg = self.cfg
        from .transformer import _hip_ops
        order = []
        for name, idxs in sites.items():
            parts = name.split(".")
            if parts[0] != "blocks" or len(parts) < 3 or ".".join(parts[2:]) not in self._PAIR_SITES:
                return None
            li = int(parts[1])
            suffix = ".".join(parts[2:])
            shape = ((B, S, cfg.n_heads, cfg.d_head) if suffix == "attn.hook_z" else
                     (B, S, cfg.d_mlp) if suffix == "mlp.hook_post" else (B, S, cfg.d_model))
            for ix in idxs:
                if _hip_ops().pair_specs(ix, shape) is None:
                    return None
            order.append((li, self._PAIR_SITES.index(suffix), name))
        deepest = max(order)
        if not all(blk.paired_ok() for blk in self.blocks[:deepest[0] + 1]):
            return None
        dev = self.embed.embed.W_E.device
        tokens, src_tokens = tokens.to(dev), src_tokens.to(dev)
        run = _Run(RunPlan(logits=logits), ops)
        ops.begin_forward()
        x = self._embed_ln(tokens, run)
        with torch.no_grad():
            xs = self._embed_ln(src_tokens, run)
        p = _hip_ops().Paired(x, torch.cat([x.detach(), xs]).contiguous())
        captures = {}
        paired = True
        for li, blk in enumerate(self.blocks):
            if paired:
                p, paired = blk.forward_paired(p, run, sites, deepest[2], captures)
            else:
                p = blk(p, run, None)
        x = p.base if paired else p
        if logits == "none":
            return None, captures
        if self.n_classes:
            pooled = torch.tanh(x[:, 0] @ ops.w(self.pooler.W) + ops.w(self.pooler.b))
            return pooled @ ops.w(self.classifier.W) + ops.w(self.classifier.b), captures
        h = F.gelu(x @ ops.w(self.mlm_head.W) + ops.w(self.mlm_head.b))
        h = self.mlm_head.ln.run(h, run)
        return h @ ops.w(self.unembed.W_U) + ops.w(self.unembed.b_U), captures

    def run_capture(self, tokens, names, truncate: bool = True, base_plan: Optional[RunPlan] = None, **kw):
        plan = RunPlan.capture_only(list(names), truncate=truncate)
        if base_plan is not None:
            plan = base_plan.merged(plan)
        with torch.no_grad():
            self.forward(tokens, plan=plan, **kw)
        return plan.cache


def from_hf_bert(hf_model) -> Dict[str, torch.Tensor]:
    """TL-layout parameters from HF ``BertForSequenceClassification`` / ``BertForMaskedLM`` / ``BertModel``."""
    bert = getattr(hf_model, "bert", hf_model)
    cfg = bert.config
    d, H = cfg.hidden_size, cfg.num_attention_heads
    dh = d // H
    t = lambda x: x.detach().clone().float()  # noqa: E731
    emb = bert.embeddings
    sd = {"embed.embed.W_E": t(emb.word_embeddings.weight), "embed.pos_embed.W_pos": t(emb.position_embeddings.weight),
          "embed.token_type_embed.W_token_type": t(emb.token_type_embeddings.weight),
          "embed.ln.w": t(emb.LayerNorm.weight), "embed.ln.b": t(emb.LayerNorm.bias)}
    for l, layer in enumerate(bert.encoder.layer):
        p = f"blocks.{l}."
        s = layer.attention.self
        for n, lin in (("Q", s.query), ("K", s.key), ("V", s.value)):
            sd[p + f"attn.W_{n}"] = t(lin.weight).reshape(H, dh, d).permute(0, 2, 1).contiguous()
            sd[p + f"attn.b_{n}"] = t(lin.bias).reshape(H, dh)
        o = layer.attention.output
        sd[p + "attn.W_O"] = t(o.dense.weight).reshape(d, H, dh).permute(1, 2, 0).contiguous()
        sd[p + "attn.b_O"] = t(o.dense.bias)
        sd[p + "ln1.w"], sd[p + "ln1.b"] = t(o.LayerNorm.weight), t(o.LayerNorm.bias)
        sd[p + "mlp.W_in"] = t(layer.intermediate.dense.weight).t().contiguous()
        sd[p + "mlp.b_in"] = t(layer.intermediate.dense.bias)
        sd[p + "mlp.W_out"] = t(layer.output.dense.weight).t().contiguous()
        sd[p + "mlp.b_out"] = t(layer.output.dense.bias)
        sd[p + "ln2.w"], sd[p + "ln2.b"] = t(layer.output.LayerNorm.weight), t(layer.output.LayerNorm.bias)
    if getattr(bert, "pooler", None) is not None and hasattr(hf_model, "classifier"):
        sd["pooler.W"] = t(bert.pooler.dense.weight).t().contiguous()
        sd["pooler.b"] = t(bert.pooler.dense.bias)
        sd["classifier.W"] = t(hf_model.classifier.weight).t().contiguous()
        sd["classifier.b"] = t(hf_model.classifier.bias)
    if hasattr(hf_model, "cls"):
        tr = hf_model.cls.predictions.transform
        sd["mlm_head.W"] = t(tr.dense.weight).t().contiguous()
        sd["mlm_head.b"] = t(tr.dense.bias)
        sd["mlm_head.ln.w"], sd["mlm_head.ln.b"] = t(tr.LayerNorm.weight), t(tr.LayerNorm.bias)
        sd["unembed.W_U"] = t(hf_model.cls.predictions.decoder.weight).t().contiguous()
        sd["unembed.b_U"] = t(hf_model.cls.predictions.bias if hasattr(hf_model.cls.predictions, "bias")
                              else hf_model.cls.predictions.decoder.bias)
    return sd
