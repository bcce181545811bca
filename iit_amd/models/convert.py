"""Weight conversion from Hugging Face ``transformers`` modules to the TL parameter layout.

The native models use TransformerLens names and layouts (``W_Q [H, d, dh]``,
``W_O [H, dh, d]``, ``W_in [d, d_mlp]``...).  These converters map an in-memory HF
module (random-init or loaded from a *local* checkpoint -- nothing is downloaded)
onto that layout, so HF architectures serve both as numerical references in the
tests (GPT-2, Llama, BERT parity) and as a way to bring existing weights in.

* GPT-2 (``GPT2LMHeadModel``): unfolded LayerNorm (``normalization_type="LN"``);
* Llama (``LlamaForCausalLM``): RMSNorm, rotary (half-split pairs), SwiGLU, GQA;
* BERT (``BertForMaskedLM`` / ``BertModel``): see :mod:`iit_amd.models.bert`.
"""
from __future__ import annotations

from typing import Any, Dict

import torch

from .config import HookedTransformerConfig


def _t(x: torch.Tensor) -> torch.Tensor:
    return x.detach().clone().float()


# ----------------------------------------------------------------------------- GPT-2
def gpt2_cfg_from_hf(hf_cfg, **overrides) -> Dict[str, Any]:
    d = hf_cfg.n_embd
    cfg = dict(n_layers=hf_cfg.n_layer, d_model=d, n_ctx=hf_cfg.n_positions, d_head=d // hf_cfg.n_head,
               n_heads=hf_cfg.n_head, d_mlp=hf_cfg.n_inner or 4 * d, act_fn="gelu_new", d_vocab=hf_cfg.vocab_size,
               eps=hf_cfg.layer_norm_epsilon, normalization_type="LN", original_architecture="GPT2LMHeadModel",
               initializer_range=hf_cfg.initializer_range)
    cfg.update(overrides)
    return cfg


def gpt2_state_dict_from_hf(hf_model) -> Dict[str, torch.Tensor]:
    tr = hf_model.transformer
    cfg = hf_model.config
    d, H = cfg.n_embd, cfg.n_head
    dh = d // H
    sd = {"embed.W_E": _t(tr.wte.weight), "pos_embed.W_pos": _t(tr.wpe.weight)}
    for l, blk in enumerate(tr.h):
        p = f"blocks.{l}."
        sd[p + "ln1.w"] = _t(blk.ln_1.weight)
        sd[p + "ln1.b"] = _t(blk.ln_1.bias)
        W = _t(blk.attn.c_attn.weight)  # [d, 3d] (Conv1D: y = x W + b)
        b = _t(blk.attn.c_attn.bias)
        for i, n in enumerate("QKV"):
            sd[p + f"attn.W_{n}"] = W[:, i * d:(i + 1) * d].reshape(d, H, dh).permute(1, 0, 2).contiguous()
            sd[p + f"attn.b_{n}"] = b[i * d:(i + 1) * d].reshape(H, dh)
        sd[p + "attn.W_O"] = _t(blk.attn.c_proj.weight).reshape(H, dh, d)
        sd[p + "attn.b_O"] = _t(blk.attn.c_proj.bias)
        sd[p + "ln2.w"] = _t(blk.ln_2.weight)
        sd[p + "ln2.b"] = _t(blk.ln_2.bias)
        sd[p + "mlp.W_in"] = _t(blk.mlp.c_fc.weight)
        sd[p + "mlp.b_in"] = _t(blk.mlp.c_fc.bias)
        sd[p + "mlp.W_out"] = _t(blk.mlp.c_proj.weight)
        sd[p + "mlp.b_out"] = _t(blk.mlp.c_proj.bias)
    sd["ln_final.w"] = _t(tr.ln_f.weight)
    sd["ln_final.b"] = _t(tr.ln_f.bias)
    sd["unembed.W_U"] = _t(hf_model.lm_head.weight).t().contiguous()
    sd["unembed.b_U"] = torch.zeros(cfg.vocab_size)
    return sd


# ----------------------------------------------------------------------------- Llama
def llama_cfg_from_hf(hf_cfg, **overrides) -> Dict[str, Any]:
    d, H = hf_cfg.hidden_size, hf_cfg.num_attention_heads
    dh = getattr(hf_cfg, "head_dim", None) or d // H
    rope = getattr(hf_cfg, "rope_theta", None)
    if rope is None:
        rope = (getattr(hf_cfg, "rope_parameters", None) or {}).get("rope_theta", 10000.0)
    cfg = dict(n_layers=hf_cfg.num_hidden_layers, d_model=d, n_ctx=hf_cfg.max_position_embeddings, d_head=dh,
               n_heads=H, d_mlp=hf_cfg.intermediate_size, act_fn="silu", d_vocab=hf_cfg.vocab_size,
               eps=hf_cfg.rms_norm_eps, normalization_type="RMS", positional_embedding_type="rotary",
               rotary_dim=dh, rotary_base=int(rope), gated_mlp=True, final_rms=True,
               n_key_value_heads=hf_cfg.num_key_value_heads, original_architecture="LlamaForCausalLM",
               initializer_range=hf_cfg.initializer_range)
    cfg.update(overrides)
    return cfg


def llama_state_dict_from_hf(hf_model) -> Dict[str, torch.Tensor]:
    m = hf_model.model
    cfg = hf_model.config
    d, H, n_kv = cfg.hidden_size, cfg.num_attention_heads, cfg.num_key_value_heads
    dh = getattr(cfg, "head_dim", None) or d // H
    gqa = n_kv != H
    sd = {"embed.W_E": _t(m.embed_tokens.weight)}
    for l, blk in enumerate(m.layers):
        p = f"blocks.{l}."
        a = blk.self_attn
        sd[p + "ln1.w"] = _t(blk.input_layernorm.weight)
        sd[p + "attn.W_Q"] = _t(a.q_proj.weight).reshape(H, dh, d).permute(0, 2, 1).contiguous()
        kname, vname = ("attn._W_K", "attn._W_V") if gqa else ("attn.W_K", "attn.W_V")
        sd[p + kname] = _t(a.k_proj.weight).reshape(n_kv, dh, d).permute(0, 2, 1).contiguous()
        sd[p + vname] = _t(a.v_proj.weight).reshape(n_kv, dh, d).permute(0, 2, 1).contiguous()
        sd[p + "attn.W_O"] = _t(a.o_proj.weight).reshape(d, H, dh).permute(1, 2, 0).contiguous()
        sd[p + "attn.b_Q"] = torch.zeros(H, dh)
        sd[p + ("attn._b_K" if gqa else "attn.b_K")] = torch.zeros(n_kv, dh)
        sd[p + ("attn._b_V" if gqa else "attn.b_V")] = torch.zeros(n_kv, dh)
        sd[p + "attn.b_O"] = torch.zeros(d)
        sd[p + "ln2.w"] = _t(blk.post_attention_layernorm.weight)
        sd[p + "mlp.W_in"] = _t(blk.mlp.up_proj.weight).t().contiguous()
        sd[p + "mlp.W_gate"] = _t(blk.mlp.gate_proj.weight).t().contiguous()
        sd[p + "mlp.b_in"] = torch.zeros(cfg.intermediate_size)
        sd[p + "mlp.W_out"] = _t(blk.mlp.down_proj.weight).t().contiguous()
        sd[p + "mlp.b_out"] = torch.zeros(d)
    sd["ln_final.w"] = _t(m.norm.weight)
    sd["unembed.W_U"] = _t(hf_model.lm_head.weight).t().contiguous()
    sd["unembed.b_U"] = torch.zeros(cfg.vocab_size)
    return sd


def llama_config_dict(size: str = "llama-3-8b", **overrides) -> Dict[str, Any]:
    """TL-style cfg for Llama-family LL models (``BASELINE.json`` config 5: Llama-3-8B)."""
    presets = {
        "llama-3-8b": dict(n_layers=32, d_model=4096, n_heads=32, n_key_value_heads=8, d_head=128, d_mlp=14336,
                           d_vocab=128256, n_ctx=8192, rotary_base=500000, eps=1e-5),
        "llama-tiny": dict(n_layers=2, d_model=64, n_heads=4, n_key_value_heads=2, d_head=16, d_mlp=172,
                           d_vocab=512, n_ctx=128, rotary_base=10000, eps=1e-5),
    }
    cfg = dict(presets[size])
    cfg.update(act_fn="silu", normalization_type="RMS", positional_embedding_type="rotary", gated_mlp=True,
               final_rms=True, rotary_dim=cfg["d_head"], original_architecture="LlamaForCausalLM",
               model_name=size, initializer_range=0.02)
    cfg.update(overrides)
    return HookedTransformerConfig.from_dict(cfg).to_dict()


def load_converted(model: torch.nn.Module, params: Dict[str, torch.Tensor]) -> torch.nn.Module:
    """Load converted parameters; buffers (causal ``mask``, ``IGNORE``, rotary tables) keep the model's own."""
    full = {k: v.clone() for k, v in model.state_dict().items()}
    unknown = set(params) - set(full)
    if unknown:
        raise KeyError(f"converted keys not in the model: {sorted(unknown)[:5]}")
    full.update({k: v.to(full[k].device, full[k].dtype) for k, v in params.items()})
    model.load_state_dict(full)
    return model
