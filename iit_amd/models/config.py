"""TransformerLens-compatible config (``cfg.to_dict()`` keys), no TL dependency.

The reference builds its LL model from ``HookedTransformer.from_pretrained("gpt2").cfg.to_dict()``
updated with ``ioi_cfg`` (``/root/reference/train_ioi.py:30-34``).  There is no hub
access here, so ``gpt2_config_dict()`` reproduces the GPT-2-small cfg that call
returns (folded LN -> ``normalization_type="LNPre"``, ``gelu_new``, V=50257,
n_ctx=1024, initializer_range=0.02).
"""
from __future__ import annotations

import dataclasses
import math
from dataclasses import dataclass, field
from typing import Any, Dict, Optional

import torch


@dataclass
class HookedTransformerConfig:
    n_layers: int
    d_model: int
    n_ctx: int
    d_head: int
    model_name: str = "custom"
    n_heads: int = -1
    d_mlp: Optional[int] = None
    act_fn: Optional[str] = None
    d_vocab: int = -1
    eps: float = 1e-5
    use_attn_result: bool = False
    use_attn_scale: bool = True
    use_split_qkv_input: bool = False
    use_hook_mlp_in: bool = False
    use_attn_in: bool = False
    use_local_attn: bool = False
    original_architecture: Optional[str] = None
    from_checkpoint: bool = False
    checkpoint_index: Optional[int] = None
    checkpoint_label_type: Optional[str] = None
    checkpoint_value: Optional[int] = None
    tokenizer_name: Optional[str] = None
    window_size: Optional[int] = None
    attn_types: Optional[list] = None
    init_mode: str = "gpt2"
    normalization_type: Optional[str] = "LN"
    device: Optional[str] = None
    n_devices: int = 1
    attention_dir: str = "causal"
    attn_only: bool = False
    seed: Optional[int] = None
    initializer_range: float = -1.0
    init_weights: bool = True
    scale_attn_by_inverse_layer_idx: bool = False
    positional_embedding_type: str = "standard"
    final_rms: bool = False
    d_vocab_out: int = -1
    parallel_attn_mlp: bool = False
    rotary_dim: Optional[int] = None
    n_params: Optional[int] = None
    use_hook_tokens: bool = False
    gated_mlp: bool = False
    default_prepend_bos: bool = True
    dtype: torch.dtype = torch.float32
    tokenizer_prepends_bos: Optional[bool] = None
    n_key_value_heads: Optional[int] = None
    post_embedding_ln: bool = False
    rotary_base: int = 10000
    trust_remote_code: bool = False
    rotary_adjacent_pairs: bool = False

    def __post_init__(self):
        if self.n_heads == -1:
            self.n_heads = self.d_model // self.d_head
        if not self.attn_only:
            if self.d_mlp is None:
                self.d_mlp = 4 * self.d_model
            if self.act_fn is None:
                raise ValueError("act_fn must be specified for non attn-only models")
        if self.initializer_range < 0:
            self.initializer_range = 0.8 / math.sqrt(self.d_model)
        if self.d_vocab_out == -1:
            self.d_vocab_out = self.d_vocab
        if self.device is None:
            self.device = "cuda" if torch.cuda.is_available() else "cpu"
        if isinstance(self.dtype, str):
            self.dtype = getattr(torch, self.dtype)
        self.n_params = self.count_params()

    def count_params(self) -> int:
        d, h, dh = self.d_model, self.n_heads, self.d_head
        per_block = 4 * h * d * dh
        if not self.attn_only:
            per_block += 2 * d * self.d_mlp * (1.5 if self.gated_mlp else 1)
        return int(per_block * self.n_layers)

    @classmethod
    def from_dict(cls, d: Dict[str, Any]) -> "HookedTransformerConfig":
        names = {f.name for f in dataclasses.fields(cls)}
        kw = {k: v for k, v in d.items() if k in names}
        kw.pop("n_params", None)
        return cls(**kw)

    def to_dict(self) -> Dict[str, Any]:
        return {f.name: getattr(self, f.name) for f in dataclasses.fields(self)}

    def __getitem__(self, key):
        return getattr(self, key)


def gpt2_config_dict() -> Dict[str, Any]:
    """The cfg dict ``HookedTransformer.from_pretrained("gpt2").cfg.to_dict()`` yields."""
    return HookedTransformerConfig(
        n_layers=12, d_model=768, n_ctx=1024, d_head=64, model_name="gpt2", n_heads=12, d_mlp=3072,
        act_fn="gelu_new", d_vocab=50257, eps=1e-5, original_architecture="GPT2LMHeadModel",
        tokenizer_name="gpt2", normalization_type="LNPre", initializer_range=0.02, d_vocab_out=50257,
        default_prepend_bos=True, tokenizer_prepends_bos=False,
    ).to_dict()


def make_config(cfg) -> HookedTransformerConfig:
    if isinstance(cfg, HookedTransformerConfig):
        return cfg
    if isinstance(cfg, dict):
        return HookedTransformerConfig.from_dict(cfg)
    raise TypeError(f"cannot make a HookedTransformerConfig from {type(cfg)}")
