"""Op backends for the native LL models.

* ``torch`` – :class:`TorchOps`, reference semantics, any device / dtype (oracle).
* ``hip``   – :class:`iit_amd.ops.hip_ops.HipOps`, hand-written gfx950 kernels
  (bf16 activations, fp32 accumulation / residual stream / master weights).

``select_ops(model, backend)`` picks per call: ``backend=None`` means "hip when
the model lives on a GPU and computes in bf16, else torch".  Asking for ``hip``
explicitly on a GPU when the extension is not built raises (no silent fallback).
"""
from __future__ import annotations

from typing import Optional

import torch

from .torch_ops import TorchOps, gelu_new

_TORCH_OPS_CACHE = {}


def _torch_ops(dtype):
    ops = _TORCH_OPS_CACHE.get(dtype)
    if ops is None:
        ops = _TORCH_OPS_CACHE[dtype] = TorchOps(dtype)
    return ops


def hip_supported(cfg) -> bool:
    """Architectures the fused HIP backend implements (GPT-2 family and BERT encoders); others run TorchOps on
    the GPU (bf16 compute, library GEMMs) until their kernels exist (RMSNorm / rotary / SwiGLU / GQA)."""
    return (cfg.positional_embedding_type == "standard" and cfg.normalization_type in ("LN", "LNPre", None)
            and not cfg.gated_mlp and (cfg.n_key_value_heads in (None, cfg.n_heads))
            and not cfg.parallel_attn_mlp and not cfg.final_rms
            and cfg.act_fn in ("gelu_new", "gelu_fast", "gelu_pytorch_tanh", "gelu", "relu"))


def select_ops(model, backend: Optional[str] = None):
    cfg = model.cfg
    dtype = cfg.dtype
    on_gpu = next(model.parameters()).is_cuda
    if backend is None:
        from .. import config as _config
        env = _config.backend()
        backend = "hip" if (on_gpu and dtype == torch.bfloat16 and env == "hip" and hip_supported(cfg)) else "torch"
    if backend == "torch":
        return _torch_ops(dtype)
    if backend == "hip":
        if not on_gpu:
            raise RuntimeError("hip op backend requires the model on a GPU")
        from .hip_ops import get_hip_ops
        return get_hip_ops(model)
    raise ValueError(f"unknown op backend {backend}")


def cross_entropy(logits: torch.Tensor, target: torch.Tensor) -> torch.Tensor:
    """Mean CE with index targets; fused HIP kernel on GPU (fp32 logits, any row stride)."""
    if logits.is_cuda and logits.dim() == 2 and not target.dtype.is_floating_point:
        from .hip_ops import cross_entropy as _hip_ce
        return _hip_ce(logits, target)
    return torch.nn.functional.cross_entropy(logits.float(), target)
