"""Intervention plans: what a forward pass must capture / splice / skip.

This replaces the reference's "Python closure per HookPoint + cache every hook +
clone/index_put" substrate (``/root/reference/iit/model_pairs/base_model_pair.py:75-105,
120-163``) with a declarative table the model executes natively:

* ``capture``: hook names whose (detached) activation must be stored.  The
  source run of an interchange intervention only captures the hooks the sampled
  HL node maps to and is truncated after the deepest one.
* ``splice``: hook name -> list of ``(TorchIndex, src)``.  Semantics equal the
  reference hook ``out = act.clone(); out[idx] = src[idx]``; the spliced slice is
  a constant, so no gradient flows upstream through it (K10).  Fused HIP kernels
  implement whole-tensor and per-head splices in their epilogues (or skip the
  dead producer); any other index that lowers to a per-dimension range table
  (``TorchIndex.to_ranges``: batch / position / head / feature / channel /
  spatial ranges and lists) is one launch of the patch-spec splice kernel
  (``csrc/splice.hip``), whose backward zeroes the spliced gradient; only
  paired list atoms or stepped slices keep the clone + index_put fallback.
* ``scale`` / ``zero_grad``: StopGrad semantics (K21).
* ``logits``: ``"full"`` (``[B,S,V]``), ``"last"`` (only position -1, K08) or ``"none"``.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

import torch

from ..core.index import EVERYTHING, TorchIndex


def _layer_of(name: str) -> int:
    parts = name.split(".")
    if len(parts) > 1 and parts[0] == "blocks":
        return int(parts[1])
    if name in ("hook_embed", "hook_pos_embed", "hook_tokens"):
        return -1
    return 1 << 30  # ln_final / unembed: after every block


@dataclass
class Splice:
    index: TorchIndex
    src: torch.Tensor  # detached source activation (full hook shape)

    @property
    def whole(self) -> bool:
        return self.index == EVERYTHING or self.index.is_everything()

    def head_mask(self, n_heads: int) -> Optional[List[int]]:
        """Heads covered when the index has the form ``[:, :, heads, :]`` (else None)."""
        idx = self.index.as_index
        if self.whole:
            return list(range(n_heads))
        if len(idx) < 3:
            return None
        if idx[0] != slice(None) or idx[1] != slice(None):
            return None
        if len(idx) == 4 and idx[3] != slice(None):
            return None
        h = idx[2]
        if isinstance(h, int):
            return [h % n_heads]
        if isinstance(h, slice):
            return list(range(n_heads))[h]
        return [v % n_heads for v in h]

    def apply(self, act: torch.Tensor) -> torch.Tensor:
        src = self.src
        if src.dtype != act.dtype or src.device != act.device:
            src = src.to(device=act.device, dtype=act.dtype)
        if self.whole:
            if src.shape != act.shape:
                src = src.expand_as(act)
            return src
        if act.is_cuda:
            from ..ops import splice as _splice
            out = _splice.splice(act, self.index, src)
            if out is not None:
                return out
        out = act.clone()
        ix = self.index.on(act.device)
        out[ix] = src[ix] if src.shape == act.shape else src.expand_as(act)[ix]
        return out


@dataclass
class RunPlan:
    capture: Dict[str, None] = field(default_factory=dict)  # ordered set
    splice: Dict[str, List[Splice]] = field(default_factory=dict)
    scale: Dict[str, float] = field(default_factory=dict)
    zero_grad: Dict[str, List[TorchIndex]] = field(default_factory=dict)
    logits: str = "full"
    truncate: bool = True
    cache: Dict[str, torch.Tensor] = field(default_factory=dict)

    @classmethod
    def capture_only(cls, names: Sequence[str], truncate: bool = True) -> "RunPlan":
        return cls(capture={n: None for n in names}, logits="none", truncate=truncate)

    @classmethod
    def with_splices(cls, splices: Sequence[Tuple[str, TorchIndex, torch.Tensor]], logits: str = "full") -> "RunPlan":
        plan = cls(logits=logits)
        for name, index, src in splices:
            plan.splice.setdefault(name, []).append(Splice(index, src))
        return plan

    def last_layer(self) -> Optional[int]:
        """Deepest block a capture-only plan needs (None = run everything)."""
        if not self.truncate or self.logits != "none" or not self.capture:
            return None
        deepest = max(_layer_of(n) for n in self.capture)
        return None if deepest >= (1 << 30) else deepest

    def touches(self, name: str) -> bool:
        return name in self.capture or name in self.splice or name in self.scale or name in self.zero_grad

    def splice_of(self, name: str) -> Optional[List[Splice]]:
        return self.splice.get(name)

    def merged(self, other: Optional["RunPlan"]) -> "RunPlan":
        """A new plan with this plan's entries plus ``other``'s (other wins on logits / splices)."""
        if other is None:
            return RunPlan(dict(self.capture), {k: list(v) for k, v in self.splice.items()}, dict(self.scale),
                           {k: list(v) for k, v in self.zero_grad.items()}, self.logits, self.truncate)
        out = self.merged(None)
        out.capture.update(other.capture)
        for k, v in other.splice.items():
            out.splice.setdefault(k, []).extend(v)
        out.scale.update(other.scale)
        for k, v in other.zero_grad.items():
            out.zero_grad.setdefault(k, []).extend(v)
        out.logits = other.logits
        out.truncate = other.truncate
        return out


def scale_site(x: torch.Tensor, scale: float) -> torch.Tensor:
    """StopGrad's forward hook ``act / scale`` (/root/reference/iit/model_pairs/stop_grad_pair.py:37-44): on the GPU
    one launch of the patch-spec kernel (csrc/splice.hip, whole-hook range), elsewhere a torch divide."""
    if x.is_cuda:
        from ..ops import splice as _splice
        out = _splice.divide(x, EVERYTHING, scale)
        if out is not None:
            return out
    return x / scale


def zero_grad_site(x: torch.Tensor, idxs) -> torch.Tensor:
    """StopGrad's backward hook ``grad[idx] = 0`` per non-circuit node (stop_grad_pair.py:62-75): on the GPU a fused
    gradient-mask launch per index (csrc/splice.hip), elsewhere a clone + index-assign tensor hook."""
    if x.is_cuda:
        from ..ops import splice as _splice
        out = _splice.grad_mask(x, idxs)
        if out is not None:
            return out

    def _mask(g, _idxs=idxs):
        g = g.clone()
        for ix in _idxs:
            g[ix.on(g.device)] = 0
        return g

    x = x.view_as(x)
    x.register_hook(_mask)
    return x
