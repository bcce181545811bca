"""Flat parameter / gradient arenas (sized for 288 GB HBM, contiguous for kernels + RCCL).

All trainable parameters of a module are re-bound as views into one fp32 master
buffer, and their ``.grad`` as views into one fp32 gradient buffer:

* ``zero_grad`` is one memset; autograd accumulates in place into the views;
* the fused optimizer (``iit_amd.ops.optim.FusedAdam``) is a single launch over
  the whole arena (global-norm clip computed on device: no host sync);
* data-parallel buckets are contiguous slices of the gradient arena, so RCCL
  all-reduces them in place (no pack/unpack copies);
* an optional bf16 shadow arena holds the compute copy of the weights that the
  HIP kernels read; the optimizer refreshes it in the same pass.

Every parameter slot starts on a 64-element boundary (256 B) so kernels can use
16-byte vector accesses on any slot.
"""
from __future__ import annotations

from typing import Dict, List, Optional, Tuple

import torch
from torch import nn

_ALIGN = 64


class FlatParams:
    def __init__(self, module: nn.Module, with_bf16_shadow: bool = False):
        self.module = module
        self.names: List[str] = []
        self.params: List[nn.Parameter] = []
        self.offsets: List[Tuple[int, int]] = []
        off = 0
        for name, p in module.named_parameters():
            if not p.requires_grad:
                continue
            self.names.append(name)
            self.params.append(p)
            n = p.numel()
            self.offsets.append((off, n))
            off += (n + _ALIGN - 1) // _ALIGN * _ALIGN
        self.numel = off
        dev = self.params[0].device if self.params else torch.device("cpu")
        self.data = torch.zeros(off, dtype=torch.float32, device=dev)
        self.grad = torch.zeros(off, dtype=torch.float32, device=dev)
        self.shadow: Optional[torch.Tensor] = None
        with torch.no_grad():
            for p, (o, n) in zip(self.params, self.offsets):
                view = self.data[o:o + n].view(p.shape)
                view.copy_(p.detach().float())
                p.data = view
                p.grad = self.grad[o:o + n].view(p.shape)
        self.index: Dict[int, int] = {id(p): i for i, p in enumerate(self.params)}
        self.version = 0
        self._listeners = []
        module._flat_params = self
        if with_bf16_shadow:
            self.shadow = torch.empty(off, dtype=torch.bfloat16, device=dev)
            self.refresh_shadow()

    # ---------------------------------------------------------------- grads
    def zero_grad(self) -> None:
        self.grad.zero_()
        self.rebind_grads()

    def rebind_grads(self) -> None:
        """Re-attach ``.grad`` views (after someone set them to None / replaced them)."""
        for p, (o, n) in zip(self.params, self.offsets):
            g = p.grad
            if g is None or g.data_ptr() != self.grad[o:o + n].data_ptr():
                view = self.grad[o:o + n].view(p.shape)
                if g is not None:
                    view.copy_(g)
                p.grad = view

    def grad_view(self, p: torch.Tensor) -> torch.Tensor:
        o, n = self.offsets[self.index[id(p)]]
        return self.grad[o:o + n].view(p.shape)

    # ---------------------------------------------------------------- updates
    def add_listener(self, fn) -> None:
        """``fn()`` runs (on the current stream) after every optimizer update of the arena."""
        self._listeners.append(fn)

    def after_step(self) -> None:
        self.version += 1
        self.module._iit_weights_version = getattr(self.module, "_iit_weights_version", 0) + 1
        self.refresh_shadow()
        for fn in self._listeners:
            fn()

    # ---------------------------------------------------------------- shadow
    def refresh_shadow(self) -> None:
        if self.shadow is not None:
            self.shadow.copy_(self.data)

    def shadow_view(self, p: torch.Tensor) -> torch.Tensor:
        o, n = self.offsets[self.index[id(p)]]
        return self.shadow[o:o + n].view(p.shape)

    # ---------------------------------------------------------------- buckets
    def buckets(self, bucket_bytes: int) -> List[Tuple[int, int]]:
        """Contiguous gradient slices of ~``bucket_bytes`` in reverse parameter order
        (≈ the order backward produces them), for overlapped all-reduce."""
        per = max(_ALIGN, bucket_bytes // 4)
        out = []
        end = self.numel
        while end > 0:
            start = max(0, end - per)
            # snap the bucket start to a parameter boundary
            for o, n in self.offsets:
                if o <= start < o + ((n + _ALIGN - 1) // _ALIGN * _ALIGN):
                    start = o
                    break
            out.append((start, end))
            end = start
        return out
