"""Fused clip + Adam over a flat parameter arena.

Math is ``torch.optim.Adam`` (amsgrad=False) preceded by
``clip_grad_norm_(params, max_norm)`` exactly as the reference does in
``step_on_loss`` (``/root/reference/iit/model_pairs/iit_behavior_model_pair.py:60-64``,
``base_model_pair.py:176-180,229``): total L2 norm over every parameter,
``coef = min(1, max_norm / (norm + 1e-6))``.

On a GPU with the HIP extension loaded the whole update is two launches
(a two-stage global-norm reduction and one fused clip+Adam+bf16-shadow pass);
the norm never leaves the device, so a training step has no host sync.
Elsewhere a vectorised torch implementation of the same math is used.
"""
from __future__ import annotations

import math
from typing import Optional

import torch

from ..engine.flat import FlatParams


class FusedAdam(torch.optim.Optimizer):
    """Adam over a :class:`FlatParams` arena.

    ``nan_guard`` (default on): a step whose (clipped) gradient holds inf/nan is
    skipped entirely -- weights, moments and the step counter stay untouched -- and
    counted in :attr:`skipped_steps`.  On the GPU the check runs inside the fused
    kernel (no host sync); the device step counter is the authoritative step count.
    """

    def __init__(self, flat: FlatParams, lr: float = 1e-3, betas=(0.9, 0.999), eps: float = 1e-8,
                 weight_decay: float = 0.0, use_hip: Optional[bool] = None, nan_guard: bool = True,
                 alloc_moments: bool = True):
        defaults = dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay)
        super().__init__(flat.params, defaults)
        self.flat = flat
        # (the sharded subclass allocates shard-sized moments itself: no transient arena-sized pair)
        flat.zeroes_missing_on_step = True  # step() zeroes None-gradient slots (one launch, rebind_grads)
        self.exp_avg = torch.zeros_like(flat.data) if alloc_moments else None
        self.exp_avg_sq = torch.zeros_like(flat.data) if alloc_moments else None
        self.step_count = 0
        self.pending_clip = None
        self.nan_guard = nan_guard
        dev = flat.data.device
        self._step_dev = torch.zeros(1, dtype=torch.int32, device=dev)  # device-side step counter
        self._skipped_dev = torch.zeros(1, dtype=torch.int32, device=dev)
        # device copy of (lr, beta1, beta2, eps, weight_decay): the fused kernel reads it, so a graph-captured
        # step follows hyper-parameter changes (an LR scheduler) made between replays -- see sync_hyper
        self._hyper_dev = torch.zeros(5, dtype=torch.float32, device=dev)
        self._hyper_host = None
        if use_hip is None:
            use_hip = flat.data.is_cuda
        self._hip = None
        if use_hip:
            from . import hip_kernels
            self._hip = hip_kernels.lib()

    def _hyper(self):
        group = self.param_groups[0]
        (b1, b2) = group["betas"]
        return (float(group["lr"]), float(b1), float(b2), float(group["eps"]), float(group["weight_decay"]))

    def sync_hyper(self) -> None:
        """Copy changed hyper-parameters to the device scalars the fused kernel reads.  Called by every eager
        ``step`` and by the graph runners before each replay of a captured phase (a replay does not run ``step``'s
        host code); a no-op while capturing and when nothing changed."""
        h = self._hyper()
        if h == self._hyper_host:
            return
        if torch.cuda.is_available() and torch.cuda.is_current_stream_capturing():
            return  # the eager warm-up before the capture has already synchronised them
        self._hyper_dev.copy_(torch.tensor(h, dtype=torch.float32))
        self._hyper_host = h

    @property
    def skipped_steps(self) -> int:
        return int(self._skipped_dev.item())

    def zero_grad(self, set_to_none: bool = False):  # noqa: D401 - arena memset
        self.flat.zero_grad()

    @torch.no_grad()
    def step(self, closure=None, clip_norm: Optional[float] = None):
        if closure is not None:
            with torch.enable_grad():
                closure()
        self.flat.rebind_grads(zero_missing=True)  # gradients no backward produced (lazy zero_grad) are zero
        group = self.param_groups[0]
        lr, (b1, b2), eps, wd = group["lr"], group["betas"], group["eps"], group["weight_decay"]
        g = self.flat.grad
        if self._hip is not None:
            from . import hip_kernels
            self.step_count += 1
            self._validate_restriction(wd)
            self.sync_hyper()
            capturing = torch.cuda.is_current_stream_capturing()
            if capturing and self._hyper_host != self._hyper():
                raise RuntimeError("FusedAdam: hyper-parameters changed since the last eager step; run one eager "
                                   "step (or sync_hyper()) before capturing")
            hip_kernels.adam_step(self.flat, self.exp_avg, self.exp_avg_sq, self._step_dev, lr=lr, b1=b1, b2=b2,
                                  eps=eps, wd=wd, clip_norm=clip_norm,
                                  skipped=self._skipped_dev if self.nan_guard else None, hyper=self._hyper_dev)
            return
        norm = torch.linalg.vector_norm(g) if (clip_norm or self.nan_guard) else None
        if self.nan_guard and not bool(torch.isfinite(norm)):
            self._skipped_dev += 1
            return
        self.step_count += 1
        self._step_dev += 1
        t = self.step_count
        bc1 = 1.0 - b1 ** t
        bc2 = 1.0 - b2 ** t
        if clip_norm:
            g.mul_(torch.clamp(clip_norm / (norm + 1e-6), max=1.0))
        if wd:
            g = g.add(self.flat.data, alpha=wd)
        self.exp_avg.mul_(b1).add_(g, alpha=1 - b1)
        self.exp_avg_sq.mul_(b2).addcmul_(g, g, value=1 - b2)
        denom = (self.exp_avg_sq.sqrt() / math.sqrt(bc2)).add_(eps)
        self.flat.data.addcdiv_(self.exp_avg, denom, value=-lr / bc1)
        self.flat.after_step()

    def _validate_restriction(self, wd: float) -> None:
        """Row restriction (``FlatParams.restrict_rows``) is exact only without weight decay and with zero
        moments on the skipped rows; checked once per restriction change (outside graph capture)."""
        flat = self.flat
        if not flat._inactive or getattr(self, "_restrict_ok_version", None) == flat.restrict_version:
            return
        if torch.cuda.is_available() and torch.cuda.is_current_stream_capturing():
            return
        ok = wd == 0 and flat.check_inactive_zero(self.exp_avg, self.exp_avg_sq, flat.grad)
        if not ok:
            flat._inactive.clear()
            flat.drop_span_cache()
            flat.restrict_version += 1
        self._restrict_ok_version = flat.restrict_version

    # ---------------------------------------------------------------- checkpointing
    def state_dict(self):
        self.step_count = int(self._step_dev.item())  # device counter is authoritative (guarded skips)
        return {"step": self.step_count, "skipped": self.skipped_steps, "exp_avg": self.exp_avg,
                "exp_avg_sq": self.exp_avg_sq, "arena_layout": self.flat.layout_tag(),
                "param_groups": [{k: v for k, v in g.items() if k != "params"} for g in self.param_groups]}

    def load_state_dict(self, sd):
        tag = sd.get("arena_layout")
        if tag is None:
            print("[iit] optimizer state without an arena layout tag (saved before round 6): loaded as is -- its "
                  "moments are only valid for the same parameter layout")
        elif tag != self.flat.layout_tag():
            raise ValueError(f"optimizer state was saved for another arena layout ({tag} != "
                             f"{self.flat.layout_tag()}): its Adam moments would land on the wrong parameters")
        self.step_count = int(sd["step"])
        self._step_dev.fill_(self.step_count)
        self._skipped_dev.fill_(int(sd.get("skipped", 0)))
        self.exp_avg.copy_(sd["exp_avg"])
        self.exp_avg_sq.copy_(sd["exp_avg_sq"])
        for g, saved in zip(self.param_groups, sd["param_groups"]):
            g.update(saved)


def clip_grad_norm_(params, max_norm: float) -> torch.Tensor:
    """Sync-free global-norm clip (same math as ``torch.nn.utils.clip_grad_norm_``)."""
    grads = [p.grad for p in params if p.grad is not None]
    if not grads:
        return torch.zeros(())
    norm = torch.linalg.vector_norm(torch.stack([torch.linalg.vector_norm(g) for g in grads]))
    coef = torch.clamp(max_norm / (norm + 1e-6), max=1.0)
    for g in grads:
        g.mul_(coef)
    return norm
