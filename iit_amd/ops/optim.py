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
import os
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
        # overlapped update (enable_overlap): a phase followed by another one in the same train step launches only the
        # norm stage; the Adam chunks run on a side stream under the next forward, each layer waiting for its chunk
        self.defer_next = False
        self._pending = None   # argument record of a deferred update not launched yet
        self._inflight = None  # per-chunk events of a launched, not yet joined, deferred update
        self._bounds = None
        self._side = None
        self._events = []
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
        self.join_pending()
        self.flat.zero_grad()

    # ---------------------------------------------------------------- overlapped update
    def enable_overlap(self, stages) -> bool:
        """Let a deferred update (``defer_next``) overlap the next forward.  ``stages``: the model's parameters in
        forward order, one list per stage (embeddings, each block, final norm + unembed); their arena ranges must
        not interleave.  The model calls :meth:`wait_stage` (k) before stage k reads its weights."""
        if self._hip is None or os.environ.get("IIT_ADAM_OVERLAP", "0") == "0":
            return False
        flat, bounds, hi = self.flat, [], 0
        for ps in stages:
            ps = [p for p in ps if flat.owns(p)]
            if ps:
                lo = min(flat.offset_of(p) for p in ps)
                if lo < hi:
                    return False  # interleaved slots: one stage's chunk would hold another's later weights
                hi = max(flat.offset_of(p) + 1 + sum((n - 1) * st for n, st in zip(p.shape, p.stride()))
                         for p in ps)
            bounds.append(hi)
        self._bounds = bounds
        self._side = torch.cuda.Stream(device=flat.data.device)
        return True

    def _launch_pending(self, overlap: bool) -> None:
        from . import hip_kernels
        rec, self._pending = self._pending, None
        cur = torch.cuda.current_stream()
        stream = self._side if overlap else cur
        if overlap:
            stream.wait_stream(cur)
        lr, b1, b2, eps, wd = self._hyper_host
        chunks = rec["chunks"]
        # one event per chunk, created once and re-recorded (no event is destroyed while a phase is being captured)
        while len(self._events) < len(chunks):
            self._events.append(torch.cuda.Event())
        book = next((k for k, (lo, hi) in enumerate(chunks) if hi > lo), 0)  # (an empty chunk launches nothing)
        with torch.cuda.stream(stream):
            for k, (lo, hi) in enumerate(chunks):
                hip_kernels.adam_chunk(self.flat, self.exp_avg, self.exp_avg_sq, self._step_dev, rec, lo, hi, lr=lr,
                                       b1=b1, b2=b2, eps=eps, wd=wd, hyper=self._hyper_dev, book=k == book)
                if overlap:
                    self._events[k].record(stream)
        if overlap and not torch.cuda.is_current_stream_capturing():
            # the side-stream chunks read the record's span table and norm partials after the host drops it: keep
            # the caching allocator from handing those blocks to the current stream meanwhile
            for t in (rec.get("spans"), rec.get("part")):
                if isinstance(t, torch.Tensor):
                    t.record_stream(stream)
        self._inflight = self._events[:len(chunks)] if overlap else None

    @property
    def split_mode(self) -> bool:
        """``IIT_ADAM_OVERLAP=2``: a graph-replayed phase with a pending update is captured as one graph per forward
        stage and the Adam chunks are launched eagerly on the side stream at replay, each stage's graph waiting for
        its chunk's event between replays (cross-stream waits outside any graph; see GraphedTrainStep)."""
        return self._bounds is not None and os.environ.get("IIT_ADAM_OVERLAP", "0") == "2"

    def wait_stage(self, k: int) -> None:
        """Forward gate: stage ``k``'s weights are about to be read (launches a deferred update on first call)."""
        splitter = self.__dict__.get("_splitter")
        if splitter is not None:  # split capture: the graph runner cuts a segment here (nothing launched / waited)
            splitter(k)
            return
        if self._pending is not None:
            self._launch_pending(overlap=True)
        ev = self._inflight
        if ev:
            torch.cuda.current_stream().wait_event(ev[min(k, len(ev) - 1)])
            if k >= len(ev) - 1:
                self._inflight = None

    def capture_guard(self):
        """(state, restore) around a graph capture of a phase that may launch a pending update: if the capture
        fails, ``restore()`` puts the pending record back, forgets events recorded inside the aborted capture and
        drains the side stream, so the eager fallback still applies the update."""
        saved = (self._pending, self._inflight)

        def restore():
            self._pending, self._inflight = saved[0], None
            if self._side is not None:
                self._side.synchronize()
        return restore

    def join_pending(self) -> None:
        """Complete any deferred update before gradients or weights are touched outside a gated forward."""
        if self._pending is not None:
            self._launch_pending(overlap=False)
        if self._inflight:
            torch.cuda.current_stream().wait_event(self._inflight[-1])
            self._inflight = None

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
            # (only with the bf16 mirror: the chunks write it; a refresh pass right here would read stale weights)
            defer = self.defer_next and self._bounds is not None and self.flat.shadow is not None
            self.defer_next = False
            self.join_pending()
            self.step_count += 1
            self._validate_restriction(wd)
            self.sync_hyper()
            capturing = torch.cuda.is_current_stream_capturing()
            if capturing and self._hyper_host != self._hyper():
                raise RuntimeError("FusedAdam: hyper-parameters changed since the last eager step; run one eager "
                                   "step (or sync_hyper()) before capturing")
            if defer:
                rec = hip_kernels.adam_norm_stage(self.flat, self._step_dev, clip_norm=clip_norm,
                                                  skipped=self._skipped_dev if self.nan_guard else None)
                idx = [0] + [self.flat.span_index(b) for b in self._bounds[:-1]] + [rec["nspans"]]
                rec["chunks"] = [(a, max(a, b)) for a, b in zip(idx[:-1], idx[1:])]
                self.flat.after_step(mirror_written=self.flat.shadow is not None)
                self._pending = rec
                return
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
        self.join_pending()
        self.step_count = int(self._step_dev.item())  # device counter is authoritative (guarded skips)
        return {"step": self.step_count, "skipped": self.skipped_steps, "exp_avg": self.exp_avg,
                "exp_avg_sq": self.exp_avg_sq,
                "param_groups": [{k: v for k, v in g.items() if k != "params"} for g in self.param_groups]}

    def load_state_dict(self, sd):
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
