"""Flat parameter / gradient arenas (sized for 288 GB HBM, contiguous for kernels + RCCL).

All trainable parameters of a module are re-bound as views into one fp32 master
buffer, and their ``.grad`` as views into one fp32 gradient buffer:

* ``zero_grad`` is one memset; autograd accumulates in place into the views;
* the fused optimizer (``iit_amd.ops.optim.FusedAdam``) is a single launch over
  the whole arena (global-norm clip computed on device: no host sync);
* data-parallel buckets are contiguous slices of the gradient arena, so RCCL
  all-reduces them in place (no pack/unpack copies);
* an optional bf16 *mirror* arena (same layout) holds the compute copy of the
  weights the HIP kernels read; the fused optimizer writes it in the same pass
  as the update, so no separate cast/transposition pass exists.

**Kernel-layout groups.**  A module may define ``_iit_arena_groups()`` returning
``[(numel, [(param, view_fn), ...]), ...]``: the members of a group share one
arena slot laid out the way the GEMM kernels want the operand (e.g. ``W_Q``,
``W_K``, ``W_V`` interleaved as one ``[d_model][3*H*d_head]`` matrix, ``W_U``
with 16-byte aligned rows), and each parameter becomes a strided view
``view_fn(slot)`` with its usual TL shape.  Parameters keep their public shapes
and semantics; only their strides change.

Every slot starts on a 64-element boundary (256 B) so kernels can use 16-byte
vector accesses on any slot.
"""
from __future__ import annotations

from typing import Callable, Dict, List, Optional, Tuple

import numpy as np
import torch
from torch import nn

_ALIGN = 64


def _align(n: int) -> int:
    return (n + _ALIGN - 1) // _ALIGN * _ALIGN


def _subtract_ranges(ranges, holes):
    """Sorted disjoint ``ranges`` minus sorted disjoint ``holes`` (both lists of half-open (start, end))."""
    out = []
    hi = 0
    for a, b in ranges:
        cur = a
        while hi < len(holes) and holes[hi][1] <= cur:
            hi += 1
        j = hi
        while j < len(holes) and holes[j][0] < b:
            ha, hb = holes[j]
            if ha > cur:
                out.append((cur, ha))
            cur = max(cur, hb)
            j += 1
        if cur < b:
            out.append((cur, b))
    return out


def make_span_tensor(spans, device) -> torch.Tensor:
    """Pack ``[(arena start4, local start4, len4), ...]`` as the kernels' 24-byte ``Span`` records (int64 triples;
    the length's high word is the zero pad)."""
    return torch.tensor(spans if spans else [(0, 0, 0)], dtype=torch.int64).view(-1, 3).to(device)


class FlatParams:
    def __init__(self, module: nn.Module, with_bf16_shadow: bool = False):
        self.module = module
        self.names: List[str] = []
        self.params: List[nn.Parameter] = []
        self._view_fns: List[Callable[[torch.Tensor], torch.Tensor]] = []
        self.slots: List[Tuple[int, int]] = []  # (offset, numel) allocation units, arena order

        groups = module._iit_arena_groups() if hasattr(module, "_iit_arena_groups") else []
        member: Dict[int, Tuple[int, Callable]] = {}
        for gi, (numel, members) in enumerate(groups):
            if not members or not all(p.requires_grad for p, _ in members):
                continue
            for p, fn in members:
                member[id(p)] = (gi, fn)
        placed: Dict[int, int] = {}
        off = 0
        for name, p in module.named_parameters():
            if not p.requires_grad:
                continue
            self.names.append(name)
            self.params.append(p)
            if id(p) in member:
                gi, fn = member[id(p)]
                n = groups[gi][0]
                if gi not in placed:
                    placed[gi] = off
                    self.slots.append((off, n))
                    off += _align(n)
                go = placed[gi]
                self._view_fns.append(lambda buf, go=go, n=n, fn=fn: fn(buf[go:go + n]))
            else:
                n = p.numel()
                self.slots.append((off, n))
                if p.dim() == 4 and p.is_contiguous(memory_format=torch.channels_last) and not p.is_contiguous():
                    # a channels-last conv weight keeps its NHWC order in the arena (an NCHW view would make every
                    # NHWC convolution transpose it on each call)
                    N_, C_, H_, W_ = p.shape
                    self._view_fns.append(lambda buf, o=off, n=n, sh=(N_, H_, W_, C_):
                                          buf[o:o + n].view(sh).permute(0, 3, 1, 2))
                else:
                    self._view_fns.append(lambda buf, o=off, n=n, shape=p.shape: buf[o:o + n].view(shape))
                off += _align(n)
        self.numel = off
        # per-parameter arena layout (slot offset, shape, element order): optimizer state saved as arena-shaped
        # tensors is only meaningful for the same layout (see ``layout_tag``)
        self._layout = [(nm, o, tuple(p.shape),
                         "nhwc" if (p.dim() == 4 and p.is_contiguous(memory_format=torch.channels_last)
                                    and not p.is_contiguous()) else "dense")
                        for nm, p, (o, _n) in zip(self.names, self.params, self.slots)] \
            if len(self.slots) == len(self.params) else [(nm, tuple(p.shape)) for nm, p in zip(self.names, self.params)]
        dev = self.params[0].device if self.params else torch.device("cpu")
        self.data = torch.zeros(off, dtype=torch.float32, device=dev)
        self.grad = torch.zeros(off, dtype=torch.float32, device=dev)
        self.shadow: Optional[torch.Tensor] = None
        with torch.no_grad():
            for p, fn in zip(self.params, self._view_fns):
                view = fn(self.data)
                assert view.shape == p.shape, (view.shape, p.shape)
                view.copy_(p.detach().float())
                p.data = view
                p.grad = fn(self.grad)
                p._iit_flat = self  # back-reference: bf16 mirror lookup by the torch op backend
        self.index: Dict[int, int] = {id(p): i for i, p in enumerate(self.params)}
        self._grad_views = None  # (grad arena, cached per-parameter grad views) for rebind_grads
        self._claimed = set()    # parameter indices whose gradient a store-producer wrote (see ``claim``)
        self._declined = set()   # ... whose producer preferred zero + accumulate (``unclaim``)
        self._zero_plan = None
        self._zero_plans = {}    # claim set -> zero plan; every device table a captured graph may read stays alive
        self._retired = []       # replaced device tables (span tables) kept alive for the same reason
        self.version = 0
        self.mirror_version = -1
        self._inactive: Dict[int, Tuple[int, int, torch.Tensor]] = {}  # param index -> (offset, row_len, live rows)
        self.restrict_version = 0
        self._span_cache = None
        self._listeners = []
        # fused gradient norm (see ``norm_cover``): off unless the training loop turns it on (single process, nothing
        # rewrites gradients between the backward and the optimizer step)
        self.norm_fuse = False
        self.gsq: Optional[torch.Tensor] = None
        self._norm_covered = set()   # parameter indices whose sum of squares a store GEMM added into ``gsq``
        self._norm_capable = set()   # ... whose producer can do so when it stores (``norm_intent``)
        self._norm_dirty = False     # a covered gradient was accumulated into afterwards: full norm pass
        self._sq_span_cache = {}
        module._flat_params = self
        if with_bf16_shadow:
            self.ensure_shadow()

    # ---------------------------------------------------------------- layout queries
    def layout_tag(self) -> str:
        """Digest of the arena layout: every parameter's name, offset, shape and element order (NHWC conv weights
        keep channels-last order).  Arena-shaped optimizer state (Adam moments, ZeRO shards) carries it, so state
        from another layout -- e.g. an NCHW-era checkpoint of a model whose conv weights are now NHWC, whose
        moments would load silently permuted -- is refused."""
        import hashlib
        return hashlib.sha1(repr((self.numel, self._layout)).encode()).hexdigest()[:16]

    def offset_of(self, p: torch.Tensor) -> int:
        """Element offset of ``p``'s first element inside the arena."""
        return (p.data_ptr() - self.data.data_ptr()) // self.data.element_size()

    @property
    def offsets(self) -> List[Tuple[int, int]]:
        """(start offset, numel) of every parameter (grouped params share their slot's span)."""
        return [(self.offset_of(p), p.numel()) for p in self.params]

    def owns(self, p: torch.Tensor) -> bool:
        base = self.data.data_ptr()
        return base <= p.data_ptr() < base + self.numel * 4

    # ---------------------------------------------------------------- sparse rows
    def restrict_rows(self, p: torch.Tensor, live_rows: Optional[torch.Tensor]) -> bool:
        """Declare that only ``live_rows`` of the 2-D parameter ``p`` can ever receive gradient (embedding rows
        of the tokens a dataset contains, positional rows below its sequence length).  The fused optimizer then
        skips the other rows: with zero gradient and zero Adam moments (and no weight decay) an Adam step leaves
        them bit-identical, so this is exact.  ``live_rows=None`` lifts the restriction.  Returns whether the
        restriction applies (it needs a plain, non-grouped slot whose rows are whole float4 groups)."""
        i = self.index.get(id(p))
        if i is None:
            return False
        # rows skipped so far were never memset by zero_grad: a backward outside the restricted data (after
        # train() returned) may have left sums there, which must not reach Adam once the rows are live again
        stale = self.inactive_ranges() if i in self._inactive else []
        g = getattr(self, "grad", None)
        if g is not None:
            for a, b in stale:
                g[a:b].zero_()
        if live_rows is None:
            self._inactive.pop(i, None)
        else:
            if p.dim() != 2 or not p.is_contiguous() or p.shape[1] % 4:
                return False
            off = self.offset_of(p)
            if off % 4:
                return False
            rows = torch.unique(live_rows.detach().long().cpu())
            rows = rows[(rows >= 0) & (rows < p.shape[0])]
            self._inactive[i] = (off, int(p.shape[1]), rows)
        self.restrict_version += 1
        self.drop_span_cache()
        return True

    def drop_span_cache(self) -> None:
        """Forget the optimizer span table; the old device table is retired, not freed (a captured optimizer
        graph keeps reading its address until it is re-captured)."""
        if self._span_cache is not None:
            self._retired.append(self._span_cache[1])
        self._span_cache = None

    def inactive_ranges(self) -> List[Tuple[int, int]]:
        """Sorted (start, end) element ranges the optimizer may skip."""
        out = []
        for i, (off, d, rows) in self._inactive.items():
            n = self.params[i].shape[0]
            live = torch.zeros(n, dtype=torch.bool)
            live[rows] = True
            r = 0
            while r < n:
                if live[r]:
                    r += 1
                    continue
                r0 = r
                while r < n and not live[r]:
                    r += 1
                out.append((off + r0 * d, off + r * d))
        return sorted(out)

    def span_table(self, span_bytes: int = 24, max_len4: int = 1024, restricted: bool = True):
        """Device table of optimizer span records (arena start, gradient / moment start, length; float4 units)
        covering the active arena (``restricted=False``: all of it), as read by the fused optimizer kernels
        (``Span`` in csrc/kernels.hip; the replicated optimizer reads gradient and moments at the arena offset).
        Cached until the restriction changes."""
        key = (restricted, max_len4)
        if self._span_cache is not None and self._span_cache[0] == key:
            return self._span_cache[1], self._span_cache[2]
        assert span_bytes == 24
        n4 = self.numel // 4
        gaps = [(a // 4, b // 4) for a, b in self.inactive_ranges()] if restricted else []
        spans = []
        pos = 0
        for a, b in gaps + [(n4, n4)]:
            while pos < a:
                ln = min(max_len4, a - pos)
                spans.append((pos, pos, ln))
                pos += ln
            pos = max(pos, b)
        tab = make_span_tensor(spans, self.data.device)
        self.drop_span_cache()
        self._span_cache = (key, tab, len(spans))
        return tab, len(spans)

    def check_inactive_zero(self, *tensors: torch.Tensor) -> bool:
        """True when every skipped range is zero in each given arena-shaped tensor (default: the gradient)."""
        for t in tensors or (self.grad,):
            for a, b in self.inactive_ranges():
                if bool(t[a:b].any()):
                    return False
        return True

    # ---------------------------------------------------------------- grads
    def zero_grad(self) -> None:
        """Zero every gradient -- lazily for *store-claimed* parameters, and never the restricted rows.

        A parameter whose gradient the previous backward produced with a single overwriting GEMM (``claim``) gets
        ``.grad = None`` instead of a memset: its producer stores into the slot (beta = 0, no read of the old
        gradient) and whatever is still ``None`` when the gradients are consumed is zeroed then
        (``rebind_grads(zero_missing=True)``: the optimizer step / the DP reducer).  Everything else -- biases,
        norms, embeddings, autograd-accumulated parameters -- is memset here.  For the GPT-2 / Llama matrices this
        removes one write pass (zero) and one read pass (accumulate) over the gradient arena per optimizer step.

        Rows excluded by :meth:`restrict_rows` (embedding rows of tokens the data never contains) are never written
        by a backward over that data, so they stay zero without a memset (GPT-2's 50k x 768 ``W_E`` slot shrinks
        to its ~100 live rows).  On the GPU the memset is one launch per 128 ranges with the ranges passed as kernel
        arguments: no device table, so a plan first needed inside a graph capture is still a single node.  Plans
        are cached per (claim set, restriction)."""
        if self._norm_covered:  # a backward ran without an optimizer step consuming its fused norm sums
            self._norm_covered, self._norm_dirty = set(), False
            self.gsq.zero_()
        key = (frozenset(self._claimed), self.restrict_version)
        plan = self._zero_plans.get(key)
        if plan is None:
            claimed = key[0]
            lazy = set()
            for o, n in self.slots:  # a slot is lazy only when every parameter in it is claimed
                members = [i for i, p in enumerate(self.params) if o <= self.offset_of(p) < o + max(n, 1)]
                if members and all(i in claimed for i in members):
                    lazy.add(o)
            ranges = []
            for o, n in self.slots:  # memset runs over the non-lazy slots (arena order)
                if o in lazy:
                    continue
                end = o + _align(n)
                if ranges and ranges[-1][1] == o:
                    ranges[-1] = (ranges[-1][0], end)
                else:
                    ranges.append((o, end))
            ranges = _subtract_ranges(ranges, self.inactive_ranges())
            none_ids = [i for i, p in enumerate(self.params)
                        if any(o <= self.offset_of(p) < o + max(n, 1) and o in lazy for o, n in self.slots)]
            starts = np.array([a for a, _ in ranges], dtype=np.int64)
            lens = np.array([b - a for a, b in ranges], dtype=np.int64)
            plan = self._zero_plans[key] = (ranges, none_ids, starts, lens)
        self._zero_plan = plan
        ranges, none_ids, starts, lens = plan
        if self.grad.is_cuda:
            from ..ops import hip_kernels
            hip_kernels.zero_ranges(self.grad, starts, lens)
        else:
            for a, b in ranges:
                self.grad[a:b].zero_()
        self.rebind_grads()
        for i in none_ids:
            self.params[i].grad = None

    # ---------------------------------------------------------------- fused gradient norm
    def norm_cover(self, *ps: torch.Tensor) -> Optional[torch.Tensor]:
        """Called by a producer that just claimed (``claim`` -> True) the gradients of ``ps`` and stores them
        complete with one GEMM: returns the 64 device slots that GEMM adds the sum of squares of the stored
        gradient into (``gemm(..., gsq=...)``), and marks ``ps`` covered, so the optimizer's norm pass skips their
        slots (``norm_spans``).  The clip's global norm then costs no separate read of these gradients.  None when
        fusion is off (``norm_fuse``: data parallelism reduces gradients after the GEMM; a pair that rewrites
        gradients before the step) or in deterministic mode (the slot sums are fp32 atomics)."""
        if not self.norm_fuse or not self.grad.is_cuda:
            return None
        from ..ops.gemm_dispatch import deterministic
        if deterministic():
            return None
        idx = [self.index.get(id(p)) for p in ps]
        if any(i is None for i in idx):
            return None
        if self.gsq is None:
            self.gsq = torch.zeros(64, dtype=torch.float32, device=self.grad.device)
        self._norm_covered.update(idx)
        return self.gsq

    def norm_intent(self, *ps: torch.Tensor) -> None:
        """A producer that covers ``ps`` whenever it stores their gradient (see ``norm_cover``) ran: the norm span
        table for that cover set is built ahead, outside graph capture (a capture cannot upload a new table)."""
        if self.norm_fuse:
            self._norm_capable.update(i for i in (self.index.get(id(p)) for p in ps) if i is not None)

    def norm_spans(self, span_bytes: int = 24, max_len4: int = 1024):
        """(span table, count, gsq) for the optimizer's norm pass: the active spans minus the slots whose every
        parameter a GEMM covered this step, and the slots those GEMMs added into; (None, 0, None) for the plain
        pass over the Adam spans.  Resets the step's cover state."""
        covered, dirty = frozenset(self._norm_covered), self._norm_dirty
        self._norm_covered, self._norm_dirty = set(), False
        capturing = self.grad.is_cuda and torch.cuda.is_current_stream_capturing()
        if self._norm_capable and not capturing:  # the table the next (possibly captured) steps will need
            self._norm_table(frozenset(self._norm_capable), span_bytes, max_len4)
        if not covered or self.gsq is None:
            return None, 0, None
        key = (covered, self.restrict_version, max_len4)
        if dirty or (capturing and key not in self._sq_span_cache):
            # a covered gradient changed after its GEMM (its sum is stale), or a cover set first seen inside a
            # capture: drop the slot sums and read every gradient
            self.gsq.zero_()
            return None, 0, None
        tab, n = self._norm_table(covered, span_bytes, max_len4)
        return tab, n, self.gsq

    def _norm_table(self, covered, span_bytes: int, max_len4: int):
        key = (covered, self.restrict_version, max_len4)
        ent = self._sq_span_cache.get(key)
        if ent is None:
            holes = []
            for o, n in self.slots:
                members = [i for i, p in enumerate(self.params) if o <= self.offset_of(p) < o + max(n, 1)]
                if members and all(i in covered for i in members):
                    holes.append((o, o + _align(n)))  # with the slot's zero padding: float4-aligned ends
            live = _subtract_ranges([(0, self.numel)], sorted(holes + self.inactive_ranges()))
            spans = []
            for a, b in live:
                assert a % 4 == 0 and b % 4 == 0, (a, b)
                a4, b4 = a // 4, b // 4
                pos = a4
                while pos < b4:
                    ln = min(max_len4, b4 - pos)
                    spans.append((pos, pos, ln))
                    pos += ln
            assert span_bytes == 24
            ent = self._sq_span_cache[key] = (make_span_tensor(spans, self.data.device), len(spans))
        return ent

    def claim(self, *ps: torch.Tensor) -> bool:
        """Called by a producer that writes the *complete* gradient of ``ps`` (one slot, e.g. the packed
        ``W_Q|W_K|W_V`` group) with a single GEMM: True -> store (the slot holds garbage, overwrite it); False
        -> accumulate (the gradients are live).  Binds ``.grad`` to the arena views either way."""
        idx = [self.index.get(id(p)) for p in ps]
        if any(i is None for i in idx):
            return False
        if any(i in self._declined for i in idx):  # producer chose zero + accumulate: bulk-memset slots
            for p in ps:
                if p.grad is None:
                    self.bind_zero(p)
            return False
        self._claimed.update(idx)  # a store-capable producer: lazily zero these from the next zero_grad on
        fresh = all(p.grad is None for p in ps)
        if not fresh:
            if self._norm_covered.intersection(idx):
                self._norm_dirty = True  # accumulating into a gradient whose square sum is already in gsq
            for p in ps:
                if p.grad is None:
                    self.bind_zero(p)
            return False
        views = self._views()
        for i, p in zip(idx, ps):
            p.grad = views[i]
        return True

    def unclaim(self, *ps: torch.Tensor) -> None:
        """The producer of ``ps`` zero-fills and accumulates after all (e.g. split-K wins): from the next
        ``zero_grad`` on their slots are part of the bulk memset again."""
        for p in ps:
            i = self.index.get(id(p))
            if i is not None:
                self._claimed.discard(i)
                self._declined.add(i)

    def bind_zero(self, p: torch.Tensor) -> torch.Tensor:
        """``p.grad`` := its (zeroed) arena view, for producers that accumulate into a ``None`` gradient."""
        i = self.index[id(p)]
        v = self._views()[i]
        if p.grad is None:
            v.zero_()
        elif p.grad is not v:
            v.copy_(p.grad)
        p.grad = v
        return v

    def _views(self):
        views = self._grad_views
        if views is None or views[0] is not self.grad:
            views = self._grad_views = (self.grad, [fn(self.grad) for fn in self._view_fns])
        return views[1]

    def rebind_grads(self, zero_missing: bool = False) -> None:
        """Re-attach ``.grad`` views (after someone set them to None / replaced them).

        A replaced gradient is copied into its slot and a ``None`` gradient
        (``optimizer.zero_grad(set_to_none=True)``, or a lazily zeroed slot no producer
        claimed) gets its slot zeroed, so the arena equals the gradients.  (``zero_missing``
        is kept for callers; ``None`` slots are always zeroed.)"""
        missing = []
        for i, (p, view) in enumerate(zip(self.params, self._views())):
            g = p.grad
            if g is view:  # the common case (host cost matters: the DP schedule calls this twice per phase)
                continue
            if g is None:
                # a None gradient is zero (set_to_none / lazy zero_grad): the arena slot may hold stale values
                missing.append(i)
            elif g.data_ptr() != view.data_ptr() or g.stride() != view.stride():
                view.copy_(g)
            p.grad = view
        if missing:  # one multi-tensor launch: whole slots whose members are all missing, else the single views
            views = self._views()
            by_slot = {}
            for i in missing:
                by_slot.setdefault(self._slot_of(i), []).append(i)
            parts = []
            for (o, n), idx in sorted(by_slot.items()):
                if len(idx) == len(self._slot_members()[(o, n)]):
                    parts.append(self.grad[o:o + n])
                else:
                    parts.extend(views[i] for i in idx)
            torch._foreach_zero_(parts)

    def _slot_of(self, i: int) -> Tuple[int, int]:
        """(offset, numel) of the arena slot holding parameter ``i``."""
        slots = self.__dict__.get("_slot_index")
        if slots is None:
            slots = self._slot_index = {}
        if i not in slots:
            off = self.offset_of(self.params[i])
            slots[i] = next((o, n) for o, n in self.slots if o <= off < o + max(n, 1))
        return slots[i]

    def _slot_members(self) -> Dict[Tuple[int, int], List[int]]:
        members = self.__dict__.get("_members")
        if members is None:
            members = self._members = {}
            for i in range(len(self.params)):
                members.setdefault(self._slot_of(i), []).append(i)
        return members

    def grad_view(self, p: torch.Tensor) -> torch.Tensor:
        return self._view_fns[self.index[id(p)]](self.grad)

    # ---------------------------------------------------------------- updates
    def add_listener(self, fn) -> None:
        """``fn()`` runs (on the current stream) after every optimizer update of the arena."""
        self._listeners.append(fn)

    def after_step(self, mirror_written: bool = False) -> None:
        self.version += 1
        self.module._iit_weights_version = getattr(self.module, "_iit_weights_version", 0) + 1
        if mirror_written:
            self.mirror_version = self.module._iit_weights_version
        else:
            self.refresh_shadow()
        for fn in self._listeners:
            fn()

    # ---------------------------------------------------------------- bf16 mirror
    def ensure_shadow(self) -> torch.Tensor:
        if self.shadow is None:
            self.shadow = torch.empty(self.numel, dtype=torch.bfloat16, device=self.data.device)
            self.refresh_shadow()
        return self.shadow

    def refresh_shadow(self) -> None:
        if self.shadow is not None:
            self.shadow.copy_(self.data)
            self.mirror_version = getattr(self.module, "_iit_weights_version", 0)

    def shadow_view(self, p: torch.Tensor) -> torch.Tensor:
        """bf16 mirror of ``p`` with ``p``'s shape and strides."""
        sh = self.ensure_shadow()
        return sh.as_strided(p.shape, p.stride(), self.offset_of(p))

    # ---------------------------------------------------------------- buckets
    def buckets(self, bucket_bytes: int) -> List[Tuple[int, int]]:
        """Contiguous gradient slices of ~``bucket_bytes`` in reverse arena order
        (≈ the order backward produces them), for overlapped all-reduce.  Bucket
        edges fall on slot boundaries, so a grouped slot is never split."""
        per = max(_ALIGN, bucket_bytes // 4)
        out = []
        end = self.numel
        while end > 0:
            start = max(0, end - per)
            for o, n in self.slots:
                if o <= start < o + _align(n):
                    start = o
                    break
            if start >= end:  # a single slot larger than the bucket size
                for o, n in self.slots:
                    if o < end <= o + _align(n):
                        start = o
                        break
            out.append((start, end))
            end = start
        return out
