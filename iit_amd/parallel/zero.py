"""Optimizer-state sharding (ZeRO stage 1) for data parallelism over RCCL/xGMI.

Replicated data parallelism (:class:`iit_amd.parallel.ddp.GradReducer` + :class:`iit_amd.ops.optim.FusedAdam`)
keeps, on every rank, the fp32 master weights, the fp32 gradient and both Adam moments of the whole model, and runs
clip + Adam over all of it: for Llama-3-8B that is 32 GB of moments per moment and a 126 ms optimizer pass per step
on every GPU (``profiles/llama3_8b_kernel_stats_v3.txt``).  With ``ShardedFusedAdam`` each optimizer phase is

  1. **reduce-scatter** per gradient bucket (in the staged schedule: per backward stage, overlapped with the next
     stage's backward exactly like the all-reduce it replaces): bucket ``[s, e)`` is split into ``N`` equal pieces of
     ``P = ceil((e - s) / N)`` (rounded to 64 elements); rank ``r`` receives the averaged gradient of piece ``r`` in
     its shard buffer;
  2. **sharded global-norm clip**: every rank sums g^2 over its pieces (the fused sumsq kernel over a shard span
     table), one 4-byte all-reduce gives the global norm, and the clip coefficient is formed on device;
  3. **sharded Adam**: the fused kernel updates only this rank's pieces -- master weights and bf16 mirror at their
     arena offsets, gradient and moments at their shard offsets -- so moments take ``8/N`` bytes per parameter
     instead of 8 and the pass is ``N`` times shorter;
  4. **all-gather** of the updated fp32 pieces per bucket back into every rank's arena, then the bf16 mirror of the
     bucket is re-derived locally (a cast pass), so the next phase's forward reads identical weights on every rank.
     On RCCL the gather is in place (each rank's piece is already at its slot of the bucket: no send copy).  With
     a model that declares ``supports_param_gate`` (the HookedTransformer family) the eager step does not wait:
     every bucket's gather is issued asynchronously, and the next forward calls the installed gate before the
     embedding and before each block, which makes the compute stream wait for (and re-derives the mirror of) only
     the buckets holding that block's weights -- the gathers of later blocks' weights run on the RCCL stream under
     the earlier blocks' kernels (:meth:`ShardedFusedAdam.attach_gates`).

Bytes on xGMI per optimizer phase equal a ring all-reduce of the gradient (reduce-scatter + all-gather of the same
size: ``2 (N-1)/N * 4 B`` per parameter); what changes is memory (moments ``/N``) and optimizer time (``/N``).
``bf16`` wire (``IIT_DP_GRAD_DTYPE=bf16``) halves the reduce-scatter bytes as for the all-reduce.

Semantics equal the replicated optimizer up to the summation order of the gradient average: every rank applies the
Adam math of ``torch.optim.Adam`` to the averaged, globally clipped gradient (``/root/reference/iit/model_pairs/
iit_behavior_model_pair.py:60-64``: zero_grad -> backward -> clip -> step).  gloo (CPU tests) has no reduce-scatter:
there the bucket is all-reduced and each rank keeps its piece.

Per-rank memory model (fp32 master + fp32 gradient + bf16 mirror replicated, moments sharded):
``P * (4 + 4 + 2) + 8 P / N`` bytes for ``P`` parameters -- Llama-3-8B at N = 8: 80.3 GB + 8.0 GB = 88.3 GB
(replicated: 144.5 GB), see :func:`memory_model`.
"""
from __future__ import annotations

from typing import Dict, List, Optional, Sequence, Tuple

import torch
import torch.distributed as dist

from ..engine.flat import FlatParams, make_span_tensor
from ..ops.optim import FusedAdam
from . import dist as pdist

_ALIGN = 64


def _piece(n: int, world: int) -> int:
    p = (n + world - 1) // world
    return (p + _ALIGN - 1) // _ALIGN * _ALIGN


class ShardPlan:
    """Which arena elements this rank owns: piece ``rank`` of every bucket ``[s, e)`` (arena order of buckets is
    irrelevant; the local shard buffers concatenate this rank's pieces bucket by bucket)."""

    def __init__(self, buckets: Sequence[Tuple[int, int]], world: int, rank: int):
        self.world, self.rank = world, rank
        self.buckets: List[Tuple[int, int]] = [(int(s), int(e)) for s, e in buckets]
        self.piece: List[int] = []     # piece length per bucket (same on every rank)
        self.local: List[int] = []     # offset of this rank's piece in the shard buffers
        self.own: List[Tuple[int, int]] = []  # owned arena range per bucket (may be empty / shorter than the piece)
        off = 0
        for s, e in self.buckets:
            p = _piece(e - s, world)
            a = min(e, s + rank * p)
            b = min(e, s + (rank + 1) * p)
            self.piece.append(p)
            self.local.append(off)
            self.own.append((a, b))
            off += p
        self.numel = off  # shard buffer length (elements)
        self.index: Dict[Tuple[int, int], int] = {bk: i for i, bk in enumerate(self.buckets)}

    def live_pieces(self, gaps: Sequence[Tuple[int, int]] = ()) -> List[Tuple[int, int, int]]:
        """(arena start, arena end, shard start) of the owned elements outside ``gaps`` (sorted arena ranges the
        optimizer may skip: embedding rows no training token reaches, ``FlatParams.inactive_ranges``)."""
        out = []
        for (a, b), loc in zip(self.own, self.local):
            cur = a
            for g0, g1 in gaps:
                if g1 <= cur or g0 >= b:
                    continue
                if g0 > cur:
                    out.append((cur, g0, loc + cur - a))
                cur = max(cur, g1)
            if cur < b:
                out.append((cur, b, loc + cur - a))
        return out

    def spans(self, max_len4: int = 1024, gaps: Sequence[Tuple[int, int]] = ()) -> List[Tuple[int, int, int]]:
        """Optimizer span records (arena start4, shard start4, len4) over the owned pieces (minus ``gaps``)."""
        out = []
        for a, b, loc in self.live_pieces(gaps):
            pos, n = a // 4, (b - a) // 4
            lpos = loc // 4
            while n > 0:
                ln = min(max_len4, n)
                out.append((pos, lpos, ln))
                pos += ln
                lpos += ln
                n -= ln
        return out


class ShardedFusedAdam(FusedAdam):
    """:class:`FusedAdam` with optimizer state sharded over the data-parallel ranks (see the module docstring).

    The gradient reducer (``GradReducer(..., shard=optimizer)``) fills :attr:`shard_grad` by reduce-scatter; ``step``
    clips with the global norm, updates this rank's pieces and all-gathers them.  ``step`` issues collectives, so a
    graph-captured phase runs it eagerly (``sharded = True``)."""

    sharded = True

    def __init__(self, flat: FlatParams, buckets: Sequence[Tuple[int, int]], lr: float = 1e-3, betas=(0.9, 0.999),
                 eps: float = 1e-8, weight_decay: float = 0.0, use_hip: Optional[bool] = None, nan_guard: bool = True):
        super().__init__(flat, lr=lr, betas=betas, eps=eps, weight_decay=weight_decay, use_hip=use_hip,
                         nan_guard=nan_guard, alloc_moments=False)
        dev = flat.data.device
        self._total = torch.zeros(1, dtype=torch.float32, device=dev)
        self._part = torch.zeros(1024, dtype=torch.float32, device=dev)
        self.plan = None
        self.set_buckets(buckets)

    def set_buckets(self, buckets: Sequence[Tuple[int, int]]) -> None:
        """(Re)build the shard plan over the reducer's gradient buckets (the staged schedule re-buckets the arena
        once, before training).  The moments live in the plan's layout, so this is only allowed before the first
        step (or with an unchanged layout)."""
        plan = ShardPlan(buckets, pdist.world_size(), pdist.rank())
        if self.plan is not None and plan.buckets == self.plan.buckets:
            return
        if self.plan is not None and self.step_count:
            raise RuntimeError("optimizer-state sharding: the gradient buckets changed after the first step")
        dev = self.flat.data.device
        self.alias = plan.world == 1
        if self.alias:
            # one rank (the IIT_DP_FORCE_REDUCER rehearsal): the rank's piece of every bucket is the whole bucket, so
            # the shard layout IS the arena layout -- the gradient arena serves as the shard gradient (no
            # reduce-scatter copy: the reducer issues nothing at world 1, as for the replicated all-reduce)
            plan.local = [s for s, _ in plan.buckets]
            plan.own = list(plan.buckets)
            plan.numel = self.flat.numel
        self.plan = plan
        # shard-sized moments and gradient (the replicated optimizer's arena-sized ones are dropped)
        self.exp_avg = torch.zeros(plan.numel, dtype=torch.float32, device=dev)
        self.exp_avg_sq = torch.zeros(plan.numel, dtype=torch.float32, device=dev)
        self.shard_grad = self.flat.grad if self.alias else torch.zeros(plan.numel, dtype=torch.float32, device=dev)
        self._gather_bufs: Dict[tuple, torch.Tensor] = {}
        self._pending: Dict[int, object] = {}  # bucket -> in-flight all-gather work (deferred gather)
        self._gate_groups = None               # gate key (None = outside every block, int = block) -> buckets
        if getattr(self, "_gated_module", None) is not None:  # re-bucketed (staged schedule): re-map the gates
            self.attach_gates(self._gated_module)
        self._spans_version = None
        self._retired_spans = []
        self._build_spans()

    def _build_spans(self) -> None:
        """Span table of the owned pieces minus the rows the training data cannot reach (``restrict_sparse_rows``):
        with zero gradient and zero moments their Adam update is the identity, as in the replicated optimizer.
        Rebuilt when the restriction changes (outside graph capture); skipping is refused if a skipped range holds
        non-zero moments (a restriction declared after unrestricted steps)."""
        flat = self.flat
        gaps = flat.inactive_ranges()
        if gaps:
            skipped = [(loc + max(a, g0) - a, loc + min(b, g1) - a)
                       for a, b, loc in self.plan.live_pieces(()) for g0, g1 in gaps if g0 < b and g1 > a]
            # the same guard as the replicated optimizer (FusedAdam._validate_restriction): the skipped rows' update
            # is the identity only without weight decay and with zero gradient and zero moments there
            wd = self.param_groups[0].get("weight_decay", 0.0) if getattr(self, "param_groups", None) else 0.0
            if wd != 0 or any(bool(t[x:y].any()) for x, y in skipped
                              for t in (self.exp_avg, self.exp_avg_sq, self.shard_grad)):
                gaps = []
        spans = self.plan.spans(gaps=gaps)
        if getattr(self, "_spans", None) is not None:
            self._retired_spans.append(self._spans)  # a captured graph may still read the old table's address
        self._spans = make_span_tensor(spans, flat.data.device)
        self._nspans = len(spans)
        self._spans_version = flat.restrict_version

    def _sync_spans(self) -> None:
        if self._spans_version != self.flat.restrict_version and not (
                torch.cuda.is_available() and torch.cuda.is_current_stream_capturing()):
            self._build_spans()

    # ------------------------------------------------------------------ gradient side (called by the reducer)
    def shard_view(self, bucket: int) -> torch.Tensor:
        p = self.plan.piece[bucket]
        loc = self.plan.local[bucket]
        return self.shard_grad[loc:loc + p]

    def padded_input(self, bucket: int, src: torch.Tensor) -> torch.Tensor:
        """``src`` (bucket ``[s, e)`` of the gradient arena) padded with zeros to ``N * piece`` elements."""
        s, e = self.plan.buckets[bucket]
        full = self.plan.piece[bucket] * self.plan.world
        if full == e - s:
            return src
        buf = self._gather_bufs.get(("in", bucket))
        if buf is None or buf.dtype != src.dtype:
            buf = self._gather_bufs[("in", bucket)] = torch.zeros(full, dtype=src.dtype, device=src.device)
        buf[:e - s].copy_(src)
        return buf

    # ------------------------------------------------------------------ optimizer
    def step_parts(self, clip_norm: Optional[float] = None):
        """The step as ``[(capturable, fn), ...]`` for a graph-replayed phase (the whole
        sharded optimizer ran eagerly): the device work -- sharded sum of squares, the Adam pass, the mirror
        refresh of the pieces other ranks own -- is capturable; the collectives between them (the 4-byte norm
        all-reduce, the all-gather of the updated pieces) stay eager, so every rank still issues the identical
        RCCL sequence.  Runs in order exactly what :meth:`step` runs.  None on the torch (non-HIP) path."""
        if self._hip is None:
            return None
        from ..ops import hip_kernels as K
        need_norm = bool(clip_norm) or self.nan_guard
        world = pdist.world_size()
        g = self.param_groups[0]

        def host_books():  # eager, first: the host-side counters / hyper-parameters of this step
            self.wait_gathers()
            self.step_count += 1
            self.sync_hyper()
            self._sync_spans()

        def norm_part():
            K.sumsq_spans(self.shard_grad, self._spans, self._nspans, self._part, self._step_dev, need_norm)
            if need_norm:
                torch.sum(self._part, dim=0, keepdim=True, out=self._total)

        def norm_reduce():
            dist.all_reduce(self._total, op=dist.ReduceOp.SUM)

        def adam_part():
            (b1, b2) = g["betas"]
            K.adam_spans(self.flat, self.shard_grad, self.exp_avg, self.exp_avg_sq, self._spans, self._nspans,
                         self._total, self._step_dev, lr=g["lr"], b1=b1, b2=b2, eps=g["eps"], wd=g["weight_decay"],
                         clip_norm=clip_norm, skipped=self._skipped_dev if self.nan_guard else None,
                         hyper=self._hyper_dev)

        parts = [(False, host_books), (True, norm_part)]
        if need_norm and world > 1:
            parts.append((False, norm_reduce))
        parts.append((True, adam_part))
        if world > 1:
            parts.append((False, lambda: self._all_gather(mirror=False)))
            parts.append((True, self._refresh_foreign_mirror))
        parts.append((False, lambda: self.flat.after_step(mirror_written=self.flat.shadow is not None)))
        return parts

    def _refresh_foreign_mirror(self) -> None:
        """bf16 mirror of the pieces other ranks updated (the owned piece's mirror was written by the Adam pass)."""
        flat = self.flat
        if flat.shadow is None:
            return
        for (s, e), (a, b) in zip(self.plan.buckets, self.plan.own):
            foreign = [(s, a), (b, e)] if b > a else [(s, e)]
            for lo, hi in foreign:
                if hi > lo:
                    flat.shadow[lo:hi].copy_(flat.data[lo:hi])

    @torch.no_grad()
    def step(self, closure=None, clip_norm: Optional[float] = None):
        if closure is not None:
            with torch.enable_grad():
                closure()
        self.wait_gathers()  # (the previous step's deferred gathers, if a forward did not consume them all)
        group = self.param_groups[0]
        lr, (b1, b2), eps, wd = group["lr"], group["betas"], group["eps"], group["weight_decay"]
        self.step_count += 1
        self.sync_hyper()
        self._sync_spans()
        need_norm = bool(clip_norm) or self.nan_guard
        if self._hip is not None:
            from ..ops import hip_kernels as K
            K.sumsq_spans(self.shard_grad, self._spans, self._nspans, self._part, self._step_dev, need_norm)
            if need_norm:
                torch.sum(self._part, dim=0, keepdim=True, out=self._total)
                if pdist.world_size() > 1:
                    dist.all_reduce(self._total, op=dist.ReduceOp.SUM)
            K.adam_spans(self.flat, self.shard_grad, self.exp_avg, self.exp_avg_sq, self._spans, self._nspans,
                         self._total, self._step_dev, lr=lr, b1=b1, b2=b2, eps=eps, wd=wd, clip_norm=clip_norm,
                         skipped=self._skipped_dev if self.nan_guard else None, hyper=self._hyper_dev)
        else:
            self._step_torch(clip_norm, lr, b1, b2, eps, wd, need_norm)
        self._all_gather(defer=self._gate_groups is not None)

    def _owned_views(self):
        """(arena view, shard view) per bucket for this rank's owned elements."""
        for (a, b), loc in zip(self.plan.own, self.plan.local):
            if b > a:
                yield self.flat.data[a:b], loc, b - a

    def _step_torch(self, clip_norm, lr, b1, b2, eps, wd, need_norm):
        g = self.shard_grad
        if need_norm:
            tot = (g.double() ** 2).sum().reshape(1)
            if pdist.world_size() > 1:
                dist.all_reduce(tot, op=dist.ReduceOp.SUM)
            norm = tot.sqrt().float()
            if self.nan_guard and not bool(torch.isfinite(norm)):
                self._skipped_dev += 1
                self.step_count -= 1
                return
        self._step_dev += 1
        t = int(self._step_dev.item())
        bc1 = 1.0 - b1 ** t
        bc2 = 1.0 - b2 ** t
        coef = 1.0
        if clip_norm:
            coef = float(torch.clamp(clip_norm / (norm + 1e-6), max=1.0))
        for p, loc, n in self._owned_views():
            gg = g[loc:loc + n] * coef
            if wd:
                gg = gg.add(p, alpha=wd)
            m = self.exp_avg[loc:loc + n]
            v = self.exp_avg_sq[loc:loc + n]
            m.mul_(b1).add_(gg, alpha=1 - b1)
            v.mul_(b2).addcmul_(gg, gg, value=1 - b2)
            denom = (v.sqrt() / (bc2 ** 0.5)).add_(eps)
            p.addcdiv_(m, denom, value=-lr / bc1)

    def _all_gather(self, mirror: bool = True, defer: bool = False) -> None:
        """Every rank's updated pieces back into every arena, one asynchronous collective per bucket; each bucket is
        then finished (:meth:`_finish`: the compute stream waits for its gather, the padded tail is copied back, the
        bf16 mirror of its foreign pieces is re-derived if ``mirror``) -- right away, or with ``defer`` when the
        next forward's gate first needs it (or at :meth:`wait_gathers`).  ``step_parts`` gathers with
        ``mirror=False``: its captured part refreshes the foreign mirror."""
        flat = self.flat
        world = self.plan.world
        if world > 1:
            nccl = dist.get_backend() == "nccl"
            import os
            poison = os.environ.get("IIT_ZERO_POISON") == "1"
            for bi, (s, e) in enumerate(self.plan.buckets):
                p = self.plan.piece[bi]
                a, b = self.plan.own[bi]
                if poison:
                    # debugging aid: the foreign pieces (master and mirror) are NaN until this bucket is finished, and
                    # its gather is only issued then (below) -- a reader that bypasses the gates always reads NaN and
                    # turns the run's losses to NaN
                    for lo, hi in ([(s, a), (b, e)] if b > a else [(s, e)]):
                        if hi > lo:
                            flat.data[lo:hi].fill_(float("nan"))
                            if flat.shadow is not None:
                                flat.shadow[lo:hi].fill_(float("nan"))
                full = p * world
                exact = full == e - s
                out = flat.data[s:e] if exact else self._gather_bufs.get(("out", bi))
                if out is None:
                    out = self._gather_bufs[("out", bi)] = torch.zeros(full, dtype=torch.float32,
                                                                     device=flat.data.device)
                piece = out[self.plan.rank * p:(self.plan.rank + 1) * p]
                if not exact:
                    piece.zero_()
                    if b > a:
                        piece[:b - a].copy_(flat.data[a:b])
                if nccl:
                    # in place: the input is this rank's slot of the output (RCCL's in-place all-gather)
                    issue = (lambda out=out, piece=piece: dist.all_gather_into_tensor(out, piece, async_op=True))
                else:  # gloo: list form, and its input must not alias the output list
                    issue = (lambda out=out, piece=piece, p=p:
                             dist.all_gather(list(out.split(p)), piece.clone(), async_op=True))
                self._pending[bi] = (issue if poison else issue(), mirror)
        elif mirror and flat.shadow is not None:
            for bi in range(len(self.plan.buckets)):
                self._pending[bi] = (None, mirror)
        if not defer:
            self.wait_gathers()
        if mirror:
            flat.after_step(mirror_written=flat.shadow is not None)

    def _finish(self, bi: int) -> None:
        item = self._pending.get(bi)
        if item is None:
            return
        if torch.cuda.is_available() and torch.cuda.is_current_stream_capturing():
            # under stream capture the wait, the tail copy and the mirror refresh would only be RECORDED into the
            # graph, not run, while the bucket left the pending set: a later join would find nothing to wait for and
            # the first replay could race the in-flight gather.  Captures are preceded by a join
            # (engine/graphs.py), so a pending bucket here is a caller bug -- it stays pending for the eager join.
            return
        work, mirror = item
        flat = self.flat
        s, e = self.plan.buckets[bi]
        if work is not None:
            if callable(work):  # (IIT_ZERO_POISON: issued at finish)
                work = work()
                self._pending[bi] = (work, mirror)
            work.wait()  # RCCL: the current stream waits for the collective (no host block)
        # popped only once the wait succeeded: a wait that raises leaves the bucket pending (never a stale mirror)
        self._pending.pop(bi, None)
        if work is not None:
            if self.plan.piece[bi] * self.plan.world != e - s:
                flat.data[s:e].copy_(self._gather_bufs[("out", bi)][:e - s])
        if mirror and flat.shadow is not None:
            if self._hip is None:  # the torch path writes no mirror: refresh the whole bucket
                flat.shadow[s:e].copy_(flat.data[s:e])
            else:  # the fused pass wrote the owned piece's mirror
                a, b = self.plan.own[bi]
                for lo, hi in ([(s, a), (b, e)] if b > a else [(s, e)]):
                    if hi > lo:
                        flat.shadow[lo:hi].copy_(flat.data[lo:hi])

    def wait_gathers(self) -> None:
        """Finish every in-flight bucket gather (checkpointing, the next step, a graph replay, a non-gated read)."""
        for bi in sorted(self._pending):
            self._finish(bi)

    def attach_gates(self, module: torch.nn.Module) -> bool:
        """Overlap the deferred all-gather with the next forward (see the module docstring).  ``module`` declares
        ``supports_param_gate`` and calls ``module._param_gate(key)`` before it reads the weights of block ``key``
        (``None``: the weights outside ``module.blocks`` -- embeddings, final norm, unembedding -- read first);
        ``module._param_join`` finishes everything (readers that bypass the gates).  Returns whether installed."""
        if not getattr(module, "supports_param_gate", False) or not hasattr(module, "blocks"):
            return False
        flat = self.flat

        def buckets_of(params):
            out = set()
            for p in params:
                if not flat.owns(p):
                    continue
                o = flat.offset_of(p)
                n = p.numel()
                for bi, (s, e) in enumerate(self.plan.buckets):
                    if s < o + n and o < e:
                        out.add(bi)
            return out

        in_blocks = set()
        groups = {}
        for li, blk in enumerate(module.blocks):
            ps = list(blk.parameters())
            in_blocks.update(id(p) for p in ps)
            groups[li] = sorted(buckets_of(ps))
        groups[None] = sorted(buckets_of([p for p in module.parameters() if id(p) not in in_blocks]))
        self._gate_groups = groups
        self._gated_module = module

        def gate(key):
            if self._pending and not (torch.cuda.is_available() and torch.cuda.is_current_stream_capturing()):
                for bi in self._gate_groups.get(key, ()):
                    self._finish(bi)

        module.__dict__["_param_gate"] = gate
        module.__dict__["_param_join"] = self.wait_gathers
        return True

    # ------------------------------------------------------------------ checkpointing
    def state_dict(self):
        self.wait_gathers()
        sd = super().state_dict()
        sd["shard"] = {"world": self.plan.world, "rank": self.plan.rank, "buckets": self.plan.buckets}
        return sd

    def load_state_dict(self, sd):
        self.wait_gathers()
        shard = sd.get("shard")
        if shard is None or shard["world"] != self.plan.world or [tuple(b) for b in shard["buckets"]] != \
                self.plan.buckets:
            raise ValueError("sharded optimizer state was saved with another data-parallel layout")
        if int(shard.get("rank", -1)) != self.plan.rank:
            # same shard length on every rank: a wrong file would load silently with another rank's moments
            raise ValueError(f"sharded optimizer state of rank {shard.get('rank')} offered to rank {self.plan.rank}")
        super().load_state_dict(sd)


def memory_model(n_params: int, world: int, mirror: bool = True) -> Dict[str, float]:
    """Per-rank bytes of the training state for ``n_params`` parameters (activations excluded): replicated
    data parallelism vs optimizer-state sharding."""
    master, grad, mom = 4 * n_params, 4 * n_params, 8 * n_params
    shadow = 2 * n_params if mirror else 0
    return {"replicated_GB": (master + grad + mom + shadow) / 1e9,
            "sharded_GB": (master + grad + shadow + mom / world) / 1e9,
            "moments_per_rank_GB": mom / world / 1e9}
