"""Bucketed, backward-overlapped gradient all-reduce over RCCL/xGMI.

Each ``step_on_loss`` of a model pair does ``backward -> all-reduce -> clip ->
Adam`` (3x per batch for Strict/IOI pairs).  ``GradReducer``
splits the flat gradient arena (:class:`iit_amd.engine.flat.FlatParams`) into
contiguous buckets in reverse parameter order.  With ``overlap=True`` a
post-accumulate-grad hook marks each parameter ready; a bucket is all-reduced
(async, on RCCL's stream) the moment its last parameter's gradient lands, so
communication of late layers overlaps the backward of early layers.  Buckets
never completed by autograd (dead compute skipped by the engine) are flushed in
``finish()``.  Reduction is in place on the arena (no pack/unpack copies), as an
average (``ReduceOp.AVG`` on RCCL, SUM + scale on gloo).

A loss may span several grad-enabled forwards (``use_single_loss``: the IIT, strict and behaviour forwards feed one
backward), and then every weight gradient is written once *per forward*: the first report of a parameter is not
its final value.  A forward hook on the LL module counts the grad-enabled forwards since the last backward; when
there was more than one, ``start`` turns the per-parameter launches off for that backward and ``finish`` reduces
every bucket after autograd is done (correct for any number of writes; only the overlap is lost).

Bucket size default 64 MiB: per xGMI ring link (~150 GB/s) that is ~0.4 ms per
bucket, large enough to amortise RCCL launch latency, small enough that the last
bucket's exposed tail is short.

Wire precision: bf16 on RCCL by default, fp32 on gloo.  With the bf16 wire each bucket is cast to a bf16 staging
buffer, all-reduced there and cast back into the fp32 arena: half the bytes on xGMI (GPT-2-small: 250 instead of
500 MB per optimizer phase, three phases per step; Llama-3-8B: 16 instead of 32 GB).  The decision is the
8-rank summation test tests/test_wire_dtype.py: the wire's rounding moves the averaged gradient by 0.3-0.45 %
(one bf16 rounding), never more than the single-GPU step's own bf16 compute error (1.3-2.4 % at GPT-2-small scale),
so the DP step stays within the precision the single-GPU step already has.  ``IIT_DP_GRAD_DTYPE=fp32`` (or
``GradReducer(..., wire_dtype=torch.float32)`` / ``training_args["grad_wire_dtype"] = "fp32"``) keeps the exact-sum
wire: the data-parallel step then equals the single-GPU step up to summation order.  gloo (CPU tests) keeps fp32 so
the multi-process tests compare against single-process runs at fp32 sums.
"""
from __future__ import annotations

import os
from typing import List, Optional

import torch
import torch.distributed as dist

from ..engine import grad_hooks
from ..engine.flat import FlatParams
from . import dist as pdist


def computes_bf16(module: Optional[torch.nn.Module], flat: FlatParams) -> bool:
    """Whether the model's forward / backward run in bf16: a bf16 weight mirror in the arena (the fused HIP backend,
    the PVR conv mirror), a bf16 ``cfg.dtype``, or bf16 autocast active."""
    if getattr(flat, "shadow", None) is not None:
        return True
    cfg = getattr(module, "cfg", None) if module is not None else None
    dt = cfg.get("dtype") if isinstance(cfg, dict) else getattr(cfg, "dtype", None)
    if dt == torch.bfloat16:
        return True
    return bool(torch.cuda.is_available() and torch.is_autocast_enabled("cuda")
                and torch.get_autocast_dtype("cuda") == torch.bfloat16)


class GradReducer:
    def __init__(self, flat: FlatParams, bucket_mb: float = 64.0, overlap: bool = True,
                 wire_dtype: Optional[torch.dtype] = None, module: Optional[torch.nn.Module] = None):
        self.flat = flat
        self.world = pdist.world_size()
        self.enabled = self.world > 1 or pdist.force_reducer()
        self._module = module
        self._wire_auto = False
        if wire_dtype is None:
            env = os.environ.get("IIT_DP_GRAD_DTYPE", "")
            if env in ("bf16", "fp32"):
                wire_dtype = torch.bfloat16 if env == "bf16" else torch.float32
            else:
                # default: bf16 on RCCL only for a model that computes in bf16 (its gradients already carry bf16
                # rounding: tests/test_wire_dtype.py), fp32 for fp32 models and on gloo -- decided at
                # the first launch, when a lazily created bf16 mirror exists
                nccl = self.enabled and dist.is_initialized() and dist.get_backend() == "nccl"
                self._wire_auto = nccl
                wire_dtype = torch.float32
        self.wire_dtype = wire_dtype if wire_dtype != torch.float32 else None
        self.overlap = overlap and self.enabled
        self._bucket_bytes = int(bucket_mb * (1 << 20))
        self.buckets = flat.buckets(self._bucket_bytes)
        self._use_avg = self.enabled and dist.get_backend() == "nccl"
        # parameter -> bucket id; bucket -> number of params
        self._param_bucket: List[int] = []
        self._bucket_count = [0] * len(self.buckets)
        for o, n in flat.offsets:
            for bi, (s, e) in enumerate(self.buckets):
                if s <= o < e:
                    self._param_bucket.append(bi)
                    self._bucket_count[bi] += 1
                    break
        self._pending = list(self._bucket_count)
        self._launched = [False] * len(self.buckets)
        self._ready = [False] * len(flat.params)
        self._works = []
        self._hooks = []
        self._listener = None
        self._subsets = {}
        self.shard = None  # ShardedFusedAdam (ZeRO-1): buckets are reduce-scattered into its shard buffers
        self.paused = False  # True while a graph-captured backward runs (reduction happens after it)
        self.deferred = False  # this backward: no per-parameter launches (several forwards wrote each gradient)
        self._grad_forwards = 0
        self._fwd_hook = None
        if module is not None:
            self._fwd_hook = module.register_forward_pre_hook(self._count_forward)
        if self.overlap:
            for i, p in enumerate(flat.params):
                self._hooks.append(p.register_post_accumulate_grad_hook(self._make_hook(i)))
            # gradients the fused HIP kernels write directly (no autograd accumulation) report here
            index = {id(p): i for i, p in enumerate(flat.params)}
            self._listener = grad_hooks.add_listener(
                lambda p, _index=index: self._mark_ready(_index[id(p)]) if id(p) in _index else None)

    def _count_forward(self, _module, _args) -> None:
        if torch.is_grad_enabled():
            self._grad_forwards += 1

    def _mark_ready(self, i: int) -> None:
        # with one grad-enabled forward each parameter's gradient is final when first reported within a backward
        # (the engine writes every weight gradient exactly once per backward pass); repeats are ignored.  With
        # several forwards behind the loss the reports are not final: ``deferred`` leaves everything to finish()
        if self.paused or self.deferred or self._ready[i]:
            return
        self._ready[i] = True
        b = self._param_bucket[i]
        self._pending[b] -= 1
        if self._pending[b] == 0:
            self._launch(b)

    def _make_hook(self, i: int):
        def hook(_p, _i=i):
            self._mark_ready(_i)
        return hook

    def attach_shard(self, optimizer) -> None:
        """Optimizer-state sharding (iit_amd.parallel.zero): reduce-scatter every bucket into ``optimizer``'s shard
        buffers instead of all-reducing it in place; the optimizer all-gathers the updated weights."""
        self.shard = optimizer
        optimizer.set_buckets(self.buckets)

    def _resolve_wire(self) -> None:
        if not self._wire_auto:
            return
        self._wire_auto = False
        if computes_bf16(self._module, self.flat):
            self.wire_dtype = torch.bfloat16
        if pdist.is_main():
            print(f"[iit dp] gradient wire dtype: {'bf16' if self.wire_dtype is not None else 'fp32'} "
                  f"(IIT_DP_GRAD_DTYPE / training_args['grad_wire_dtype'] override)", flush=True)

    def _launch(self, b: int):
        if self._launched[b]:
            return
        self._launched[b] = True
        self._resolve_wire()
        s, e = self.buckets[b]
        if self.shard is not None:
            self._launch_reduce_scatter(b, s, e)
            return
        self._launch_span(s, e)

    def _launch_reduce_scatter(self, b: int, s: int, e: int) -> None:
        """Bucket ``b`` -> the averaged gradient of this rank's piece in the shard buffer (async)."""
        sh = self.shard
        if getattr(sh, "alias", False):
            return  # one rank: the shard gradient IS the arena gradient (ShardedFusedAdam.set_buckets)
        world, rank, piece = sh.plan.world, sh.plan.rank, sh.plan.piece[b]
        out = sh.shard_view(b)
        src = self.flat.grad[s:e]
        if self.wire_dtype is not None:
            src = src.to(self.wire_dtype)
        inp = sh.padded_input(b, src)
        if self._use_avg:  # RCCL: reduce-scatter with AVG
            dst = out if self.wire_dtype is None else torch.empty(piece, dtype=self.wire_dtype, device=out.device)
            work = dist.reduce_scatter_tensor(dst, inp, op=dist.ReduceOp.AVG, async_op=True)
            post = None if dst is out else (lambda d=dst, o=out: o.copy_(d))
        else:  # gloo (no reduce-scatter): all-reduce the padded bucket, keep this rank's piece
            if inp is src:
                inp = inp.clone()
            work = dist.all_reduce(inp, op=dist.ReduceOp.SUM, async_op=True)
            post = lambda i=inp, o=out: o.copy_(i[rank * piece:(rank + 1) * piece]).div_(world)  # noqa: E731
        self._works.append((work, None, None, None, post))

    def _launch_span(self, s: int, e: int) -> None:
        """Async all-reduce of arena elements [s, e): rows-restricted parameters compactly, the rest in place."""
        if self.world == 1:
            # a one-rank group (IIT_DP_FORCE_REDUCER rehearsals of the DP schedule): the average over one rank is
            # the identity, so nothing is issued -- RCCL would run a full read + scale + write pass of the range
            # (oneRankReduce, 3.1 ms/step in profiles/dp_schedule_1gpu_breakdown_v4.txt) that no real world-N run
            # has (there the ring reduction replaces it)
            return
        op = dist.ReduceOp.AVG if self._use_avg else dist.ReduceOp.SUM
        pieces, cur = [], s
        subsets = self.__dict__.get("_subsets_sorted")
        if subsets is None or subsets[0] != len(self._subsets):
            subsets = self._subsets_sorted = (len(self._subsets),
                                              sorted(self._subsets.items(), key=lambda kv: kv[1][0]))
        for i, (o, n, width, rows) in subsets[1]:
            if o >= s and o + n <= e:
                if o > cur:
                    pieces.append(("dense", cur, o))
                pieces.append(("rows", o, n, width, rows))
                cur = o + n
        if cur < e:
            pieces.append(("dense", cur, e))
        for pc in pieces:
            if pc[0] == "dense":
                dst = self.flat.grad[pc[1]:pc[2]]
                scatter = None
            else:
                _, o, n, width, rows = pc
                full = self.flat.grad[o:o + n].view(-1, width)
                dst = full.index_select(0, rows)
                scatter = (full, rows)
            buf = dst if self.wire_dtype is None else dst.to(self.wire_dtype)
            home = None if self.wire_dtype is None else dst  # fp32 destination of the bf16 wire buffer
            self._works.append((dist.all_reduce(buf, op=op, async_op=True), buf, scatter, home, None))

    def launch_range(self, s: int, e: int) -> None:
        """Start reducing every bucket inside arena range [s, e) now (async; ``finish`` waits).  The staged
        graph-captured backward calls this after each backward segment so the segment's gradients travel
        while the next segment computes.  Ranges must fall on bucket boundaries of :meth:`segment_buckets`."""
        if not self.enabled:
            return
        for b, (bs, be) in enumerate(self.buckets):
            if bs >= s and be <= e:
                self._launch(b)

    def segment_buckets(self, cuts, whole_segments: bool = True) -> None:
        """Re-bucket so every arena offset in ``cuts`` is a bucket edge (segment ranges reduce exactly).

        ``whole_segments`` (the staged backward's default): one bucket per segment.  Every bucket of a segment is
        launched at the same moment (``launch_range`` after the segment's graph), so splitting a segment only adds
        collective calls -- host time between the segment graphs -- without adding overlap; one large all-reduce
        per segment is also RCCL's most efficient message size on xGMI."""
        edges = sorted({0, self.flat.numel, *[int(c) for c in cuts]})
        per = max(64, int(self._bucket_bytes) // 4)
        out = []
        for a, b in zip(edges[:-1], edges[1:]):
            if whole_segments:
                out.append((a, b))
                continue
            pieces, end = [], b  # slot-aligned pieces of <= bucket size, back to front
            while end > a:
                start = max(a, end - per)
                for o, n in self.flat.slots:
                    if o <= start < o + ((n + 63) // 64) * 64:
                        start = max(a, o)
                        break
                if start >= end:
                    start = a
                pieces.append((start, end))
                end = start
            out.extend(pieces)
        out.sort(key=lambda r: -r[0])  # reverse arena order, like ``FlatParams.buckets``
        self.buckets = out
        if self.shard is not None:
            self.shard.set_buckets(self.buckets)
        self._param_bucket = []
        self._bucket_count = [0] * len(self.buckets)
        for o, n in self.flat.offsets:
            for bi, (s, e) in enumerate(self.buckets):
                if s <= o < e:
                    self._param_bucket.append(bi)
                    self._bucket_count[bi] += 1
                    break
        self._pending = list(self._bucket_count)
        self._launched = [False] * len(self.buckets)

    def start(self):
        """Call before ``backward``: every gradient must live in the arena the buckets reduce.

        Per-parameter launches stay on only if exactly one grad-enabled forward of the module (or an unknown
        number, when no module was given) produced the loss."""
        self.deferred = self._fwd_hook is not None and self._grad_forwards != 1
        self._grad_forwards = 0
        self.flat.rebind_grads(zero_missing=True)
        self._pending = list(self._bucket_count)
        self._launched = [False] * len(self.buckets)
        self._ready = [False] * len(self.flat.params)
        self._works = []

    def finish(self):
        """Call after ``backward``: flush remaining buckets and wait for every reduction."""
        if not self.enabled:
            return
        for b in range(len(self.buckets)):
            if not self._launched[b]:
                self._launch(b)
        for work, buf, scatter, home, post in self._works:
            work.wait()
            if post is not None:  # reduce-scatter into the optimizer shard
                post()
                continue
            if home is not None:  # bf16 wire buffer back into its fp32 destination
                home.copy_(buf)
                buf = home
            if not self._use_avg:
                buf.div_(self.world)
            if scatter is not None:
                full, rows = scatter
                full.index_copy_(0, rows, buf)
        self._works = []
        self.deferred = False
        self.flat.rebind_grads()

    def reduce_all(self) -> None:
        """Non-overlapped reduction of the whole arena (the graph-captured step's collective phase)."""
        if not self.enabled:
            return
        self.start()
        self.finish()

    def set_row_subset(self, param, rows: torch.Tensor) -> None:
        """Reduce only ``rows`` of ``param``'s gradient (e.g. the embedding rows of the tokens the dataset
        contains; every other row is zero on every rank).  Exact, and ~25 % less traffic for GPT-2's W_E."""
        i = self.flat.index[id(param)]
        o = self.flat.offset_of(param)
        n = param.numel()
        width = param.shape[-1]
        self._subsets[i] = (o, n, width, rows.to(self.flat.grad.device).long().unique())
        self.__dict__.pop("_subsets_sorted", None)

    def remove(self):
        for h in self._hooks:
            h.remove()
        self._hooks = []
        if self._fwd_hook is not None:
            self._fwd_hook.remove()
            self._fwd_hook = None
        if self._listener is not None:
            grad_hooks.remove_listener(self._listener)
            self._listener = None
