"""HIP-graph captured IIT training steps (HIP graphs instead of a tracing compiler).

An IIT step is a short chain of optimizer *phases* (IIT, strict, behaviour for
``IOI_ModelPair``); each phase is a fixed kernel sequence for a given sampled
node: source capture forward, spliced base forward, HL forwards, loss, backward,
fused clip+Adam.  The only host decisions are the node samples, taken from the
pair's RNG *before* the phase runs.  So :class:`GraphedTrainStep`:

* keeps static device buffers for the batch (each new batch is copied in: six
  small tensors, copied with one multi-tensor launch per dtype);
* runs the first ``warmup`` occurrences of every phase key eagerly (this also
  settles lazily-built state: GEMM autotune decisions, the bf16 weight mirror,
  hipBLASLt heuristics), then captures the phase once with
  ``torch.cuda.graph`` into a memory pool shared by all phase graphs (phases
  never run concurrently) and replays it from then on;
* returns clones of the captured loss outputs, so metric stores never alias
  buffers a later replay overwrites.

The fused Adam keeps its step counter / bias corrections / NaN-guard on device,
so replays are exact continuations of the eager schedule; the step-level
semantics (RNG stream, phase order, 3 optimizer steps per IOI batch) are the
pair's own ``run_train_step`` -- this class only swaps the phase executor.

Batches whose shapes differ from the captured ones (e.g. a short final batch)
run eagerly.

Data parallel: collectives are never captured.  Each phase becomes graphs
around eager gradient all-reduces -- ``[forward + backward of the top layers]``,
then one graph per lower stage of layers, each followed by the bucketed RCCL
all-reduce of the arena range it finished (overlapping the next stage, see
:mod:`iit_amd.engine.staged`; ``IIT_DP_STAGES``, default 6), then ``[clip +
Adam]`` -- so every rank issues the identical collective sequence whatever gets
captured, and the launch-bound compute still runs as replays.
(``IIT_GRAPHS_DP=0`` keeps DP runs fully eager.)
"""
from __future__ import annotations

import os
from typing import Dict, Optional, Tuple

import torch

from ..utils.tracing import sync_point, trace_range


# "thread_local": only this thread's unsafe HIP calls break a capture.  Under data parallelism the RCCL
# process group's watchdog thread polls its work events (hipEventQuery) while a phase is being captured;
# in the default "global" mode such a call from another thread can invalidate the capture.
_CAPTURE_MODE = "thread_local"
_SYNC_BEFORE_REPLAY = os.environ.get("IIT_GRAPH_SYNC_BEFORE_REPLAY") == "1"  # diagnostics
_RECAPTURE_ALL = os.environ.get("IIT_GRAPH_RECAPTURE_ALL") == "1"  # diagnostics


def _join_gathers(optimizer) -> None:
    """Finish a ZeRO-1 optimizer's deferred all-gathers (``ShardedFusedAdam.wait_gathers``): before a graph replay
    (a replayed forward calls no gates) and before the weights are read or written wholesale."""
    wait = getattr(optimizer, "wait_gathers", None)
    if wait is not None:
        wait()


def _sync_gemm_decisions() -> None:
    """Rank-consistent GEMM choices before a data-parallel capture (``gemm_dispatch.sync_decisions``)."""
    from ..ops.gemm_dispatch import sync_decisions
    sync_decisions()


def _sync_hyper(optimizer) -> None:
    """A captured optimizer step replays the kernel arguments of its capture; the fused Adam reads its learning
    rate (and betas / eps / weight decay) from device scalars, refreshed here when the host values changed (an LR
    scheduler stepped between epochs).  Optimizers without device hyper-parameters are left alone."""
    sync = getattr(optimizer, "sync_hyper", None)
    if sync is not None:
        sync()
    _join_gathers(optimizer)  # a replayed forward passes no ZeRO-1 gates


def _clone_out(out):
    """Copies of a replayed phase's outputs (the captured buffers are overwritten by the next replay).  Scalar
    losses are packed by one ``stack`` -- a single copy kernel instead of one per metric."""
    if isinstance(out, tuple):
        loss, extras = out
        ts = [loss] + list(extras.values())
        if all(t.dim() == 0 and t.dtype == loss.dtype and t.device == loss.device for t in ts):
            vals = torch.stack(ts).unbind(0)
            return vals[0], dict(zip(extras.keys(), vals[1:]))
        return loss.clone(), {k: v.clone() for k, v in extras.items()}
    return out.clone()


def _detach_out(out):
    if isinstance(out, tuple):
        loss, extras = out
        return loss.detach(), {k: v.detach() for k, v in extras.items()}
    return out.detach()



_FOREACH_COPY = os.environ.get("IIT_FOREACH_COPY", "1") != "0"


def _copy_all(dst, src) -> None:
    """Batch tensors into the static graph inputs: one multi-tensor launch per dtype instead of a copy per tensor
    (``IIT_FOREACH_COPY=0``: a copy per tensor)."""
    if _FOREACH_COPY:
        try:
            torch._foreach_copy_(list(dst), list(src), non_blocking=True)
            return
        except (RuntimeError, TypeError, AttributeError):  # pragma: no cover - older torch / unsupported layouts
            pass
    for d, s_ in zip(dst, src):
        d.copy_(s_, non_blocking=True)

class _CaptureGC:
    """Context for a graph capture: collect cyclic garbage first, keep the collector off during the capture.

    Objects holding CUDA graphs or graph memory pools (earlier runners, pairs referencing them in a cycle) may be
    cyclic garbage; destroying one *inside* another capture is an illegal HIP call that aborts the process, and
    the collector can run at any allocation.  So it runs before, never during, a capture."""

    def __init__(self, collect: bool = True):
        self.collect = collect

    def __enter__(self):
        import gc
        if self.collect:
            gc.collect()
        self._was = gc.isenabled()
        gc.disable()
        return self

    def __exit__(self, *exc):
        import gc
        if self._was:
            gc.enable()
        return False


def _fused_backend(pair) -> bool:
    """Whether the pair's LL model runs on the fused HIP op backend (its backward writes arena gradients itself)."""
    module = pair._ll_module() if hasattr(pair, "_ll_module") else getattr(pair, "ll_model", None)
    ops = getattr(module, "ops", None)
    try:
        return bool(getattr(ops() if callable(ops) else ops, "fused", False))
    except Exception:  # noqa: BLE001 - models without an op backend
        return False


class _TrainState:
    """In-place snapshot of everything a training step mutates: the LL weights (the flat arena and its bf16 mirror
    when there is one, else each parameter), the optimizer state (fused: moments + device step / skip counters;
    ``torch.optim``: every state tensor and scalar), and the torch CPU / GPU RNGs.  ``restore`` copies the saved
    values back into the same tensors."""

    def __init__(self, pair, optimizer):
        import copy
        _join_gathers(optimizer)
        ll = pair._ll_module() if hasattr(pair, "_ll_module") else pair.ll_model
        flat = getattr(ll, "_flat_params", None)
        self.ll, self.flat = ll, flat
        self.pairs = []  # (live tensor, saved clone)
        if flat is not None:
            self.pairs.append((flat.data, flat.data.clone()))
            if flat.shadow is not None:
                self.pairs.append((flat.shadow, flat.shadow.clone()))
        else:
            self.pairs += [(p.data, p.data.clone()) for p in ll.parameters()]
        # module buffers the priming steps mutate in training mode: BatchNorm running statistics and
        # ``num_batches_tracked`` of the PVR ResNet (constant buffers -- causal masks -- are copied back unchanged)
        self.pairs += [(b, b.clone()) for b in ll.buffers() if b is not None]
        self.opt = optimizer
        self.scalars = {}
        if optimizer is not None and hasattr(optimizer, "exp_avg"):  # FusedAdam / ShardedFusedAdam
            for t in (optimizer.exp_avg, optimizer.exp_avg_sq, optimizer._step_dev, optimizer._skipped_dev):
                if t is not None:
                    self.pairs.append((t, t.clone()))
            self.scalars = {"step_count": optimizer.step_count}
        elif optimizer is not None:
            self.opt_state = {}
            for p, st in optimizer.state.items():
                saved = {}
                for k, v in st.items():
                    if torch.is_tensor(v):
                        self.pairs.append((v, v.clone()))
                    else:
                        saved[k] = copy.deepcopy(v)
                self.opt_state[p] = (set(st.keys()), saved)
        self.cpu_rng = torch.get_rng_state()
        self.cuda_rng = torch.cuda.get_rng_state() if torch.cuda.is_available() else None

    @torch.no_grad()
    def restore(self) -> None:
        opt = self.opt
        _join_gathers(opt)  # (a gather still in flight would land after the restore)
        for live, saved in self.pairs:
            live.copy_(saved)
        for k, v in self.scalars.items():
            setattr(opt, k, v)
        if opt is not None and hasattr(self, "opt_state"):
            for p, st in opt.state.items():
                if p not in self.opt_state:
                    # state the priming steps created: zeroed in place, which for Adam-style optimizers IS the
                    # fresh state (step 0, zero moments) -- deleting it would free tensors a captured graph holds
                    for k, v in st.items():
                        if torch.is_tensor(v):
                            v.zero_()
                        elif isinstance(v, (int, float)):
                            st[k] = type(v)(0)
            for p, (keys, saved) in self.opt_state.items():
                st = opt.state[p]
                for k in list(st.keys()):
                    if k not in keys:
                        del st[k]
                st.update(saved)
        torch.set_rng_state(self.cpu_rng)
        if self.cuda_rng is not None:
            torch.cuda.set_rng_state(self.cuda_rng)
        if self.flat is not None:  # weights changed: version bump + listeners (the op backend's bf16 copies)
            self.flat.after_step(mirror_written=self.flat.shadow is not None)
        elif hasattr(self.ll, "mark_weights_changed"):
            self.ll.mark_weights_changed()


class GraphedTrainStep:
    def __init__(self, pair, optimizer=None, loss_fn=None, warmup: int = 1, enabled: Optional[bool] = None):
        self.pair = pair
        self.optimizer = optimizer
        self.loss_fn = loss_fn
        self.warmup = warmup
        ws = torch.distributed.get_world_size() if (torch.distributed.is_available()
                                                   and torch.distributed.is_initialized()) else 1
        if enabled is None:
            enabled = torch.cuda.is_available()
            if ws > 1 and os.environ.get("IIT_GRAPHS_DP", "1") == "0":
                enabled = False
        self.enabled = enabled
        from ..parallel.dist import force_reducer
        self.split = ws > 1 or force_reducer()  # DP: graphs around the (eager) gradient all-reduce
        self.staged = None
        self.force_staged = False  # tests: stage the backward graphs even without a data-parallel reducer
        if self.split and enabled:
            from .staged import staged_for
            self.staged = staged_for(pair)
            reducer = getattr(pair, "_reducer", None)
            if self.staged is not None and reducer is not None:
                reducer.segment_buckets(self.staged.edges)
        self.graphs: Dict[Tuple, Tuple[torch.cuda.CUDAGraph, object]] = {}
        self.seen: Dict[Tuple, int] = {}
        self.pool = None  # shared graph memory pool, created at the first capture
        # torch-op backend: every step -- eager warm-ups, captures and replays -- runs on one dedicated stream.
        # Autograd's AccumulateGrad nodes run on the stream they were created on, so a node made by an eager phase
        # on the default stream and kept alive would accumulate *outside* a later capture (silently missing from
        # the graph).  The fused HIP backend writes every arena gradient from its own backward functions (no
        # AccumulateGrad) and keeps the plain arrangement -- eager on the caller's stream, captures on torch's
        # capture stream -- which also keeps the stream count low: a dedicated stream next to gloo's pool streams
        # deadlocked the two-rank gloo rehearsal on one GPU (scripts/gpu_dp_rehearsal_debug.sh).
        # ``IIT_GRAPH_STREAM=1|0`` forces it on / off.
        mode = os.environ.get("IIT_GRAPH_STREAM", "auto")
        dedicated = mode == "1" or (mode == "auto" and not _fused_backend(pair))
        self.stream = torch.cuda.Stream() if (enabled and torch.cuda.is_available() and dedicated) else None
        if enabled:
            from ..ops.gemm_dispatch import select_graph_safe_blas
            select_graph_safe_blas()
        self._static = None
        self._sig = None
        self.captures = 0
        self.replays = 0
        self.calls = 0
        self.failed: Dict[Tuple, str] = {}
        pair._phase_runner = self._run_phase

    # ------------------------------------------------------------------ static inputs
    def _stage(self, base, abl):
        """Returns (base, abl, eager): static buffers holding this batch, or the batch itself + eager=True."""
        if not self.enabled:
            return base, abl, True
        sig = tuple((tuple(t.shape), t.dtype, t.device) for t in tuple(base) + tuple(abl))
        if self._static is None:
            self._static = (tuple(t.clone() for t in base), tuple(t.clone() for t in abl))
            self._sig = sig
            return self._static[0], self._static[1], False
        if sig != self._sig:  # e.g. a short last batch: eager, keep the captured buffers
            return base, abl, True
        sb, sa = self._static
        _copy_all(sb + sa, tuple(base) + tuple(abl))
        return sb, sa, False

    # ------------------------------------------------------------------ phases
    @staticmethod
    def _eager(compute_loss, optimizer, step_fn):
        out = compute_loss()
        loss = out[0] if isinstance(out, tuple) else out
        step_fn(loss, optimizer)
        return _detach_out(out)

    def _splittable(self, step_fn) -> bool:
        from ..model_pairs.iit_behavior_model_pair import IITBehaviorModelPair
        return getattr(step_fn, "__func__", None) is IITBehaviorModelPair.step_on_loss

    def _run_split_phase(self, full, key, compute_loss, optimizer):
        """DP phase: graph(forward + backward) -> eager all-reduce -> graph(clip + Adam).

        With a :class:`~iit_amd.engine.staged.StagedBackward` the backward is several graphs (one per stage
        of layers) and each stage's gradient range is all-reduced while the next stage computes."""
        pair = self.pair
        reducer = getattr(pair, "_reducer", None)
        stg = self.staged if (reducer is not None and reducer.enabled) or self.force_staged else None

        def fwd_bwd():
            if stg is not None:
                stg.arm()
            try:
                out = compute_loss()
            finally:
                if stg is not None:
                    stg.disarm()
            loss = out[0] if isinstance(out, tuple) else out
            optimizer.zero_grad()
            if reducer is not None:
                reducer.paused = True  # no collective may be issued from inside a capture
            try:
                loss.backward()
            finally:
                if reducer is not None:
                    reducer.paused = False
            return _detach_out(out)

        def update():
            pair.clip_grad_fn(optimizer)
            pair.optimizer_step(optimizer)

        def reduce_eagerly(run_stage):
            """Host side of the collective schedule (identical on every rank); ``run_stage(i, k)`` computes stage i."""
            if reducer is None:
                for i, k in enumerate(stg.stages() if stg is not None else ()):
                    run_stage(i, k)
                return
            reducer.start()
            # launches come only from the explicit ranges: a stage's backward may cover several forwards (a
            # single combined loss), so a parameter's first gradient report inside it is not its final value
            reducer.paused = True
            try:
                if stg is None:
                    reducer.launch_range(0, reducer.flat.numel)
                else:
                    rng = stg.ranges()
                    reducer.launch_range(*rng[0])
                    for i, k in enumerate(stg.stages()):
                        run_stage(i, k)
                        reducer.launch_range(*rng[i + 1])
            finally:
                reducer.paused = False
            reducer.finish()

        def eager_phase():
            out = fwd_bwd()
            reduce_eagerly(lambda i, k: stg.run_stage(k))
            if stg is not None:
                stg.release()
            update()
            return out

        ent = self.graphs.get(full)
        if ent is None:
            n = self.seen.get(full, 0)
            if n < self.warmup or full in self.failed:
                self.seen[full] = n + 1
                return eager_phase()
            if self.pool is None or os.environ.get("IIT_GRAPH_POOL") == "private":
                self.pool = torch.cuda.graph_pool_handle()
            ga, gb = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
            parts = None
            if getattr(optimizer, "sharded", False):
                # the sharded optimizer step issues collectives (norm all-reduce, all-gather): its device parts
                # are captured one graph each, the collectives and host books between them stay eager
                gb = None
                clip = self.pair.training_args.get("clip_grad_norm") or None
                spec = optimizer.step_parts(clip_norm=clip) if hasattr(optimizer, "step_parts") else None
                if spec is not None:
                    parts = [(torch.cuda.CUDAGraph() if cap else None, fn) for cap, fn in spec]
            gs = []
            # a ZeRO-1 warm-up step deferred its bucket gathers: finish them eagerly BEFORE the capture (a gate
            # inside the capture records nothing that runs now)
            _join_gathers(optimizer)
            # every rank captures this phase at the same call (phase keys follow the identically seeded node RNG):
            # agree on the GEMM kernels first, so the graphs hold rank 0's choices on every rank
            _sync_gemm_decisions()
            try:
                with _CaptureGC(), torch.cuda.graph(ga, pool=self.pool, stream=self.stream, capture_error_mode=_CAPTURE_MODE):
                    static_out = fwd_bwd()
                for k in (stg.stages() if stg is not None else ()):
                    g = torch.cuda.CUDAGraph()
                    with _CaptureGC(), torch.cuda.graph(g, pool=self.pool, stream=self.stream, capture_error_mode=_CAPTURE_MODE):
                        stg.run_stage(k)
                    gs.append(g)
                if stg is not None:
                    stg.release()
                if gb is not None:
                    with _CaptureGC(), torch.cuda.graph(gb, pool=self.pool, stream=self.stream,
                                                        capture_error_mode=_CAPTURE_MODE):
                        update()
                elif parts is not None:
                    # capturing runs nothing: the eager pieces are NOT run here either (the replay below runs the
                    # whole sequence), so the host books of the step are not doubled
                    for g_, fn in parts:
                        if g_ is not None:
                            with _CaptureGC(), torch.cuda.graph(g_, pool=self.pool, stream=self.stream,
                                                                capture_error_mode=_CAPTURE_MODE):
                                fn()
            except Exception as e:
                self.failed[full] = repr(e)
                self.pool = None  # see _run_phase: the aborted capture's pool is not reusable
                print(f"[iit graphs] DP phase {key} not captured ({type(e).__name__}: {str(e)[:160]}); eager")
                torch.cuda.synchronize()
                if stg is not None:
                    stg.release()
                return eager_phase()
            ent = self.graphs[full] = ((ga, gs, gb, parts), static_out)
            self.captures += 1
        (ga, gs, gb, parts), static_out = ent
        _sync_hyper(optimizer)
        with trace_range("graph:fwd_bwd"):
            ga.replay()
        sync_point()
        with trace_range("grad_allreduce"):
            reduce_eagerly(lambda i, k: gs[i].replay())
        sync_point()
        with trace_range("graph:clip_adam"):
            if gb is not None:
                gb.replay()
            elif parts is not None:
                self.pair.clip_grad_fn(optimizer)  # (host books only: the fused optimizer clips itself)
                optimizer.pending_clip = None
                for g_, fn in parts:
                    if g_ is not None:
                        g_.replay()
                    else:
                        fn()
            else:
                update()
        sync_point()
        self.replays += 1
        return _clone_out(static_out)

    def _graph_key(self, key, optimizer=None):
        """Graph identity of a phase: the pair's phase key, the batch signature, the LL module's train / eval mode
        (a graph captured in eval mode replays eval-mode BatchNorm / dropout) and the optimizer's row-restriction
        version (a sharded step captures its span table)."""
        module = self.pair._ll_module() if hasattr(self.pair, "_ll_module") else getattr(self.pair, "ll_model", None)
        training = bool(getattr(module, "training", True))
        opt = optimizer if optimizer is not None else self.optimizer
        flat = getattr(opt, "flat", None)
        rv = getattr(flat, "restrict_version", 0) if flat is not None else 0
        return (key, self._sig, training, rv)

    def _run_phase(self, key, compute_loss, optimizer, step_fn):
        full = self._graph_key(key, optimizer)
        if not self.enabled or self._current_eager:
            return self._eager(compute_loss, optimizer, step_fn)
        if self.split:
            if not self._splittable(step_fn):
                return self._eager(compute_loss, optimizer, step_fn)
            return self._run_split_phase(full, key, compute_loss, optimizer)
        ent = self.graphs.get(full)
        if ent is None:
            n = self.seen.get(full, 0)
            if n < self.warmup:
                self.seen[full] = n + 1
                return self._eager(compute_loss, optimizer, step_fn)
            if full in self.failed:
                return self._eager(compute_loss, optimizer, step_fn)
            if self.pool is None or os.environ.get("IIT_GRAPH_POOL") == "private":
                self.pool = torch.cuda.graph_pool_handle()
            g = torch.cuda.CUDAGraph()
            _join_gathers(optimizer)  # (see _run_split_phase)
            try:
                with _CaptureGC(), torch.cuda.graph(g, pool=self.pool, stream=self.stream, capture_error_mode=_CAPTURE_MODE):
                    out = compute_loss()
                    loss = out[0] if isinstance(out, tuple) else out
                    step_fn(loss, optimizer)
                    static_out = _detach_out(out)
            except Exception as e:  # something in the phase is not capturable: keep it eager
                self.failed[full] = repr(e)
                # an aborted capture leaves its private memory pool unusable for the next capture (the caching
                # allocator asserts on it): later captures get a fresh pool (graphs already captured keep theirs)
                self.pool = None
                import traceback
                tb = "".join(traceback.format_exc(limit=12)) if len(self.failed) == 1 else ""
                print(f"[iit graphs] phase {key} not captured ({type(e).__name__}: {str(e)[:160]}); "
                      f"running it eagerly\n{tb}")
                torch.cuda.synchronize()
                return self._eager(compute_loss, optimizer, step_fn)
            if _RECAPTURE_ALL:  # diagnostics: a new capture drops every other graph (recaptured at next use)
                self.graphs.clear()
            ent = self.graphs[full] = (g, static_out)
            self.captures += 1
        g, static_out = ent
        _sync_hyper(optimizer)
        if _SYNC_BEFORE_REPLAY:
            torch.cuda.current_stream().synchronize()
        with trace_range("graph:phase"):
            g.replay()
        sync_point()
        self.replays += 1
        return _clone_out(static_out)

    # ------------------------------------------------------------------ step
    def __call__(self, base_input, ablation_input, loss_fn=None, optimizer=None):
        loss_fn = loss_fn or self.loss_fn
        optimizer = optimizer or self.optimizer
        self.calls += 1
        if self.stream is None or torch.cuda.current_stream() == self.stream:
            # (callers running their whole loop on ``self.stream`` -- bench.py, BaseModelPair.train -- skip the
            # per-step stream handoff)
            return self._step(base_input, ablation_input, loss_fn, optimizer)
        if not self._handoff_warned:
            self._handoff_warned = True
            print("[iit graphs] train step called from another stream: run the loop (and any evaluation between "
                  "steps) inside `with step.stream_context():` -- mixing streams between captured phases and other "
                  "work has been seen to corrupt later replays (scripts/diag_graph_node.py)")
        cur = torch.cuda.current_stream()
        self.stream.wait_stream(cur)
        # the batch was produced on the caller's stream and is read on ours: without this the caller's next
        # allocation (the loader's next batch) could reuse its memory while our copies / eager phases still read it
        for t in tuple(base_input) + tuple(ablation_input):
            if isinstance(t, torch.Tensor) and t.is_cuda:
                t.record_stream(self.stream)
        try:
            with torch.cuda.stream(self.stream):
                return self._step(base_input, ablation_input, loss_fn, optimizer)
        finally:
            cur.wait_stream(self.stream)

    def _step(self, base_input, ablation_input, loss_fn, optimizer):
        sb, sa, eager = self._stage(base_input, ablation_input)
        self._current_eager = eager
        try:
            return self.pair.run_train_step(sb, sa, loss_fn, optimizer)
        finally:
            self._current_eager = False

    _current_eager = False
    _handoff_warned = False

    def stream_context(self):
        """``with step.stream_context(): ...`` runs a whole training loop on the runner's stream (no per-step
        stream handoff); a no-op context when graphs are off."""
        import contextlib
        if self.stream is None:
            return contextlib.nullcontext()

        @contextlib.contextmanager
        def ctx():
            cur = torch.cuda.current_stream()
            self.stream.wait_stream(cur)
            try:
                with torch.cuda.stream(self.stream):
                    yield
            finally:
                cur.wait_stream(self.stream)
        return ctx()

    def prime(self, base_input, ablation_input, loss_fn=None, optimizer=None) -> int:
        """Capture every phase key up front (untimed warmup): force each HL / strict node in turn.

        Each forced phase is a real optimizer step (warmup steps train too); the pair's
        node-sampling RNG is saved and restored, so the sampled sequence of the run
        that follows is unchanged.  Returns the number of graphs captured so far."""
        import copy
        pair = self.pair
        rng_state = copy.deepcopy(pair.rng)
        hl_nodes = list(pair.corr.keys())
        ll_nodes = list(getattr(pair, "nodes_not_in_circuit", []) or [None])
        orig_hl = pair.__dict__.get("sample_hl_name")
        orig_ll = pair.__dict__.get("sample_ll_node")
        try:
            n = max(len(hl_nodes), len(ll_nodes))
            for rep in range(self.warmup + 1):
                for i in range(n):
                    pair.sample_hl_name = lambda i=i: hl_nodes[i % len(hl_nodes)]
                    if ll_nodes[0] is not None:
                        pair.sample_ll_node = lambda i=i: ll_nodes[i % len(ll_nodes)]
                    self(base_input, ablation_input, loss_fn, optimizer)
        finally:
            for name, orig in (("sample_hl_name", orig_hl), ("sample_ll_node", orig_ll)):
                if orig is None:
                    pair.__dict__.pop(name, None)
                else:
                    setattr(pair, name, orig)
            pair.rng = rng_state
        return self.captures

    def prime_preserving(self, base_input, ablation_input, loss_fn=None, optimizer=None) -> int:
        """:meth:`prime` for a real training run: every (phase, node) graph is captured before the first timed
        epoch, then the training state is put back exactly as it was -- weights (fp32 master and bf16 mirror), the
        optimizer's moments and step counters, every RNG -- so the run that follows is the run an unprimed loop
        would have made, minus the capture warm-up (epochs 0-4 ran at 203 / 58 / 23 / 25 / 21
        ms/step while the 4 IIT + 32 strict node graphs were captured as they were first sampled).  The restore is
        in place (``copy_``), so the captured graphs keep pointing at the live tensors."""
        optimizer = optimizer or self.optimizer
        if not self.enabled:
            return 0
        snap = _TrainState(self.pair, optimizer)
        try:
            return self.prime(base_input, ablation_input, loss_fn, optimizer)
        finally:
            snap.restore()

    def detach(self) -> None:
        """Restore eager phases on the pair (graphs are released)."""
        if getattr(self.pair, "_phase_runner", None) == self._run_phase:
            self.pair._phase_runner = None
        self.graphs.clear()


class GraphedEvalStep:
    """Evaluation steps (``pair.run_eval_step``) captured as HIP graphs, one per sampled HL node.

    An eval step is a fixed kernel sequence for a given HL node (the source / base interventions and the
    behaviour forward, no autograd, no optimizer), so -- like :class:`GraphedTrainStep` -- the node is drawn from
    the pair's RNG first (the same single draw ``run_eval_step`` makes), the batch is copied into static
    buffers, and the step for that node is captured once (after ``warmup`` eager runs) and replayed.  The metric
    outputs are cloned after each replay.  Batches of another shape (an epoch's short tail) run eagerly; a pair
    whose eval step does not draw exactly one HL node stays eager."""

    def __init__(self, pair, loss_fn, warmup: int = 1, stream=None):
        self.pair = pair
        self.loss_fn = loss_fn
        self.warmup = warmup
        self.stream = stream  # capture stream (the training runner's dedicated stream, or torch's default)
        self.graphs: Dict[Tuple, Tuple[torch.cuda.CUDAGraph, dict]] = {}
        self.seen: Dict[Tuple, int] = {}
        self.failed: Dict[Tuple, str] = {}
        self.pool = None
        self._static = None
        self._sig = None
        self.ok = True  # False once a step draws a number of HL nodes other than one
        self.replays = 0

    def _eager(self, base, abl):
        return self.pair.run_eval_step(base, abl, self.loss_fn)

    def _join(self) -> None:
        """Finish a ZeRO-1 optimizer's deferred gathers (``module._param_join``, installed by ``attach_gates``)."""
        pair = self.pair
        module = pair._ll_module() if hasattr(pair, "_ll_module") else getattr(pair, "ll_model", None)
        join = getattr(module, "_param_join", None) if module is not None else None
        if join is not None:
            join()

    def __call__(self, base, abl):
        pair = self.pair
        if not self.ok:
            return self._eager(base, abl)
        node = pair.sample_hl_name()
        draws = [0]

        def fixed(_node=node):
            draws[0] += 1
            return _node
        own = pair.__dict__.get("sample_hl_name")  # an instance-level sampler (tests, prime) is restored after
        pair.sample_hl_name = fixed
        try:
            out = self._run(node, base, abl)
        finally:
            if own is None:
                del pair.sample_hl_name
            else:
                pair.sample_hl_name = own
        if draws[0] != 1:  # the step's sampling is not the single draw this runner replays: go eager from now on
            self.ok = False
        return out

    def _run(self, node, base, abl):
        sig = tuple((tuple(t.shape), t.dtype, t.device) for t in tuple(base) + tuple(abl))
        if self._static is None:
            self._static = (tuple(t.clone() for t in base), tuple(t.clone() for t in abl))
            self._sig = sig
        if sig != self._sig:
            return self._eager(base, abl)
        sb, sa = self._static
        _copy_all(sb + sa, tuple(base) + tuple(abl))
        key = (node.name, sig)
        self._join()  # a replayed (or captured) forward passes no ZeRO-1 gates
        ent = self.graphs.get(key)
        if ent is None:
            n = self.seen.get(key, 0)
            if n < self.warmup or key in self.failed:
                self.seen[key] = n + 1
                return self._eager(sb, sa)
            if self.pool is None:
                self.pool = torch.cuda.graph_pool_handle()
            g = torch.cuda.CUDAGraph()
            try:
                with _CaptureGC(), torch.cuda.graph(g, pool=self.pool, stream=self.stream, capture_error_mode=_CAPTURE_MODE):
                    static_out = self._eager(sb, sa)
            except Exception as e:  # not capturable: keep this node eager
                self.failed[key] = repr(e)
                self.pool = None
                print(f"[iit graphs] eval step for {node.name} not captured ({type(e).__name__}: {str(e)[:160]}); eager")
                torch.cuda.synchronize()
                return self._eager(sb, sa)
            ent = self.graphs[key] = (g, static_out)
        g, static_out = ent
        with trace_range("graph:eval_step"):
            g.replay()
        sync_point()
        self.replays += 1
        return {k: (v.clone() if isinstance(v, torch.Tensor) else v) for k, v in static_out.items()}
