"""Model-pair engine core (parity: ``/root/reference/iit/model_pairs/base_model_pair.py:23-326``).

A model pair holds an HL causal model, an LL network and a correspondence
``corr: {HLNode: {LLNode}}``.  ``do_intervention`` runs the source ("ablation")
input through both models, then re-runs the base input with source activations
spliced in at the HL node / its mapped LL nodes.

MI355X-native execution: when the LL model is a native
``iit_amd`` model (it accepts a ``RunPlan``), the intervention is compiled to a
plan instead of Python hook closures:

1. source LL run: ``no_grad``, captures only ``corr[hl_node]`` hooks, stops after
   the deepest one (the reference caches every hook of a full forward);
2. base LL run: the splice happens inside the fused kernels / skips dead producers;
   only the logits the loss reads are computed (``logits="last"`` for IOI).

Any other ``HookedRootModule`` LL model takes the reference path
(``run_with_cache`` + ``run_with_hooks`` with clone/index-put hooks).

Training (``train``): same loop, metric names, early stop and scheduler logic as
the reference, plus: a flat fp32 parameter arena with a fused clip+Adam
(:mod:`iit_amd.ops.optim`), data parallelism over RCCL with bucketed all-reduce
overlapped with backward (:mod:`iit_amd.parallel.ddp`), device-resident loaders,
deferred metric reads (no per-step ``.item()``), a NaN/Inf step guard, optional
wandb / JSONL sinks, and checkpoint / resume (:mod:`iit_amd.utils.checkpoint`).
"""
from __future__ import annotations

from abc import ABC, abstractmethod
from typing import Any, Callable, Dict, Iterable, List, Optional, Tuple, final

import numpy as np
import torch
from torch import Tensor

from ..config import WANDB_ENTITY
from ..core.correspondence import Correspondence
from ..core.index import EVERYTHING, Ix, TorchIndex
from ..core.metric import MetricStoreCollection, MetricType
from ..core.nodes import HLNode, HookName, LLNode
from ..data.iit_dataset import IITDataset
from ..engine.plan import RunPlan
from ..hooks.hook_points import ActivationCache, HookPoint
from ..parallel import dist as pdist
from ..utils.progress import progress
from ..utils.sinks import make_sink
from ..utils.tracing import StepTimer, sync_point, trace_range


def _is_native(model) -> bool:
    return getattr(model, "supports_run_plan", False) or hasattr(model, "run_capture")


def _underlying_module(model) -> torch.nn.Module:
    return model if isinstance(model, torch.nn.Module) else getattr(model, "model")


def dataset_token_ids(dataset) -> Optional[Tensor]:
    """Distinct input token ids of a (possibly nested / subset) IOI-style dataset, or None."""
    seen = set()
    while dataset is not None and id(dataset) not in seen:
        seen.add(id(dataset))
        fn = getattr(dataset, "token_ids", None)
        if callable(fn):
            return fn()
        dataset = getattr(dataset, "base_data", None) or getattr(dataset, "dataset", None)
    return None


def dataset_seq_len(dataset) -> Optional[int]:
    """Input sequence length of a token dataset (``x`` of its first item is ``[S]``), or None."""
    try:
        x = dataset[0][0]
    except Exception:  # noqa: BLE001 - any dataset shape
        return None
    if isinstance(x, (tuple, list)):
        x = x[0]
    if isinstance(x, Tensor) and x.dim() == 1 and not x.dtype.is_floating_point:
        return int(x.shape[0])
    return None


def _ll_nodes_of(corr, hl_node) -> List[LLNode]:
    v = corr[hl_node]
    if isinstance(v, LLNode):
        return [v]
    return sorted(v, key=lambda n: (n.name, repr(n.index)))


class BaseModelPair(ABC):
    hl_model: Any
    ll_model: Any
    hl_cache: Any
    ll_cache: Any
    corr: Correspondence
    training_args: Dict[str, Any]
    wandb_method: str
    rng: np.random.Generator
    dataset_class = IITDataset

    # ------------------------------------------------------------------ abstract API
    @property
    @abstractmethod
    def loss_fn(self) -> Callable[[Tensor, Tensor], Tensor]:
        ...

    @staticmethod
    @abstractmethod
    def make_train_metrics() -> MetricStoreCollection:
        ...

    @staticmethod
    @abstractmethod
    def make_test_metrics() -> MetricStoreCollection:
        ...

    @abstractmethod
    def run_train_step(self, base_input, ablation_input, loss_fn, optimizer) -> Dict[str, Any]:
        ...

    @abstractmethod
    def run_eval_step(self, base_input, ablation_input, loss_fn) -> Dict[str, Any]:
        ...

    # ------------------------------------------------------------------ intervention
    def hl_run_kwargs(self) -> Dict[str, Any]:
        """Extra kwargs for HL forwards (IOI uses ``last_only`` to skip [B,S,V] logits)."""
        return {}

    def ll_logits_mode(self) -> str:
        """Which LL logits the losses read: ``full`` ([B,S,V]) or ``last`` ([B,V])."""
        return "full"

    def native(self) -> bool:
        """Use the plan-driven engine (False = reference closure/hook semantics, "reference-equivalent eager")."""
        return self.training_args.get("engine", "native") != "reference" and _is_native(self.ll_model)

    def ll_source_cache(self, x: Tensor, ll_nodes: Iterable[LLNode]):
        names = sorted({n.name for n in ll_nodes})
        model = self.ll_model
        if self.native():
            pf = getattr(self, "_source_prefetch", None)
            if pf is not None:  # evaluation: the double-buffered cache computed ahead on a side stream
                cached = pf.lookup(x, names)
                if cached is not None:
                    return ActivationCache(cached, model)
            return ActivationCache(model.run_capture(x, names), model)
        _, cache = model.run_with_cache(x)
        return cache

    def ll_intervened_forward(self, x: Tensor, ll_nodes: Iterable[LLNode], logits: Optional[str] = None):
        logits = logits or self.ll_logits_mode()
        model = self.ll_model
        if self.native():
            plan = RunPlan.with_splices(
                [(n.name, n.index, self.ll_cache[n.name]) for n in ll_nodes], logits=logits)
            return model(x, plan=plan)
        out = model.run_with_hooks(x, fwd_hooks=[(n.name, self.make_ll_ablation_hook(n)) for n in ll_nodes])
        return out[:, -1] if logits == "last" and out.dim() == 3 else out

    def ll_intervention(self, base_x: Tensor, ablation_x: Tensor, ll_nodes: Iterable[LLNode]) -> Tensor:
        """The LL side of an interchange intervention: the source run's activations at ``ll_nodes`` (kept in
        ``self.ll_cache``) spliced into the base run -- one paired forward when the native engine covers it, else
        the truncated source capture followed by the spliced forward."""
        with trace_range("ll_paired_fwd"):
            ll_output = self.ll_paired_intervention(base_x, ablation_x, ll_nodes)
        if ll_output is None:
            with trace_range("ll_source_cache"):
                self.ll_cache = self.ll_source_cache(ablation_x, ll_nodes)
            sync_point()
            with trace_range("ll_spliced_fwd"):
                ll_output = self.ll_intervened_forward(base_x, ll_nodes)
        sync_point()
        return ll_output

    def ll_paired_intervention(self, base_x: Tensor, ablation_x: Tensor, ll_nodes: Iterable[LLNode],
                               logits: Optional[str] = None):
        """``ll_source_cache`` + ``ll_intervened_forward`` as ONE paired forward of source and base rows
        (``HookedTransformer.run_paired``) when the native engine covers the configuration;
        sets ``self.ll_cache`` to the source activations at the splice sites.  None = not covered (two forwards).
        ``training_args["paired"] = False`` turns it off; pairs that customise the two runs (StopGrad) keep them."""
        if not self.native() or self.training_args.get("paired", True) is False:
            return None
        if getattr(self, "_source_prefetch", None) is not None:
            return None
        cls = type(self)
        if (cls.ll_intervened_forward is not BaseModelPair.ll_intervened_forward
                or cls.ll_source_cache is not BaseModelPair.ll_source_cache):
            return None
        fn = getattr(self.ll_model, "run_paired", None)
        if fn is None:
            return None
        sites = {}
        for n in ll_nodes:
            if n.subspace is not None:
                return None
            sites.setdefault(n.name, []).append(n.index)
        res = fn(base_x, ablation_x, sites, logits=logits or self.ll_logits_mode())
        if res is None:
            return None
        out, caps = res
        self.ll_cache = ActivationCache(caps, self.ll_model)
        return out

    def ll_forward(self, x: Tensor, logits: Optional[str] = None):
        logits = logits or self.ll_logits_mode()
        model = self.ll_model
        if logits in ("last", "argmax") and self.native():
            return model(x, plan=RunPlan(logits=logits))
        out = model(x)
        if logits == "argmax":
            return out.argmax(dim=-1)
        return out[:, -1] if logits == "last" and out.dim() == 3 else out

    def do_intervention(self, base_input, ablation_input, hl_node: HLNode, verbose: bool = False
                        ) -> Tuple[Tensor, Tensor]:
        ablation_x = ablation_input[0]
        base_x = base_input[0]
        hl_kw = self.hl_run_kwargs()
        with trace_range("hl_source_cache"):
            hl_ablation_output, self.hl_cache = self.hl_model.run_with_cache(ablation_input, **hl_kw)
        with trace_range("hl_intervened_fwd"):
            hl_output = self.hl_model.run_with_hooks(
                base_input, fwd_hooks=[(hl_node.name, self.make_hl_ablation_hook(hl_node))], **hl_kw)
        ll_nodes = _ll_nodes_of(self.corr, hl_node)
        ll_output = self.ll_intervention(base_x, ablation_x, ll_nodes)
        if verbose:
            print(f"{hl_node=}, {ll_nodes=}\n{hl_output=}")
        return hl_output, ll_output

    @staticmethod
    def get_label_idxs():
        return Ix[[None]]

    def make_hl_model(self, hl_graph):
        raise NotImplementedError

    def set_corr(self, corr):
        self.corr = corr

    def sample_hl_name(self) -> HLNode:
        return self.rng.choice(list(self.corr.keys()))

    def make_hl_ablation_hook(self, hl_node: HLNode):
        if not isinstance(hl_node, HLNode):
            raise AssertionError(f"hl_node is not an instance of HLNode, but {type(hl_node)}")
        if hl_node.index is None:
            return self.hl_ablation_hook
        index = hl_node.index

        def hl_ablation_hook(act: Tensor, hook: HookPoint) -> Tensor:
            src = self.hl_cache[hook.name]
            if isinstance(act, (int, float)):
                return src
            if index == EVERYTHING:
                return src.clone()
            out = act.clone()
            out[index.as_index] = src[index.as_index]
            return out

        return hl_ablation_hook

    def hl_ablation_hook(self, act: Tensor, hook: HookPoint) -> Tensor:
        return self.hl_cache[hook.name]

    def make_ll_ablation_hook(self, ll_node: LLNode) -> Callable[[Tensor, HookPoint], Tensor]:
        if ll_node.subspace is not None:
            raise NotImplementedError("subspace interventions are not supported")
        index = ll_node.index if ll_node.index is not None else EVERYTHING

        def ll_ablation_hook(act: Tensor, hook: HookPoint) -> Tensor:
            out = act.clone()
            out[index.as_index] = self.ll_cache[hook.name][index.as_index].to(out.dtype)
            return out

        return ll_ablation_hook

    def run_phase(self, key, compute_loss: Callable[[], Tensor], optimizer, step_fn):
        """One optimizer phase of a train step: ``loss = compute_loss(); step_fn(loss, optimizer)``.

        ``compute_loss`` may return ``(loss, extras)``; the phase then returns
        ``(loss, extras)`` detached (e.g. the parts of a single combined loss).

        ``key`` names the phase's static structure (phase kind + sampled node), so
        :class:`iit_amd.engine.graphs.GraphedTrainStep` can capture each distinct
        phase once as a HIP graph and replay it; without a runner it runs eagerly.

        (A phase's Adam overlapped with the next phase's forward was measured and removed: the forward GEMMs leave
        no room for a co-resident memory-bound pass, profiles/adam_overlap_r4.txt.)"""
        runner = getattr(self, "_phase_runner", None)
        if runner is not None:
            with trace_range(f"phase:{key[0]}"):
                return runner(key, compute_loss, optimizer, step_fn)
        out = compute_loss()
        if isinstance(out, tuple):  # (loss, {name: tensor}) -> (loss, detached extras)
            loss, extras = out
            step_fn(loss, optimizer)
            return loss.detach(), {k: v.detach() for k, v in extras.items()}
        step_fn(out, optimizer)
        return out.detach()

    def get_IIT_loss_over_batch(self, base_input, ablation_input, hl_node: HookName, loss_fn):
        hl_output, ll_output = self.do_intervention(base_input, ablation_input, hl_node)
        return loss_fn(ll_output, hl_output)

    # ------------------------------------------------------------------ optimisation
    def _ll_module(self) -> torch.nn.Module:
        return _underlying_module(self.ll_model)

    def make_optimizer(self, lr: float):
        module = self._ll_module()
        fused = self.training_args.get("fused_optimizer", None)
        if fused is None:
            fused = next(module.parameters()).is_cuda
        if fused:
            from ..engine.flat import FlatParams
            from ..ops.optim import FusedAdam
            flat = getattr(module, "_flat_params", None)
            if flat is None:
                flat = FlatParams(module, with_bf16_shadow=getattr(module, "wants_bf16_shadow", False))
                module._flat_params = flat
            if self._zero_requested():
                # optimizer-state sharding over the data-parallel ranks (ZeRO-1, iit_amd/parallel/zero.py); the
                # reducer's buckets define the shards (set again when the staged schedule re-buckets)
                from ..parallel.zero import ShardedFusedAdam
                opt = ShardedFusedAdam(flat, flat.buckets(int(self.training_args.get("bucket_mb", 64.0) * (1 << 20))),
                                       lr=lr)
                if self.training_args.get("zero_overlap_gather", True):
                    opt.attach_gates(module)  # the all-gather of the updated pieces overlaps the next forward
            else:
                opt = FusedAdam(flat, lr=lr)
        else:
            opt = torch.optim.Adam(module.parameters(), lr=lr)
        self._setup_reducer(opt)
        if fused:
            # the clip's global norm from the weight-gradient GEMMs (FlatParams.norm_cover): only when the gradients
            # those GEMMs store are the ones the optimizer steps on -- one process, no reducer, no gradient rewrite
            import os
            # (a one-rank reducer -- the IIT_DP_FORCE_REDUCER rehearsal -- averages over one rank: the identity, so
            # the per-rank sums ARE the global ones; at N > 1 the norm pass reads the reduced gradient once more)
            opt.flat.norm_fuse = ((self._reducer is None or pdist.world_size() == 1)
                                  and not getattr(opt, "sharded", False)
                                  and not self.rewrites_grads_before_step()
                                  and os.environ.get("IIT_FUSED_NORM", "1") != "0")
        return opt

    def sync_params(self) -> None:
        """Make every rank's parameters final: finishes the ZeRO-1 optimizer's deferred all-gathers (the next forward
        finishes them block by block; a direct read of the parameters -- ``state_dict``, a copy -- needs this)."""
        wait = getattr(getattr(self, "optimizer", None), "wait_gathers", None)
        if wait is not None:
            wait()

    def rewrites_grads_before_step(self) -> bool:
        """Whether this pair changes parameter gradients between the backward and the optimizer step (beyond the
        clip, which the optimizer does itself)."""
        return False

    def _zero_requested(self) -> bool:
        """Optimizer-state sharding: ``training_args["zero"]`` (or ``IIT_ZERO=1``) under data parallelism."""
        import os
        want = self.training_args.get("zero", os.environ.get("IIT_ZERO", "0") == "1")
        return bool(want) and (pdist.world_size() > 1 or pdist.force_reducer())

    def _setup_reducer(self, optimizer):
        self._reducer = None
        if pdist.world_size() > 1 or pdist.force_reducer():
            from ..engine.flat import FlatParams
            from ..parallel.ddp import GradReducer
            flat = getattr(optimizer, "flat", None)
            if flat is None:
                module = self._ll_module()
                flat = getattr(module, "_flat_params", None) or FlatParams(module)
                module._flat_params = flat
            # "bf16" / "fp32" overrides the reducer's default (bf16 on RCCL, fp32 on gloo: ddp.py)
            wire = self.training_args.get("grad_wire_dtype")
            self._reducer = GradReducer(flat, bucket_mb=self.training_args.get("bucket_mb", 64.0),
                                        overlap=self.training_args.get("overlap_allreduce", True),
                                        wire_dtype={"bf16": torch.bfloat16, "fp32": torch.float32}.get(wire),
                                        module=self._ll_module())
            if getattr(optimizer, "sharded", False):
                self._reducer.attach_shard(optimizer)

    def restrict_sparse_rows(self, dataset, optimizer_rows: bool = True) -> None:
        """Exploit the gradient sparsity of the embedding tables for ``dataset``:

        * only the ``W_E`` rows of tokens the dataset contains and the ``W_pos`` rows below its sequence
          length can receive gradient, so data parallelism all-reduces just those rows, and
        * (``optimizer_rows``) the fused optimizer skips the other rows -- zero gradient and zero moments
          make their Adam update the identity (checked on the first step; no weight decay), so both are
          exact.  Training on inputs outside the dataset afterwards needs ``restrict_sparse_rows(None)``.
        """
        module = self._ll_module()
        flat = getattr(module, "_flat_params", None)
        reducer = getattr(self, "_reducer", None)
        embed = getattr(getattr(module, "embed", None), "W_E", None)
        pos = getattr(getattr(module, "pos_embed", None), "W_pos", None)
        ids = dataset_token_ids(dataset) if dataset is not None else None
        seq = dataset_seq_len(dataset) if dataset is not None else None
        rows = []
        if embed is not None and ids is not None:
            rows.append((embed, ids))
        if pos is not None and seq is not None:
            rows.append((pos, torch.arange(min(seq, pos.shape[0]))))
        if dataset is None:
            rows = [(p, None) for p in (embed, pos) if p is not None]
        for p, r in rows:
            if reducer is not None and id(p) in reducer.flat.index and r is not None:
                reducer.set_row_subset(p, r.to(p.device))
            if optimizer_rows and flat is not None:
                flat.restrict_rows(p, r)

    def restrict_embedding_reduce(self, dataset) -> None:
        """Data-parallel part of :meth:`restrict_sparse_rows` only (reduce just the live embedding rows)."""
        self.restrict_sparse_rows(dataset, optimizer_rows=False)

    def backward(self, loss: Tensor) -> None:
        """``loss.backward()`` + data-parallel gradient averaging + reference grad semantics."""
        reducer = getattr(self, "_reducer", None)
        if reducer is not None:
            reducer.start()
        with trace_range("backward"):
            loss.backward()
        sync_point()
        if reducer is not None:
            with trace_range("grad_allreduce"):
                reducer.finish()
            sync_point()
        # the reference's hook-based splices leave every LL parameter on the autograd
        # graph (zero gradients for dead paths); the native engine skips dead compute,
        # so give untouched parameters an explicit zero gradient (Adam still steps them).  Arena parameters keep
        # ``None``: the fused optimizer zeroes every missing slot in one multi-tensor launch when it binds the
        # arena (FlatParams.rebind_grads) instead of a fill here plus a copy into the arena there per parameter.
        module = self._ll_module()
        flat = getattr(module, "_flat_params", None)
        if flat is not None and not getattr(flat, "zeroes_missing_on_step", False):
            flat = None
        for p in module.parameters():
            if p.requires_grad and p.grad is None and not (flat is not None and flat.owns(p)):
                p.grad = torch.zeros_like(p)

    def clip_grad_fn(self, optimizer=None):
        max_norm = self.training_args.get("clip_grad_norm")
        if not max_norm:
            return
        if optimizer is not None and hasattr(optimizer, "flat"):
            optimizer.pending_clip = max_norm
            return
        from ..ops.optim import clip_grad_norm_
        clip_grad_norm_(list(self._ll_module().parameters()), max_norm)

    def optimizer_step(self, optimizer):
        clip = getattr(optimizer, "pending_clip", None)
        with trace_range("clip_adam"):
            if clip is not None and hasattr(optimizer, "flat"):
                optimizer.pending_clip = None
                optimizer.step(clip_norm=clip)
            else:
                optimizer.step()
        sync_point()

    def step_scheduler(self, lr_scheduler, test_metrics):
        if isinstance(lr_scheduler, torch.optim.lr_scheduler.ReduceLROnPlateau):
            val_metric = self.training_args.get("scheduler_val_metric", "val/accuracy")
            values = test_metrics.to_dict()
            if val_metric not in values:
                raise ValueError(f"val_metric {val_metric} not found in test_metrics {test_metrics}")
            lr_scheduler.step(values[val_metric])
            return
        try:
            lr_scheduler.step()
        except Exception as e:  # pragma: no cover - parity with reference warning path
            print(f"WARNING: Could not step lr_scheduler {lr_scheduler} with exception {e}")

    # ------------------------------------------------------------------ training loop
    def train(self, train_set, test_set, epochs: int = 1000, use_wandb: bool = False,
              checkpoint_dir: Optional[str] = None, resume: bool = False, max_steps: Optional[int] = None,
              fault_hook: Optional[Callable[[int], None]] = None):
        """Reference training loop (``base_model_pair.py:204-261``) plus resume and a test-only
        ``fault_hook(epoch)`` called after each epoch's checkpoint (fault-injection seam)."""
        training_args = self.training_args
        if pdist.is_main():
            print(f"{training_args=}")
        if not isinstance(train_set, IITDataset):
            raise AssertionError(f"train_set is not an instance of IITDataset, but {type(train_set)}")
        if not isinstance(test_set, IITDataset):
            raise AssertionError(f"test_set is not an instance of IITDataset, but {type(test_set)}")
        pdist.broadcast_module(self._ll_module())
        train_loader, test_loader = self.make_loaders(train_set, test_set, training_args["batch_size"],
                                                      training_args["num_workers"])
        early_stop = training_args["early_stop"]
        optimizer = self.make_optimizer(training_args["lr"])
        # only the embedding rows the training data can reach get gradient: reduce (DP) and update just those
        # (exact, see restrict_sparse_rows); evaluation reads the other rows unchanged
        self.restrict_sparse_rows(train_set)
        loss_fn = self.loss_fn
        scheduler_cls = training_args.get("lr_scheduler", None)
        lr_scheduler = None
        if scheduler_cls == torch.optim.lr_scheduler.ReduceLROnPlateau:
            lr_scheduler = scheduler_cls(optimizer, mode=training_args.get("scheduler_mode", "max"),
                                         factor=0.1, patience=10)
        elif scheduler_cls:
            lr_scheduler = scheduler_cls(optimizer)
        sink = make_sink(use_wandb and pdist.is_main(), project="iit", entity=WANDB_ENTITY,
                         config={**{k: str(v) for k, v in training_args.items()}, "method": self.wandb_method})
        start_epoch = 0
        if checkpoint_dir and resume:
            from ..utils.checkpoint import load_resume_state
            start_epoch = load_resume_state(checkpoint_dir, self, optimizer, lr_scheduler)
        self.optimizer = optimizer
        self._prime_train_graphs(train_loader, loss_fn, optimizer)
        epoch = start_epoch
        for epoch in progress(range(start_epoch, epochs), disable=not pdist.is_main()):
            train_metrics = self._run_train_epoch(train_loader, loss_fn, optimizer, max_steps=max_steps)
            # evaluation on the same stream as the (graphed) training steps: every kernel of the run is ordered on
            # one stream, so the caching allocator never hands memory across streams between epochs
            step = getattr(self, "_graph_step", None)
            import contextlib
            with (step.stream_context() if step is not None else contextlib.nullcontext()):
                test_metrics = self._run_eval_epoch(test_loader, loss_fn)
            self._reduce_metrics(train_metrics)
            self._reduce_metrics(test_metrics)
            if lr_scheduler is not None:
                self.step_scheduler(lr_scheduler, test_metrics)
            self.test_metrics = test_metrics
            self.train_metrics = train_metrics
            if pdist.is_main():
                self._print_and_log_metrics(epoch, train_metrics.metrics + test_metrics.metrics, sink)
                self._log_throughput(epoch, sink)
            if checkpoint_dir:
                from ..utils.checkpoint import save_resume_state
                save_resume_state(checkpoint_dir, self, optimizer, lr_scheduler, epoch + 1)
                pdist.barrier()
            if fault_hook is not None:
                fault_hook(epoch)
            if early_stop and self._check_early_stop_condition(test_metrics.metrics):
                break
        self.sync_params()
        # lift the row restriction: later backwards (fine-tuning on other data) may touch any embedding row
        self.restrict_sparse_rows(None)
        if sink is not None:
            sink.log({"final epoch": epoch})
            sink.close()

    def _prime_train_graphs(self, train_loader, loss_fn, optimizer) -> None:
        """Capture every (phase, sampled node) graph before epoch 0 and put the training state back exactly
        (:meth:`GraphedTrainStep.prime_preserving`), so no epoch pays the capture warm-up.  The priming batch is
        the loader's first; the torch RNG its shuffle consumed is restored with the rest.  ``training_args["prime_graphs"]``
        or ``IIT_PRIME_GRAPHS=1|0``."""
        import os
        want = self.training_args.get("prime_graphs", None)
        if want is None:  # on by default (validated on MI355X: tests/test_eval_graphs_gpu.py, profiles/time_to_iia_r4.txt)
            want = os.environ.get("IIT_PRIME_GRAPHS", "1") == "1"
        if not want:
            return
        step = self.train_step_fn(optimizer, loss_fn)
        if not hasattr(step, "prime_preserving"):
            return
        import time
        t0 = time.perf_counter()
        rng = torch.get_rng_state()
        try:
            base, abl = next(iter(train_loader))
        finally:
            torch.set_rng_state(rng)
        # the phase graphs are captured in training mode (BatchNorm batch statistics, dropout), whatever mode an
        # earlier evaluation left the module in; the previous mode is put back afterwards
        module = self._ll_module()
        was_training = module.training
        module.train()
        try:
            with step.stream_context():
                n = step.prime_preserving(base, abl, loss_fn, optimizer)
        finally:
            module.train(was_training)
        if torch.cuda.is_available():
            torch.cuda.synchronize()
        from ..utils import tracing
        if tracing.PROFILE and pdist.is_main():
            print(f"[perf] primed {n} phase graphs in {time.perf_counter() - t0:.2f} s before epoch 0")

    def _log_throughput(self, epoch: int, sink) -> None:
        """The epoch's training throughput (``self.throughput``): to the metric sink when there is one, and to
        stdout with ``IIT_PROFILE=1`` (the default stdout stays the reference's metric lines)."""
        tp = getattr(self, "throughput", None)
        if not tp:
            return
        if sink is not None:
            sink.log({"perf/pairs_per_s": tp["pairs_per_s"], "perf/ms_per_step": tp["ms_per_step"]})
        from ..utils import tracing
        if tracing.PROFILE:
            print(f"[perf] epoch {epoch}: {tp['ms_per_step']:.2f} ms/step, {tp['pairs_per_s']:.0f} pairs/s "
                  f"({int(tp['steps'])} timed steps, {pdist.world_size()} rank(s))")

    @final
    @staticmethod
    def make_loaders(dataset: IITDataset, test_dataset: IITDataset, batch_size: int, num_workers: int):
        return dataset.make_loader(batch_size, num_workers), test_dataset.make_loader(batch_size, num_workers)

    def train_step_fn(self, optimizer, loss_fn) -> Callable:
        """The per-batch step the training loop calls: :class:`iit_amd.engine.graphs.GraphedTrainStep` (every
        optimizer phase captured once per sampled node as a HIP graph, then replayed) for a native LL model on
        the GPU, else the plain ``run_train_step``.  ``training_args["graphs"]`` (default: on when the LL model
        is on a GPU; ``IIT_GRAPHS=0`` turns it off) selects; batches of other shapes (a short epoch tail) and
        phases that cannot be captured run eagerly inside the runner."""
        runner = getattr(self, "_graph_step", None)
        if runner is not None and runner.optimizer is optimizer:
            return runner
        import os
        use = self.training_args.get("graphs", None)
        if use is None:
            module = self._ll_module()
            # default on for native GPU models up to a few billion parameters (each phase graph keeps its
            # activations in the graph memory pool; the 8B Llama runs its phases eagerly unless asked)
            n_params = sum(p.numel() for p in module.parameters())
            use = (os.environ.get("IIT_GRAPHS", "1") != "0" and self.native()
                   and next(module.parameters()).is_cuda and n_params < 2_000_000_000)
        if use:
            from ..engine.graphs import GraphedTrainStep
            g = GraphedTrainStep(self, optimizer, loss_fn)
            if g.enabled:
                self._graph_step = g
                return g
        return self.run_train_step

    def _run_train_epoch(self, loader, loss_fn, optimizer, max_steps: Optional[int] = None) -> MetricStoreCollection:
        self._ll_module().train()
        metrics = self.make_train_metrics()
        step = self.train_step_fn(optimizer, loss_fn)
        import contextlib
        # a graphed step runs on its own stream; the epoch's batches are produced there too (no per-step handoff)
        ctx = step.stream_context() if hasattr(step, "stream_context") else contextlib.nullcontext()
        timer = StepTimer(pdist.world_size())
        with ctx:
            for i, (base_input, ablation_input) in enumerate(progress(loader, total=len(loader),
                                                                      disable=not pdist.is_main(), leave=False)):
                timer.start()
                with trace_range("train_step"):
                    out = step(base_input, ablation_input, loss_fn, optimizer)
                timer.stop(len(base_input[0]))
                metrics.update(out)
                if max_steps is not None and i + 1 >= max_steps:
                    break
            # ms/step and whole-job intervened pairs/s of this epoch (device time, HIP events)
            self.throughput = timer.summary()
        return metrics

    def _run_eval_epoch(self, loader, loss_fn) -> MetricStoreCollection:
        self._ll_module().eval()
        metrics = self.make_test_metrics()
        from ..engine import prefetch
        use_prefetch = prefetch.supported(self)
        batches = prefetch.prefetched_batches(self, loader) if use_prefetch else loader
        step = self.eval_step_fn(loss_fn) if not use_prefetch else None
        with torch.no_grad(), trace_range("eval_epoch"):
            for base_input, ablation_input in batches:
                if step is not None:
                    metrics.update(step(base_input, ablation_input))
                else:
                    metrics.update(self.run_eval_step(base_input, ablation_input, loss_fn))
        return metrics

    def eval_step_fn(self, loss_fn):
        """The graphed evaluation step (:class:`iit_amd.engine.graphs.GraphedEvalStep`) when training runs graphed
        phases (``train_step_fn``), else None (plain ``run_eval_step``).  ``training_args["eval_graphs"]=False``
        keeps evaluation eager."""
        train_step = getattr(self, "_graph_step", None)
        if train_step is None or not self.training_args.get("eval_graphs", True):
            return None
        ev = getattr(self, "_graph_eval", None)
        if ev is None or ev.loss_fn is not loss_fn:
            from ..engine.graphs import GraphedEvalStep
            ev = self._graph_eval = GraphedEvalStep(self, loss_fn, stream=train_step.stream)
        return ev

    @staticmethod
    def _reduce_metrics(collection: MetricStoreCollection) -> None:
        """Epoch metrics over data-parallel ranks as the single-process mean: every store's per-step values are
        summed and counted on each rank, one all-reduce adds the sums and counts, and the store
        keeps sum / count -- exact also when ranks ran different numbers of batches (a mean of per-rank means is
        not)."""
        if pdist.world_size() <= 1:
            return
        stores, parts = [], []
        for m in collection.metrics:
            if len(m) == 0:
                continue
            vals = np.stack([np.atleast_1d(np.asarray(v, dtype=np.float64)) for v in m._values()])
            stores.append((m, vals.shape[1]))
            parts.append(vals.sum(axis=0))
            parts.append(np.array([float(len(vals))]))
        if not parts:
            return
        flat = torch.tensor(np.concatenate(parts), dtype=torch.float64)
        if torch.distributed.get_backend() == "nccl":
            flat = flat.cuda()
        torch.distributed.all_reduce(flat, op=torch.distributed.ReduceOp.SUM)
        flat = flat.cpu().numpy()
        off = 0
        for m, n in stores:
            total, count = flat[off:off + n], flat[off + n]
            off += n + 1
            mean = total / count
            m._store = [mean if (m.type == MetricType.LOG) else float(mean[0])]

    @staticmethod
    def _check_early_stop_condition(test_metrics) -> bool:
        """True iff every ACCURACY metric reached 100 % (reference Q1 semantics)."""
        got = False
        for metric in test_metrics:
            if metric.type == MetricType.ACCURACY:
                got = True
                if metric.get_value() < 100:
                    return False
        if not got:
            raise ValueError("No accuracy metric found in test_metrics!")
        return True

    @staticmethod
    def _print_and_log_metrics(epoch, metrics, sink=None):
        line = ", ".join(str(m) for m in metrics)
        print(f"\nEpoch {epoch}: {line}")
        if sink is not None:
            sink.log({"epoch": epoch})
            for m in metrics:
                v = m.get_value()
                sink.log({m.get_name(): v.tolist() if isinstance(v, np.ndarray) else v})
