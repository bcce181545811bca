"""Stop-gradient pair (parity: ``/root/reference/iit/model_pairs/stop_grad_pair.py:8-152``).

``StopGradHookedModel`` wraps the LL model.  Its ``forward`` divides the whole
hook of every layer component containing a non-circuit node by ``scale`` (1e6)
and zeroes the gradient of every non-circuit node slice.  Like the reference
(``run_with_hooks(..., reset_hooks_end=False)``, quirk Q7) these effects
**persist** into later ``run_with_cache`` / ``run_with_hooks`` / intervention runs
on the same wrapper until the next ``forward`` re-installs them.

On native models the effects are a persistent ``RunPlan`` (``scale`` + ``zero_grad``
entries) merged into every run, so they execute inside the engine rather than as
Python hooks; other models get TL-style hooks exactly like the reference.
"""
from __future__ import annotations

from typing import Any, Optional

import torch
from torch import Tensor

from ..core.index import EVERYTHING
from ..core.nodes import LLNode
from ..engine.plan import RunPlan
from ..utils import node_picker
from .freeze_model_pair import FreezedModelPair


class StopGradHookedModel:
    def __init__(self, model, params_not_in_circuit, nodes_not_in_circuit, post_nodes_not_in_circuit,
                 scale: float = 1e6, use_forward_hooks: bool = True):
        self.model = model
        self.params_not_in_circuit = params_not_in_circuit
        self.nodes_not_in_circuit = nodes_not_in_circuit
        self.post_nodes_not_in_circuit = post_nodes_not_in_circuit
        self.scale = scale
        self.use_forward_hooks = use_forward_hooks
        self.native = getattr(model, "supports_run_plan", False)
        self.persistent_plan: Optional[RunPlan] = None
        self.supports_run_plan = self.native

    def __getattr__(self, name: str) -> Any:
        if name in ("model",):
            raise AttributeError(name)
        return getattr(self.model, name)

    # -------------------------------------------------------------- reference hooks
    @staticmethod
    def make_ln_hook(ll_node: LLNode, scale: float):
        def hook_fn(act: Tensor, hook) -> Tensor:
            return act / scale
        return hook_fn

    @staticmethod
    def make_detached_hook(ll_node: LLNode):
        def hook_fn(act: Tensor, hook) -> Tensor:
            idx = ll_node.get_index()
            act[idx] = act[idx].clone().detach()
            return act
        return hook_fn

    def make_zero_grad_hook(self, ll_node: LLNode):
        def hook_fn(grad: Tensor, hook) -> Tensor:
            idx = ll_node.get_index()
            grad = grad.clone()
            grad[idx] = 0
            return [grad]
        return hook_fn

    def _stop_plan(self) -> RunPlan:
        plan = RunPlan()
        if self.use_forward_hooks:
            for n in self.post_nodes_not_in_circuit:
                plan.scale[n.name] = self.scale
        for n in self.nodes_not_in_circuit:
            plan.zero_grad.setdefault(n.name, []).append(n.index)
        return plan

    # -------------------------------------------------------------- execution
    def forward(self, x, plan: Optional[RunPlan] = None):
        self.model.reset_hooks()
        if self.native:
            self.persistent_plan = self._stop_plan()
            return self.model(x, plan=self.persistent_plan.merged(plan) if plan is not None
                              else self.persistent_plan.merged(RunPlan()))
        fwd = [(n.name, self.make_ln_hook(n, self.scale)) for n in self.post_nodes_not_in_circuit] \
            if self.use_forward_hooks else []
        bwd = [(n.name, self.make_zero_grad_hook(n)) for n in self.nodes_not_in_circuit]
        return self.model.run_with_hooks(x, fwd_hooks=fwd, bwd_hooks=bwd, reset_hooks_end=False)

    def __call__(self, *args, **kwargs):
        return self.forward(*args, **kwargs)

    def run_capture(self, x, names, truncate: bool = True):
        return self.model.run_capture(x, names, truncate=truncate, base_plan=self.persistent_plan)

    def run_with_cache(self, *args, **kwargs):
        if self.native and self.persistent_plan is not None:
            raise NotImplementedError("use run_capture on native models wrapped by StopGradHookedModel")
        return self.model.run_with_cache(*args, **kwargs)


class StopGradModelPair(FreezedModelPair):
    def __init__(self, hl_model, ll_model, corr, training_args=None):
        defaults = {
            "batch_size": 256,
            "lr": 0.001,
            "num_workers": 0,
            "use_single_loss": False,
            "iit_weight": 1.0,
            "behavior_weight": 1.0,
            "scale": 1e6,
            "use_ln_hooks": True,
        }
        training_args = {**defaults, **(training_args or {})}
        super().__init__(hl_model, ll_model, corr=corr, training_args=training_args)
        self.ll_model = StopGradHookedModel(
            ll_model,
            node_picker.get_params_not_in_circuit(corr, ll_model),
            node_picker.get_nodes_not_in_circuit(ll_model, corr),
            node_picker.get_post_nodes_not_in_circuit(ll_model, corr),
            scale=training_args["scale"],
            use_forward_hooks=training_args["use_ln_hooks"],
        )
        self.wandb_method = "stop grads"

    def ll_intervened_forward(self, x, ll_nodes, logits=None):
        wrapper = self.ll_model
        if wrapper.native:
            logits = logits or self.ll_logits_mode()
            plan = RunPlan.with_splices([(n.name, n.index, self.ll_cache[n.name]) for n in ll_nodes], logits=logits)
            base = wrapper.persistent_plan
            return wrapper.model(x, plan=base.merged(plan) if base is not None else plan)
        return super().ll_intervened_forward(x, ll_nodes, logits)

    def ll_forward(self, x, logits=None):
        logits = logits or self.ll_logits_mode()
        wrapper = self.ll_model
        if wrapper.native:
            return wrapper.forward(x, plan=RunPlan(logits=logits))
        out = wrapper.forward(x)
        if logits == "argmax":
            return out.argmax(-1)
        return out[:, -1] if logits == "last" and out.dim() == 3 else out
