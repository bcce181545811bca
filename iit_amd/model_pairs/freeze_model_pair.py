"""Freeze pair (parity: ``/root/reference/iit/model_pairs/freeze_model_pair.py:8-38``).

The reference intends to zero gradients of parameters outside the circuit but
assigns ``.grad`` on an indexed *view* (``param[idx].grad = 0``), which is a no-op
(SURVEY.md Q6).  ``training_args["freeze_mode"]``:

* ``"parity"`` (default) - reproduce the reference (gradients untouched);
* ``"mask"``   - do what was intended: zero ``param.grad[idx]`` for every
  parameter slice not in the circuit, before clipping.
"""
from __future__ import annotations

import torch

from ..utils import node_picker
from .iit_behavior_model_pair import IITBehaviorModelPair


class FreezedModelPair(IITBehaviorModelPair):
    def __init__(self, hl_model, ll_model, corr, training_args=None):
        defaults = {
            "batch_size": 256,
            "lr": 0.001,
            "num_workers": 0,
            "use_single_loss": False,
            "iit_weight": 1.0,
            "behavior_weight": 1.0,
            "freeze_mode": "parity",
        }
        super().__init__(hl_model, ll_model, corr=corr, training_args={**defaults, **(training_args or {})})
        self.params_not_in_circuit = node_picker.get_params_not_in_circuit(corr, ll_model)
        self.wandb_method = "freeze_unwanted"

    def rewrites_grads_before_step(self) -> bool:
        return self.training_args.get("freeze_mode", "parity") == "mask"

    def zero_grad_for_not_in_circuit(self):
        if self.training_args.get("freeze_mode", "parity") != "mask":
            return  # reference semantics: the assignment targets a temporary view
        params = dict(self._ll_module().named_parameters())
        with torch.no_grad():
            for node in self.params_not_in_circuit:
                p = params.get(node.name)
                if p is not None and p.grad is not None:
                    p.grad[node.index.as_index] = 0

    def step_on_loss(self, loss, optimizer):
        optimizer.zero_grad()
        self.backward(loss)
        self.zero_grad_for_not_in_circuit()
        self.clip_grad_fn(optimizer)
        self.optimizer_step(optimizer)
