"""Strict IIT pair (parity: ``/root/reference/iit/model_pairs/strict_iit_model_pair.py:5-91``).

Adds a "strict" loss: patch a *non-circuit* LL node (sampled with the same RNG
stream as HL nodes) from source into base and require the base
label.  Three optimizer steps per batch (IIT, strict, behaviour) unless
``use_single_loss``.  Each phase's source run uses the weights after the previous
phase's step, exactly like the reference.
"""
from __future__ import annotations

from ..core.metric import MetricStore, MetricStoreCollection, MetricType
from ..core.nodes import LLNode
from ..utils import node_picker
from .iit_behavior_model_pair import IITBehaviorModelPair


class StrictIITModelPair(IITBehaviorModelPair):
    def __init__(self, hl_model, ll_model, corr, training_args=None):
        defaults = {
            "batch_size": 256,
            "lr": 0.001,
            "num_workers": 0,
            "use_single_loss": False,
            "iit_weight": 1.0,
            "behavior_weight": 1.0,
            "strict_weight": 1.0,
            "clip_grad_norm": 1.0,
        }
        super().__init__(hl_model, ll_model, corr=corr, training_args={**defaults, **(training_args or {})})
        self.nodes_not_in_circuit = node_picker.get_nodes_not_in_circuit(self.ll_model, self.corr)

    @staticmethod
    def make_train_metrics():
        return MetricStoreCollection([
            MetricStore("train/iit_loss", MetricType.LOSS),
            MetricStore("train/behavior_loss", MetricType.LOSS),
            MetricStore("train/strict_loss", MetricType.LOSS),
        ])

    def sample_ll_node(self) -> LLNode:
        return self.rng.choice(self.nodes_not_in_circuit)

    def get_strict_loss_over_batch(self, base_input, ablation_input, ll_node: LLNode, loss_fn):
        base_x, base_y = base_input[0], base_input[1]
        out = self.ll_paired_intervention(base_x, ablation_input[0], [ll_node])
        if out is None:
            self.ll_cache = self.ll_source_cache(ablation_input[0], [ll_node])
            out = self.ll_intervened_forward(base_x, [ll_node])
        if out.dim() > 1 and out.shape[0] == 1:
            return loss_fn(out, base_y)
        return loss_fn(out.squeeze(), base_y)

    def run_train_step(self, base_input, ablation_input, loss_fn, optimizer):
        args = self.training_args
        hl_node = self.sample_hl_name()

        def iit():
            return self.get_IIT_loss_over_batch(base_input, ablation_input, hl_node, loss_fn) * args["iit_weight"]

        if args["use_single_loss"]:
            ll_node = self.sample_ll_node()

            def total():
                parts = {"iit": iit(),
                         "strict": self.get_strict_loss_over_batch(base_input, ablation_input, ll_node, loss_fn)
                         * args["strict_weight"],
                         "behavior": self.get_behaviour_loss_over_batch(base_input, loss_fn) * args["behavior_weight"]}
                return parts["iit"] + parts["behavior"] + parts["strict"], parts

            _, parts = self.run_phase(("single", hl_node.name, ll_node.name, repr(ll_node.index)), total, optimizer,
                                      self.step_on_loss)
            return {"train/iit_loss": parts["iit"], "train/behavior_loss": parts["behavior"],
                    "train/strict_loss": parts["strict"]}
        iit_loss = self.run_phase(("iit", hl_node.name), iit, optimizer, self.step_on_loss)
        # the strict node is drawn after the IIT phase, as in the reference (same RNG stream)
        ll_node = self.sample_ll_node()
        strict_loss = self.run_phase(
            ("strict", ll_node.name, repr(ll_node.index)),
            lambda: self.get_strict_loss_over_batch(base_input, ablation_input, ll_node, loss_fn) * args["strict_weight"],
            optimizer, self.step_on_loss)
        behavior_loss = self.run_phase(
            ("behavior",), lambda: self.get_behaviour_loss_over_batch(base_input, loss_fn) * args["behavior_weight"],
            optimizer, self.step_on_loss)
        return {"train/iit_loss": iit_loss, "train/behavior_loss": behavior_loss, "train/strict_loss": strict_loss}
