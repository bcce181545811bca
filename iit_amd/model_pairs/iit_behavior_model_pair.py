"""IIT + behaviour multi-task pair (parity: ``/root/reference/iit/model_pairs/iit_behavior_model_pair.py:6-141``).

Two optimizer steps per batch (IIT, then behaviour) unless ``use_single_loss``.
Categorical HL models use CE / argmax IIA; regression HL models MSE and
``|ll - hl| < atol`` IIA.
"""
from __future__ import annotations

import torch
from torch import Tensor

from ..core.metric import MetricStore, MetricStoreCollection, MetricType
from .iit_model_pair import IITModelPair, labels_of


class IITBehaviorModelPair(IITModelPair):
    def __init__(self, hl_model, ll_model, corr, training_args=None):
        defaults = {
            "lr": 0.001,
            "atol": 5e-2,
            "early_stop": True,
            "use_single_loss": False,
            "iit_weight": 1.0,
            "behavior_weight": 1.0,
        }
        super().__init__(hl_model, ll_model, corr=corr, training_args={**defaults, **(training_args or {})})
        self.wandb_method = "iit_and_behavior"

    def _categorical(self) -> bool:
        try:
            return bool(self.hl_model.is_categorical())
        except AttributeError:
            return True

    @property
    def loss_fn(self):
        if self._loss_fn_override is not None:
            return self._loss_fn_override
        return torch.nn.CrossEntropyLoss() if self._categorical() else torch.nn.MSELoss()

    @loss_fn.setter
    def loss_fn(self, value):
        self._loss_fn_override = value

    @staticmethod
    def make_train_metrics():
        return MetricStoreCollection([
            MetricStore("train/iit_loss", MetricType.LOSS),
            MetricStore("train/behavior_loss", MetricType.LOSS),
        ])

    @staticmethod
    def make_test_metrics():
        return MetricStoreCollection([
            MetricStore("val/iit_loss", MetricType.LOSS),
            MetricStore("val/IIA", MetricType.ACCURACY),
            MetricStore("val/accuracy", MetricType.ACCURACY),
        ])

    def get_behaviour_loss_over_batch(self, base_input, loss_fn):
        base_x, base_y = base_input[0], base_input[1]
        output = self.ll_forward(base_x)
        if output.dim() > 1 and output.shape[0] == 1:
            return loss_fn(output, base_y)
        return loss_fn(output.squeeze(), base_y)

    def step_on_loss(self, loss: Tensor, optimizer) -> None:
        optimizer.zero_grad()
        self.backward(loss)
        self.clip_grad_fn(optimizer)
        self.optimizer_step(optimizer)

    def run_train_step(self, base_input, ablation_input, loss_fn, optimizer):
        args = self.training_args
        hl_node = self.sample_hl_name()

        def iit():
            return self.get_IIT_loss_over_batch(base_input, ablation_input, hl_node, loss_fn) * args["iit_weight"]

        def behavior():
            return self.get_behaviour_loss_over_batch(base_input, loss_fn) * args["behavior_weight"]

        if args["use_single_loss"]:
            def total():
                parts = {"iit": iit(), "behavior": behavior()}
                return parts["iit"] + parts["behavior"], parts

            _, parts = self.run_phase(("single", hl_node.name), total, optimizer, self.step_on_loss)
            return {"train/iit_loss": parts["iit"], "train/behavior_loss": parts["behavior"]}
        iit_loss = self.run_phase(("iit", hl_node.name), iit, optimizer, self.step_on_loss)
        behavior_loss = self.run_phase(("behavior",), behavior, optimizer, self.step_on_loss)
        return {"train/iit_loss": iit_loss, "train/behavior_loss": behavior_loss}

    def run_eval_step(self, base_input, ablation_input, loss_fn):
        atol = self.training_args["atol"]
        hl_node = self.sample_hl_name()
        hl_output, ll_output = self.do_intervention(base_input, ablation_input, hl_node)
        loss = loss_fn(ll_output, hl_output)
        if self._categorical():
            top1 = torch.argmax(ll_output, dim=-1)
            iia = (top1 == labels_of(hl_output, ll_output)).float().mean()
        else:
            iia = ((ll_output - hl_output).abs() < atol).float().mean()
        base_x, base_y = base_input[0], base_input[1]
        output = self.ll_forward(base_x)
        if self._categorical():
            accuracy = (torch.argmax(output, dim=-1) == labels_of(base_y, output)).float().mean()
        else:
            accuracy = ((output.squeeze() - base_y).abs() < atol).float().mean()
        return {"val/iit_loss": loss.detach(), "val/IIA": iia, "val/accuracy": accuracy}
