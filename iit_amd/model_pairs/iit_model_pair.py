"""Vanilla IIT pair (parity: ``/root/reference/iit/model_pairs/iit_model_pair.py:6-99``).

One IIT loss per batch, CE loss, Adam lr 1e-3, ReduceLROnPlateau on
``val/accuracy``.  Kept quirk Q5: ``clip_grad_norm`` is a default but this pair's
train step does not clip.  Fixed quirk Q4: the ``loss_fn`` setter works.
"""
from __future__ import annotations

from typing import Callable

import numpy as np
import torch
from torch import Tensor

from ..core.metric import MetricStore, MetricStoreCollection, MetricType
from .base_model_pair import BaseModelPair


def labels_of(target: Tensor, like: Tensor) -> Tensor:
    """Index labels from either index or one-hot / probability targets."""
    if target.dtype.is_floating_point and target.shape == like.shape:
        return target.argmax(dim=-1)
    return target


class IITModelPair(BaseModelPair):
    def __init__(self, hl_model=None, ll_model=None, hl_graph=None, corr=None, seed: int = 0, training_args=None):
        corr = {} if corr is None else corr
        training_args = {} if training_args is None else training_args
        if hl_model is None:
            if hl_graph is None:
                raise AssertionError("either hl_model or hl_graph is required")
            hl_model = self.make_hl_model(hl_graph)
        self.hl_model = hl_model
        self.ll_model = ll_model
        self.hl_model.requires_grad_(False)
        self.corr = corr
        missing = [str(k) for k in corr.keys() if str(k) not in self.hl_model.hook_dict]
        if missing:
            raise AssertionError(f"correspondence keys {missing} are not hooks of the HL model")
        self.rng = np.random.default_rng(seed)
        defaults = {
            "batch_size": 256,
            "lr": 0.001,
            "num_workers": 0,
            "early_stop": True,
            "lr_scheduler": torch.optim.lr_scheduler.ReduceLROnPlateau,
            "scheduler_val_metric": "val/accuracy",
            "scheduler_mode": "max",
            "clip_grad_norm": 1.0,
        }
        self.training_args = {**defaults, **training_args}
        self.wandb_method = "iit"
        self._loss_fn_override = None

    @property
    def loss_fn(self) -> Callable[[Tensor, Tensor], Tensor]:
        if self._loss_fn_override is not None:
            return self._loss_fn_override
        return torch.nn.CrossEntropyLoss()

    @loss_fn.setter
    def loss_fn(self, value):
        self._loss_fn_override = value

    @staticmethod
    def make_train_metrics():
        return MetricStoreCollection([MetricStore("train/iit_loss", MetricType.LOSS)])

    @staticmethod
    def make_test_metrics():
        return MetricStoreCollection([
            MetricStore("val/iit_loss", MetricType.LOSS),
            MetricStore("val/accuracy", MetricType.ACCURACY),
        ])

    def run_eval_step(self, base_input, ablation_input, loss_fn):
        hl_node = self.sample_hl_name()
        hl_output, ll_output = self.do_intervention(base_input, ablation_input, hl_node)
        loss = loss_fn(ll_output, hl_output)
        top1 = torch.argmax(ll_output, dim=-1)
        accuracy = (top1 == labels_of(hl_output, ll_output)).float().mean()
        return {"val/iit_loss": loss.detach(), "val/accuracy": accuracy}

    def _plain_step(self, loss, optimizer) -> None:
        """zero_grad -> backward -> step (no clipping: reference ``iit_model_pair.py:85-99``)."""
        optimizer.zero_grad()
        self.backward(loss)
        self.optimizer_step(optimizer)

    def run_train_step(self, base_input, ablation_input, loss_fn, optimizer):
        hl_node = self.sample_hl_name()
        loss = self.run_phase(("iit", hl_node.name),
                              lambda: self.get_IIT_loss_over_batch(base_input, ablation_input, hl_node, loss_fn),
                              optimizer, self._plain_step)
        return {"train/iit_loss": loss}
