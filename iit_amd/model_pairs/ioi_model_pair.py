"""IOI specialisation of strict IIT (parity: ``/root/reference/iit/model_pairs/ioi_model_pair.py:11-171``).

* IIT target: ``argmax(hl_out[:, -1])`` against ``ll_out[:, -1]`` (the reference's
  soft one-hot CE is exactly index CE, so no ``[B, V]`` one-hot is built);
* strict / behaviour losses read only position -1 (``next_token=False``), so the
  native engine computes last-position logits only and the IOI HL model runs in
  ``last_only`` mode (no ``[B, S, V]`` fp32 tensors in training);
* eval: IIA at the last position, behaviour accuracy and per-position accuracy
  (the latter via a fused unembed+argmax, never materialising full logits on GPU).

Q2 fixed: ``next_token`` is read from the merged training args (same default
``False``, so default behaviour is identical).  With ``next_token=True`` the loss
is the intended per-position CE with weight 10 on the last position.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn.functional as F
from torch import Tensor

from ..config import DEVICE
from ..core import index as index_mod
from ..core.metric import MetricStore, MetricStoreCollection, MetricType, PerTokenMetricStore
from .base_model_pair import _ll_nodes_of
from .strict_iit_model_pair import StrictIITModelPair


def _last(t: Tensor, seq_dim_present: bool) -> Tensor:
    return t[:, -1] if seq_dim_present else t


class IOI_ModelPair(StrictIITModelPair):
    def __init__(self, hl_model, ll_model, corr, training_args=None):
        super().__init__(hl_model, ll_model, corr, training_args=training_args)
        defaults = {"next_token": False, "non_ioi_thresh": 0.65, "use_per_token_check": False}
        self.training_args = {**defaults, **self.training_args}
        self.next_token = bool(self.training_args["next_token"])

    # ------------------------------------------------------------------ modes
    def ll_logits_mode(self) -> str:
        return "full" if (self.next_token or not self.native()) else "last"

    def hl_run_kwargs(self):
        if self.native() and not self.next_token and getattr(self.hl_model, "supports_last_only", False):
            return {"last_only": True}
        return {}

    # ------------------------------------------------------------------ loss
    @property
    def loss_fn(self):
        if self._loss_fn_override is not None:
            return self._loss_fn_override
        return self.per_token_weighted_cross_entropy

    @loss_fn.setter
    def loss_fn(self, value):
        self._loss_fn_override = value

    def per_token_weighted_cross_entropy(self, output: Tensor, target: Tensor) -> Tensor:
        output = output.float()
        if output.dim() == 2:
            # last-position logits [B, V]; target may be [B], [B, V] probs, [B, S] ids or [B, S, V] probs
            if target.dim() == 3 or (target.dim() == 2 and not target.dtype.is_floating_point):
                target = target[:, -1]
            if target.dtype.is_floating_point and target.dim() == 2:
                target = target.argmax(-1) if bool((target.sum(-1) == 1).all()) else target
            if not target.dtype.is_floating_point:
                from ..ops import cross_entropy
                return cross_entropy(output, target)
            return F.cross_entropy(output, target)
        if self.next_token:
            B, S, V = output.shape
            if target.dtype.is_floating_point:
                per = -(target * F.log_softmax(output, -1)).sum(-1)
            else:
                per = F.cross_entropy(output.reshape(B * S, V), target.reshape(B * S), reduction="none").view(B, S)
            w = torch.ones(S, device=output.device)
            w[-1] = 10
            return (per * w).sum() / (w.sum() * B)
        return F.cross_entropy(output[:, -1, :], target[:, -1])

    @staticmethod
    def get_label_idxs():
        return index_mod.Ix[:, -1]

    @staticmethod
    def make_test_metrics():
        return MetricStoreCollection([
            MetricStore("val/iit_loss", MetricType.LOSS),
            MetricStore("val/IIA", MetricType.ACCURACY),
            MetricStore("val/accuracy", MetricType.ACCURACY),
            PerTokenMetricStore("val/per_token_accuracy"),
        ])

    @staticmethod
    def _hl_label(hl_output: Tensor) -> Tensor:
        return torch.argmax(hl_output[:, -1] if hl_output.dim() == 3 else hl_output, dim=-1)

    def fast_hl_label(self, base_x: Tensor, ablation_x: Tensor, hl_node):
        """The intervened IOI HL label ``argmax(hl_out[:, -1])`` in one kernel launch (csrc/ioi_hl.hip) instead of
        two HL forwards and a [B, V] argmax; None when not applicable (another HL model, live hooks on it, CPU
        tensors, ``training_args["fast_hl"] = False``)."""
        from ..tasks.ioi.ioi_hl import IOI_HL
        hl = self.hl_model
        if not (self.native() and self.training_args.get("fast_hl", True) and type(hl) is IOI_HL
                and base_x.is_cuda and base_x.dtype == torch.long and ablation_x.dtype == torch.long):
            return None
        from ..ops import hip_kernels as K
        node = K.IOI_HL_NODES.get(hl_node.name)
        if node is None or not (hl_node.index is None or hl_node.index.is_everything()):
            return None
        if base_x.dim() != 2 or base_x.shape != ablation_x.shape or base_x.shape[1] > 64:
            return None
        if any(hp.is_live for hp in hl.hook_dict.values()):
            return None
        nm = hl.name_mover_head
        table = nm.name_table
        if table.device != base_x.device:
            table = nm.name_table = table.to(base_x.device)
        out = torch.empty(base_x.shape[0], dtype=torch.long, device=base_x.device)
        K.ioi_hl_label(base_x.contiguous(), ablation_x.contiguous(), table, nm.d_vocab_out, node, out)
        return out

    def _label_and_ll(self, base_input, ablation_input, hl_node):
        """(IIT label [B], LL output) of one interchange intervention."""
        label = self.fast_hl_label(base_input[0], ablation_input[0], hl_node)
        if label is None:
            hl_output, ll_output = self.do_intervention(base_input, ablation_input, hl_node)
            return self._hl_label(hl_output), ll_output
        return label, self.ll_intervention(base_input[0], ablation_input[0], _ll_nodes_of(self.corr, hl_node))

    def get_IIT_loss_over_batch(self, base_input, ablation_input, hl_node, loss_fn):
        hl_label, ll_output = self._label_and_ll(base_input, ablation_input, hl_node)
        ll_last = ll_output[:, -1] if ll_output.dim() == 3 else ll_output
        return loss_fn(ll_last, hl_label)

    # ------------------------------------------------------------------ eval
    def run_eval_step(self, base_input, ablation_input, loss_fn):
        hl_node = self.sample_hl_name()
        hl_label, ll_output = self._label_and_ll(base_input, ablation_input, hl_node)
        ll_last = ll_output[:, -1] if ll_output.dim() == 3 else ll_output
        loss = loss_fn(ll_last, hl_label)
        iia = (torch.argmax(ll_last, dim=-1) == hl_label).float().mean()
        base_x, base_y = base_input[0], base_input[1]
        top1 = self.ll_forward(base_x, logits="argmax")  # [B, S]
        if base_y.dtype.is_floating_point and base_y.dim() == 3:
            base_y = torch.argmax(base_y, dim=-1)
        per_token = (top1 == base_y).float().mean(dim=0)
        accuracy = per_token.mean() if self.next_token else per_token[-1]
        return {"val/iit_loss": loss.detach(), "val/IIA": iia, "val/accuracy": accuracy,
                "val/per_token_accuracy": per_token}

    # ------------------------------------------------------------------ early stop
    @staticmethod
    def _check_early_stop_fn(test_metrics, verbose: bool = False, non_ioi_thresh: float = 0.65,
                             use_per_token_check: bool = False) -> bool:
        say = print if verbose else (lambda *a, **k: None)
        for metric in test_metrics:
            if metric.get_name() == "val/IIA" and metric.get_value() < 100:
                say(f"IIA is not enough: {metric.get_value()}")
                return False
            if metric.get_name() == "val/per_token_accuracy":
                acc = np.asarray(metric.get_value())
                if acc[-1] < 1:
                    say(f"per_token_acc at IOI index is not enough: {acc[-1]}")
                    return False
                if np.mean(acc) < non_ioi_thresh:
                    say(f"mean per_token_acc is not enough: {np.mean(acc)}")
                    return False
                if use_per_token_check:
                    for i, a in enumerate(acc):
                        if i in (2, 4, 5, 8, 10, 13):
                            continue
                        if a < non_ioi_thresh:
                            say(f"per_token_acc at {i} is not enough: {a}")
                            return False
        return True

    def _check_early_stop_condition(self, *args, **kwargs):
        if not self.training_args["next_token"]:
            return super()._check_early_stop_condition(*args, **kwargs)
        return self._check_early_stop_fn(*args, **kwargs, non_ioi_thresh=self.training_args["non_ioi_thresh"],
                                         use_per_token_check=self.training_args["use_per_token_check"])
