"""IIT + linear probes, trained sequentially (``/root/reference/iit/model_pairs/probed_sequential_pair.py:5-196``).

The reference class is broken (wrong metric keys, ``make_loaders``
called with 2 of 4 args, ``output["accuracy"]``).  This implements the evident
semantics: per batch one IIT optimizer step, then a second forward of the base
input whose behaviour loss + ``probe_weight`` x probe loss (on *detached* node
activations, as TL caches are) updates LL params and probes together.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn.functional as F

from ..core.metric import MetricStore, MetricStoreCollection, MetricType
from ..engine.plan import RunPlan
from ..parallel import dist as pdist
from ..utils.probes import _nodes, construct_probes, probe_logits
from ..utils.progress import progress
from ..utils.sinks import make_sink
from .iit_model_pair import IITModelPair, labels_of


class IITProbeSequentialPair(IITModelPair):
    def __init__(self, hl_model=None, ll_model=None, hl_graph=None, corr=None, seed: int = 0, training_args=None):
        super().__init__(hl_model, ll_model, hl_graph, corr, seed, training_args)
        defaults = {"batch_size": 256, "lr": 0.001, "num_workers": 0, "probe_weight": 1.0}
        self.training_args = {**self.training_args, **defaults, **(training_args or {})}

    def _forward_with_cache(self, x):
        names = [n.name for v in self.corr.values() for n in _nodes(v)]
        model = self.ll_model
        if getattr(model, "supports_run_plan", False):
            plan = RunPlan(capture={n: None for n in names}, logits=self.ll_logits_mode())
            out = model(x, plan=plan)
            return out, plan.cache
        return model.run_with_cache(x)

    def _probe_losses(self, probes, cache, int_vars, loss_fn):
        total = 0
        accs = []
        for hl_name, probe in probes.items():
            gt = self.hl_model.get_idx_to_intermediate(hl_name)(int_vars)
            nodes = _nodes(self.corr[hl_name])
            if len(nodes) > 1:
                raise NotImplementedError
            out = probe_logits(probe, cache, nodes[0])
            total = total + loss_fn(out, gt)
            accs.append((out.argmax(1) == gt).float().mean())
        return total, torch.stack(accs).mean() if accs else torch.zeros(())

    def run_train_step(self, base_input, ablation_input, loss_fn, optimizer, probes=None, probe_optimizer=None,
                       training_args=None):
        training_args = training_args or self.training_args
        iit_loss = super().run_train_step(base_input, ablation_input, loss_fn, optimizer)["train/iit_loss"]
        if probes is None:
            return {"train/iit_loss": iit_loss}
        probe_optimizer.zero_grad()
        for p in probes.values():
            p.train()
        base_x, base_y, base_iv = base_input
        out, cache = self._forward_with_cache(base_x)
        probe_loss, _ = self._probe_losses(probes, cache, base_iv, loss_fn)
        behavior_loss = loss_fn(out, base_y)
        loss = behavior_loss + training_args["probe_weight"] * probe_loss
        self.backward(loss)
        probe_optimizer.step()
        return {"train/iit_loss": iit_loss, "train/probe_loss": probe_loss.detach(),
                "train/behavior_loss": behavior_loss.detach()}

    def train(self, dataset, test_dataset, epochs: int = 1000, use_wandb: bool = False, **_):
        args = self.training_args
        sample_x = dataset[0][0][0]
        probes = construct_probes(self, tuple(sample_x.unsqueeze(0).shape), input_dtype=sample_x.dtype)
        loader, test_loader = self.make_loaders(dataset, test_dataset, args["batch_size"], args["num_workers"])
        ll_params = list(self._ll_module().parameters())
        probe_optimizer = torch.optim.Adam(ll_params + [p for pr in probes.values() for p in pr.parameters()],
                                           lr=args["lr"])
        optimizer = torch.optim.Adam(ll_params, lr=args["lr"])
        self._setup_reducer(optimizer)
        loss_fn = torch.nn.CrossEntropyLoss()
        sink = make_sink(use_wandb and pdist.is_main(), project="iit", config={"method": "IIT + Probes (Sequential)"})
        self.probes = probes
        history = []
        for epoch in progress(range(epochs), disable=not pdist.is_main()):
            self._ll_module().train()
            tr = {"iit": [], "probe": [], "behavior": []}
            for base_input, ablation_input in loader:
                r = self.run_train_step(base_input, ablation_input, loss_fn, optimizer, probes, probe_optimizer, args)
                tr["iit"].append(r["train/iit_loss"])
                tr["probe"].append(r["train/probe_loss"])
                tr["behavior"].append(r["train/behavior_loss"])
            self._ll_module().eval()
            te = {"loss": [], "acc": [], "probe_acc": [], "probe_loss": [], "beh_acc": []}
            with torch.no_grad():
                for p in probes.values():
                    p.eval()
                for base_input, ablation_input in test_loader:
                    out = self.run_eval_step(base_input, ablation_input, loss_fn)
                    te["acc"].append(out["val/accuracy"])
                    te["loss"].append(out["val/iit_loss"])
                    base_x, base_y, base_iv = base_input
                    o, cache = self._forward_with_cache(base_x)
                    te["beh_acc"].append((torch.argmax(o, dim=-1) == labels_of(base_y, o)).float().mean())
                    pl, pa = self._probe_losses(probes, cache, base_iv, loss_fn)
                    te["probe_loss"].append(pl / max(1, len(probes)))
                    te["probe_acc"].append(pa)
            row = {k: float(torch.stack([torch.as_tensor(v, dtype=torch.float32) for v in vs]).mean())
                   for k, vs in {**{f"train_{k}": v for k, v in tr.items()}, **{f"test_{k}": v for k, v in te.items()}}.items() if vs}
            history.append(row)
            if pdist.is_main():
                print(f"Epoch {epoch}: " + ", ".join(f"{k}={v:.4f}" for k, v in row.items()))
            if sink is not None:
                sink.log({"epoch": epoch, **row})
        self.history = history
        return history
