"""Linear probes from LL node activations to HL intermediate variables.

Parity: ``/root/reference/iit/utils/probes.py:8-132``.  A probe is a bias-free
``nn.Linear`` from the flattened node activation (``cache[name][index]``) to the
HL node's ``num_classes``; ground truth comes from
``hl_model.get_idx_to_intermediate(name)(int_vars)``.  Probe GEMMs are plain
library GEMMs (hipBLASLt via torch), SURVEY.md §2.3 K22.

On native LL models the activations are gathered with a capture-only plan (only
the probed hooks, forward truncated after the deepest), instead of caching every
hook of a full forward.
"""
from __future__ import annotations

from typing import Dict, Iterable, List, Optional

import os

import torch
import torch.nn as nn

from ..config import DEVICE
from ..core.nodes import HLNode, LLNode


def _nodes(v) -> List[LLNode]:
    return [v] if isinstance(v, LLNode) else list(v)


def capture_hooks(ll_model, x: torch.Tensor, names: Iterable[str], reference: bool = False) -> Dict[str, torch.Tensor]:
    """The named hook activations of ``ll_model`` on ``x``: a capture-only plan run (only those hooks, stopped
    after the last one) on a plan-capable model, else -- or with ``reference`` -- ``run_with_cache``."""
    names = sorted(set(names))
    if not reference and (getattr(ll_model, "supports_run_plan", False) or hasattr(ll_model, "run_capture")):
        return ll_model.run_capture(x, names)
    _, cache = ll_model.run_with_cache(x, names_filter=lambda n: n in names)
    return cache


def _reference(model_pair) -> bool:
    return getattr(model_pair, "training_args", {}).get("engine", "native") == "reference"


def construct_probe(high_level_node: HLNode, ll_nodes, dummy_cache, bias: bool = False) -> nn.Linear:
    nodes = _nodes(ll_nodes)
    if len(nodes) > 1:
        raise NotImplementedError("probing a union of LL nodes is not supported")
    size = sum(dummy_cache[n.name][n.index.as_index].flatten().shape[0] for n in nodes)
    return nn.Linear(size, high_level_node.num_classes, bias=bias).to(DEVICE)


def construct_probes(model_pair, input_shape, bias: bool = False, input_dtype: Optional[torch.dtype] = None):
    dtype = input_dtype
    if dtype is None:
        # token models (hooked transformer / encoder) take ids; wrapped CNNs (also plan-capable) take images
        dtype = torch.long if hasattr(model_pair.ll_model, "cfg") else torch.float32
    names = [n.name for v in model_pair.corr.values() for n in _nodes(v)]
    with torch.no_grad():
        dummy = capture_hooks(model_pair.ll_model, torch.zeros(input_shape, dtype=dtype, device=DEVICE), names)
    return {hl.name: construct_probe(hl, lls, dummy, bias=bias) for hl, lls in model_pair.corr.items()}


def _batches(dataset, batch_size: int, shuffle: bool, num_workers: int = 0):
    """``(x, y, int_vars)`` batches; device-side ``gather`` when the dataset supports it (no per-item Python)."""
    gather = getattr(dataset, "gather", None)
    if gather is not None:
        n = len(dataset)
        order = torch.randperm(n) if shuffle else torch.arange(n)
        order = order.to(DEVICE)
        for s in range(0, n, batch_size):
            yield gather(order[s:s + batch_size])
        return
    yield from torch.utils.data.DataLoader(dataset, batch_size=batch_size, shuffle=shuffle, num_workers=num_workers)


def _num_batches(dataset, batch_size: int) -> int:
    return (len(dataset) + batch_size - 1) // batch_size


def probe_logits(probe: nn.Linear, cache, ll_node: LLNode) -> torch.Tensor:
    act = cache[ll_node.name][ll_node.index.as_index]
    return probe(act.reshape(-1, probe.weight.shape[1]).to(probe.weight.dtype))


class ActivationBank:
    """Every named hook's activation for every sample of ``dataset`` (natural order, captured in batches of ``bs``
    with one truncated forward per batch) plus the samples' intermediate variables: the probe sweeps of
    ``eval_information`` then train and evaluate every hook point's probes from gathers of these tensors instead of
    one forward per (hook point, batch) -- and per probe, on the evaluation side.  The batches the probes see are the
    same draws as the per-batch path (the same ``randperm`` per epoch / per probe)."""

    def __init__(self, ll_model, dataset, names, bs: int = 1024):
        n = len(dataset)
        names = sorted(set(names))
        parts = {nm: [] for nm in names}
        ivs = []
        with torch.no_grad():
            for s0 in range(0, n, bs):
                x, _, iv = dataset.gather(torch.arange(s0, min(n, s0 + bs), device=DEVICE))
                cache = capture_hooks(ll_model, x, names)
                for nm in names:
                    parts[nm].append(cache[nm])
                ivs.append(iv)
        self.n = n
        self.acts = {nm: torch.cat(v) for nm, v in parts.items()}
        self.iv = torch.cat(ivs)

    @staticmethod
    def estimate_bytes(ll_model, dataset, names, sample: int = 2) -> int:
        """Bytes the bank of ``names`` over ``dataset`` would hold: one capture of ``sample`` rows, scaled."""
        n = len(dataset)
        k = max(1, min(sample, n))
        with torch.no_grad():
            x, _, iv = dataset.gather(torch.arange(0, k, device=DEVICE))
            cache = capture_hooks(ll_model, x, sorted(set(names)))
            per = sum(cache[nm].element_size() * cache[nm].numel() for nm in set(names)) + iv.element_size() * iv.numel()
        return per * n // k

    @staticmethod
    def budget_bytes() -> int:
        """Device memory a bank may take: ``IIT_PROBE_BANK_GB``, else half of the currently free device memory
        (host: 8 GB)."""
        env = os.environ.get("IIT_PROBE_BANK_GB")
        if env:
            return int(float(env) * (1 << 30))
        if torch.cuda.is_available():
            free, _total = torch.cuda.mem_get_info()
            return free // 2
        return 8 << 30

    @classmethod
    def fits(cls, ll_model, datasets, names) -> bool:
        """Whether banks over every dataset of ``datasets`` fit the budget together (a full 60k MNIST-PVR
        sweep of every hook point needs tens of GB -- above the budget the per-batch path runs instead)."""
        need = sum(cls.estimate_bytes(ll_model, d, names) for d in datasets)
        ok = need <= cls.budget_bytes()
        if not ok:
            print(f"[iit probes] activation bank would take {need / 2**30:.1f} GB (budget "
                  f"{cls.budget_bytes() / 2**30:.1f} GB): per-batch capture instead")
        return ok

    def batch(self, idx: torch.Tensor, names):
        return {nm: self.acts[nm].index_select(0, idx) for nm in names}, self.iv.index_select(0, idx)


def train_probes_on_model_pair(model_pair, input_shape, train_set, training_args: dict,
                               bank: Optional[ActivationBank] = None):
    probes = construct_probes(model_pair, input_shape=input_shape)
    params = [p for probe in probes.values() for p in probe.parameters()]
    for probe in probes.values():
        probe.train()
    opt = torch.optim.Adam(params, lr=training_args["lr"])
    criterion = nn.CrossEntropyLoss()
    losses = {k: [] for k in probes}
    accs = {k: [] for k in probes}
    bs = training_args["batch_size"]
    names = [n.name for v in model_pair.corr.values() for n in _nodes(v)]
    for _ in range(training_args["epochs"]):
        loss_run = {k: torch.zeros((), device=DEVICE) for k in probes}
        acc_run = {k: torch.zeros((), device=DEVICE) for k in probes}
        if bank is not None:  # the same randperm draw as _batches, the activations gathered from the bank
            order = torch.randperm(bank.n).to(DEVICE)
            batches = (bank.batch(order[s0:s0 + bs], names) for s0 in range(0, bank.n, bs))
        else:
            batches = ((None, b[2], b[0]) for b in _batches(train_set, bs, True, training_args.get("num_workers", 0)))
        for item in batches:
            if bank is not None:
                cache, int_vars = item
            else:
                _, int_vars, x = item
                with torch.no_grad():
                    cache = capture_hooks(model_pair.ll_model, x.to(DEVICE), names, _reference(model_pair))
            opt.zero_grad()
            total = 0
            for hl_name, probe in probes.items():
                gt = model_pair.hl_model.get_idx_to_intermediate(hl_name)(int_vars.to(DEVICE)).to(DEVICE)
                for node in _nodes(model_pair.corr[hl_name]):
                    out = probe_logits(probe, cache, node)
                    l = criterion(out, gt)
                    total = total + l
                    loss_run[hl_name] += l.detach()
                    acc_run[hl_name] += (out.argmax(1) == gt).float().mean()
            total.backward()
            opt.step()
        n = max(1, _num_batches(train_set, bs))
        for k in probes:
            losses[k].append(float(loss_run[k]) / n)
            accs[k].append(float(acc_run[k]) / n)
    return {"probes": probes, "loss": losses, "accuracy": accs}


def _evaluate_probes_cached(probes, model_pair, test_set, criterion, bs: int = 256,
                            bank: Optional[ActivationBank] = None):
    """:func:`evaluate_probe` with ONE capture pass over the test set for all probes: the probed activations of every
    sample are captured once (natural order, the evaluation's batch size) and each probe then walks its own shuffled
    batches over them -- the same ``randperm`` draw per probe as the per-probe loop, so the same batches -- instead of
    a truncated forward per (probe, batch): 4-12x fewer forwards per hook point on the PVR sweeps."""
    n = len(test_set)
    nodes = {hl: _nodes(v) for hl, v in model_pair.corr.items()}
    if any(len(v) != 1 for v in nodes.values()):
        raise NotImplementedError("probing a union of LL nodes is not supported")
    names = sorted({v[0].name for v in nodes.values()})
    if bank is None:
        bank = ActivationBank(model_pair.ll_model, test_set, names, bs)
    with torch.no_grad():
        ivs = bank.iv
        acts = {}
        for hl in probes:
            node = nodes[hl][0]
            acts[hl] = bank.acts[node.name][node.index.as_index].reshape(n, -1)
    stats = {"test loss": {}, "test accuracy": {}}
    nb = max(1, _num_batches(test_set, bs))
    for hl_name, probe in probes.items():
        probe.eval()
        loss = torch.zeros((), device=DEVICE)
        acc = torch.zeros((), device=DEVICE)
        order = torch.randperm(n).to(DEVICE)  # the per-probe loop's shuffle draw
        to_gt = model_pair.hl_model.get_idx_to_intermediate(hl_name)
        with torch.no_grad():
            for s0 in range(0, n, bs):
                idx = order[s0:s0 + bs]
                out = probe(acts[hl_name].index_select(0, idx).to(probe.weight.dtype))
                gt = to_gt(ivs.index_select(0, idx)).to(DEVICE)
                loss += criterion(out, gt)
                acc += (out.argmax(1) == gt).float().mean()
        stats["test loss"][hl_name] = float(loss) / nb
        stats["test accuracy"][hl_name] = float(acc) / nb
    return stats


def evaluate_probe(probes, model_pair, test_set, criterion, bank: Optional[ActivationBank] = None):
    if not _reference(model_pair) and getattr(test_set, "gather", None) is not None and \
            getattr(model_pair.ll_model, "supports_run_plan", False):
        return _evaluate_probes_cached(probes, model_pair, test_set, criterion, bank=bank)
    stats = {"test loss": {}, "test accuracy": {}}
    names = [n.name for v in model_pair.corr.values() for n in _nodes(v)]
    for hl_name, probe in probes.items():
        probe.eval()
        loss = torch.zeros((), device=DEVICE)
        acc = torch.zeros((), device=DEVICE)
        with torch.no_grad():
            for x, y, int_vars in _batches(test_set, 256, True):
                cache = capture_hooks(model_pair.ll_model, x.to(DEVICE), names, _reference(model_pair))
                gt = model_pair.hl_model.get_idx_to_intermediate(hl_name)(int_vars.to(DEVICE)).to(DEVICE)
                for node in _nodes(model_pair.corr[hl_name]):
                    out = probe_logits(probe, cache, node)
                    loss += criterion(out, gt)
                    acc += (out.argmax(1) == gt).float().mean()
        n = max(1, _num_batches(test_set, 256))
        stats["test loss"][hl_name] = float(loss) / n
        stats["test accuracy"][hl_name] = float(acc) / n
    return stats
