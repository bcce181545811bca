"""Post-training circuit verification sweeps (parity: ``/root/reference/iit/utils/eval_ablations.py:15-352``).

For every candidate LL node (all / in-circuit / not-in-circuit, via
:mod:`iit_amd.utils.node_picker`):

* **resample ablation** — patch the node's activation from the source input
  into the base run and score the change against the HL's *base* output:
  KL(HL_base || LL_patched) at the label index (default) or, with
  ``Categorical_Metric.ACCURACY``, the fraction of label-changing pairs whose
  prediction flipped away from the HL base label; regression HL: fraction of
  label-changing pairs whose output moved by more than ``atol``;
* **mean / zero ablation** — replace the node by its dataset mean (or 0) and count
  the fraction of correctly-predicted base inputs whose prediction flips.

MI355X-native execution: with a plan-capable LL model each batch costs ONE
truncated source capture of every candidate node's hook (the reference re-runs
the source forward for every node), ONE HL base output and -- for mean / zero
ablation -- ONE unablated base forward, all shared by the node loop; each node is
then a single spliced forward (:class:`iit_amd.engine.plan.RunPlan`: in-kernel or
patch-spec-kernel splices, a broadcast mean as the source), computing only the
logits the metric reads, with scores accumulated on device (one host read per
sweep instead of one per node per batch).  Nodes whose hook lies in the same
block share ONE forward over stacked copies of the batch (M = nodes x B rows,
resumed from the base run's residual at that block; ``_RowGroupSplice`` splices
each node into its own rows), and each sweep's per-batch body is one HIP graph
replay (``_SweepGraph``).  The scores equal the per-node reference-semantics path
(tests/test_eval_ablations.py: bit for bit per node, within fp rounding for the
grouped forwards).  Any other LL model takes the reference hook path.
"""
from __future__ import annotations

import os
from enum import Enum
from typing import Callable, Dict, Optional

import torch

from ..core.index import EVERYTHING, TorchIndex
from ..core.nodes import LLNode
from ..engine.plan import RunPlan
from ..hooks.hook_points import HookPoint
from .eval_metrics import kl_div, kl_div_from_stats, target_stats
from .node_picker import get_all_nodes, get_nodes_in_circuit, get_nodes_not_in_circuit
from .progress import progress


class Categorical_Metric(Enum):
    ACCURACY = 1
    KL = 2


# ----------------------------------------------------------------------------- helpers
def _native(model_pair) -> bool:
    return model_pair.native() if hasattr(model_pair, "native") else False


def _reduced_logits(model_pair) -> bool:
    """LL outputs are already at the label position ([B, V]) in the native IOI mode."""
    return _native(model_pair) and model_pair.ll_logits_mode() == "last"


def _at(out: torch.Tensor, label_idx: TorchIndex, reduced: bool) -> torch.Tensor:
    return out if reduced else out[label_idx.as_index]


def _hl_out(model_pair, base_in):
    kw = model_pair.hl_run_kwargs() if hasattr(model_pair, "hl_run_kwargs") else {}
    with torch.no_grad():
        out = model_pair.hl_model(base_in, **kw)
    return out, bool(kw.get("last_only", False))


def _labels_at(y: torch.Tensor, label_idx: TorchIndex) -> torch.Tensor:
    if y.dtype.is_floating_point:
        y = torch.argmax(y, dim=-1)
    return y[label_idx.as_index]


def _nodes(model_pair, node_type: str, with_suffixes: bool = False):
    assert node_type in ["a", "c", "n"], "type must be one of 'a', 'c', or 'n'"
    if node_type == "n":
        return get_nodes_not_in_circuit(model_pair.ll_model, model_pair.corr)
    if node_type == "c":
        return get_nodes_in_circuit(model_pair.corr)
    if with_suffixes:
        return get_all_nodes(model_pair.ll_model, model_pair.corr.get_suffixes())
    return get_all_nodes(model_pair.ll_model)


# ----------------------------------------------------------------------------- resample ablation
def do_intervention(model_pair, base_input, ablation_input, node: LLNode, hooker: Optional[Callable] = None):
    """LL output on ``base_input`` with ``node`` patched from ``ablation_input`` (``eval_ablations.py:20-32``)."""
    if _native(model_pair):
        with torch.no_grad():
            model_pair.ll_cache = model_pair.ll_source_cache(ablation_input, [node])
            return model_pair.ll_intervened_forward(base_input, [node])
    _, cache = model_pair.ll_model.run_with_cache(ablation_input)
    model_pair.ll_cache = cache
    hooker = hooker or model_pair.make_ll_ablation_hook(node)
    return model_pair.ll_model.run_with_hooks(base_input, fwd_hooks=[(node.name, hooker)])


def _resample_score(model_pair, base_in, ablation_in, ll_out, base_hl_out, hl_reduced, atol: float = 5e-2,
                    verbose: bool = False, node=None, categorical_metric: Categorical_Metric = Categorical_Metric.KL,
                    hl_stats=None):
    base_y, ablation_y = base_in[1], ablation_in[1]
    reduced = _reduced_logits(model_pair)
    if model_pair.hl_model.is_categorical():
        label_idx = model_pair.get_label_idxs()
        label_unchanged = _labels_at(base_y, label_idx) == _labels_at(ablation_y, label_idx)
        ll_at = _at(ll_out, label_idx, reduced)
        hl_at = _at(base_hl_out.squeeze() if not hl_reduced else base_hl_out, label_idx, hl_reduced)
        if categorical_metric == Categorical_Metric.KL:
            if hl_stats is not None and ll_at.dim() == 2:  # batched sweep: the HL side computed once per batch
                score = kl_div_from_stats(ll_at, hl_stats).mean()
            else:
                score = kl_div(ll_at, hl_at, EVERYTHING).mean()
            if verbose:
                print(node, "kl base_hl vs ll_out:", float(score),
                      "fraction of labels changed:", float((~label_unchanged).float().mean()))
        else:
            ll_pred = torch.argmax(ll_at, dim=-1)
            hl_pred = torch.argmax(hl_at, dim=-1)
            changed = (~label_unchanged).float() * (ll_pred != hl_pred).float()
            score = changed.sum() / (~label_unchanged).float().sum()
    else:
        label_unchanged = base_y == ablation_y
        ll_unchanged = torch.isclose(ll_out.float().squeeze(), base_hl_out.float().to(ll_out.device).squeeze(),
                                     atol=atol)
        changed = (~label_unchanged).float().reshape(ll_unchanged.shape) * (~ll_unchanged).float()
        score = changed.sum() / (~label_unchanged).float().sum()
    return score.detach()


def resample_ablate_node(model_pair, base_in, ablation_in, node: LLNode, results: Dict, hooker: Optional[Callable] = None,
                         atol: float = 5e-2, verbose: bool = False,
                         categorical_metric: Categorical_Metric = Categorical_Metric.KL) -> None:
    """Adds this batch's score for ``node`` to ``results[node]`` (a device scalar; summed over batches)."""
    ll_out = do_intervention(model_pair, base_in[0], ablation_in[0], node, hooker)
    base_hl_out, hl_reduced = _hl_out(model_pair, base_in)
    results[node] = results[node] + _resample_score(model_pair, base_in, ablation_in, ll_out, base_hl_out, hl_reduced,
                                                    atol, verbose, node, categorical_metric)


_PREFIX = os.environ.get("IIT_EVAL_PREFIX", "1") != "0"


def _node_layer(name: str) -> Optional[int]:
    parts = name.split(".")
    if len(parts) >= 3 and parts[0] == "blocks" and parts[1].isdigit():
        return int(parts[1])
    return None


class _BasePrefix:
    """Shared prefix of a sweep's spliced forwards: a splice at a node of block L leaves blocks 0..L-1 of the base run
    unchanged, so the base residual entering every node's block is captured once per batch (one truncated
    capture-only forward) and each node's forward resumes there (``HookedTransformer.forward(start_at_layer=L)``):
    on average about half of the blocks per node are skipped.  ``IIT_EVAL_PREFIX=0`` runs every forward from the
    tokens."""

    def __init__(self, model_pair, base_x, nodes, src_x=None):
        """``src_x`` (optional, same shape as ``base_x``): also capture every node's hook on the source input in the
        SAME truncated forward (one capture over the stacked [base; source] rows instead of two forwards);
        ``self.src_cache`` then holds it ({} when not done -- the caller captures the source itself)."""
        self.model = model_pair.ll_model
        self.cache = {}
        self.src_cache = {}
        layers = sorted({L for L in (_node_layer(n.name) for n in nodes) if L})
        ok = (_PREFIX and layers and hasattr(self.model, "blocks") and getattr(self.model, "supports_run_plan", False)
              and "start_at_layer" in getattr(self.model.forward, "__code__", type("", (), {"co_varnames": ()})
                                              ).co_varnames)
        if ok:
            names = [f"blocks.{L}.hook_resid_pre" for L in layers]
            if (src_x is not None and isinstance(src_x, torch.Tensor) and isinstance(base_x, torch.Tensor)
                    and src_x.shape == base_x.shape and src_x.device == base_x.device):
                B = base_x.shape[0]
                src_names = sorted({n.name for n in nodes})
                cap = self.model.run_capture(torch.cat([base_x, src_x]), sorted(set(names) | set(src_names)))
                self.cache = {L: cap[n][:B] for L, n in zip(layers, names)}
                self.src_cache = {n: cap[n][B:] for n in src_names}
            else:
                cap = self.model.run_capture(base_x, names)  # ONE truncated forward for every block's residual
                self.cache = {L: cap[n] for L, n in zip(layers, names)}

        self.ok = bool(ok)

    def forward(self, base_x, node, plan):
        L = _node_layer(node.name)
        resid = self.cache.get(L) if L else None
        if resid is None:
            return self.model(base_x, plan=plan)
        # a copy: the resumed blocks must never see a buffer the next node at this layer reuses
        return self.model(resid.clone(), plan=plan, start_at_layer=L)

    def forward_rows(self, base_x, layer, n, plan):
        """One forward over ``n`` stacked copies of the base batch (rows ``[i B, (i+1) B)`` are copy ``i``),
        resumed at ``layer`` from the shared prefix when it is cached."""
        resid = self.cache.get(layer) if layer else None
        if resid is None:
            return self.model(base_x.repeat(n, *([1] * (base_x.dim() - 1))), plan=plan)
        return self.model(resid.repeat(n, *([1] * (resid.dim() - 1))), plan=plan, start_at_layer=layer)


class _RowGroupSplice:
    """The splices of one hook in a node-batched sweep forward: the activation holds ``n`` stacked copies of the base
    batch, and group ``(r0, r1, index, src)`` splices ``index`` from ``src`` (the node's B-row source or a broadcast
    [1, ...] value) into rows ``[r0, r1)`` only -- ``out[r0:r1][index] = src[index]``, the reference hook's semantics
    per copy (``/root/reference/iit/utils/eval_ablations.py:20-32``), one strided copy per node."""

    whole = False

    def __init__(self):
        self.groups = []

    def head_mask(self, n_heads: int):
        return None

    def apply(self, act: torch.Tensor) -> torch.Tensor:
        out = act.clone()
        for r0, r1, index, src in self.groups:
            view = out[r0:r1]
            if src.dtype != act.dtype or src.device != act.device:
                src = src.to(device=act.device, dtype=act.dtype)
            if src.shape != view.shape:
                src = src.expand_as(view)
            if index == EVERYTHING or index.is_everything():
                view.copy_(src)
            else:
                ix = index.on(act.device)
                view[ix] = src[ix]
        return out


_GROUP_ROWS = int(os.environ.get("IIT_EVAL_GROUP_ROWS", "131072"))


def _node_groups(model_pair, base_x, prefix: "_BasePrefix", nodes):
    """Node-batched sweep schedule: nodes whose hook lies in the same block share one forward
    of M = n x B rows (large GEMMs instead of n small ones), resumed from the shared base prefix at that block.
    Returns ``[(layer, [node positions])]`` plus the positions left to the per-node path.  ``IIT_EVAL_GROUP_ROWS``
    caps the token rows of one grouped forward (0 = per-node forwards only)."""
    if not prefix.ok or _GROUP_ROWS <= 0:
        return [], list(range(len(nodes)))
    per = base_x.numel()  # token rows of one copy of the batch
    cap = max(1, _GROUP_ROWS // max(per, 1))
    by_layer: Dict[int, list] = {}
    single = []
    for i, node in enumerate(nodes):
        L = _node_layer(node.name)
        if L is None or cap < 2:
            single.append(i)
        else:
            by_layer.setdefault(L, []).append(i)
    groups = []
    for L in sorted(by_layer):
        idx = by_layer[L]
        for k in range(0, len(idx), cap):
            chunk = idx[k:k + cap]
            if len(chunk) == 1:
                single.extend(chunk)
            else:
                groups.append((L, chunk))
    return groups, sorted(single)


def _group_plan(model_pair, nodes, positions, srcs, B: int) -> RunPlan:
    plan = RunPlan(logits=model_pair.ll_logits_mode())
    for i, p in enumerate(positions):
        node = nodes[p]
        spl = plan.splice.setdefault(node.name, [_RowGroupSplice()])[0]
        spl.groups.append((i * B, (i + 1) * B, node.index if node.index is not None else EVERYTHING, srcs[p]))
    return plan


def _resample_scores(model_pair, base_in, ablation_in, nodes, atol: float = 5e-2, verbose: bool = False,
                     categorical_metric: Categorical_Metric = Categorical_Metric.KL) -> torch.Tensor:
    """One batch of the native resample sweep: one source capture of every node's hook and one HL base output,
    then one spliced base forward per node; the scores as one device vector (node order)."""
    with torch.no_grad():
        base_x = base_in[0]
        prefix = _BasePrefix(model_pair, base_x, nodes, src_x=ablation_in[0])
        cache = prefix.src_cache or model_pair.ll_source_cache(ablation_in[0], nodes)
        model_pair.ll_cache = cache
        base_hl_out, hl_reduced = _hl_out(model_pair, base_in)
        scores = [None] * len(nodes)
        groups, single = _node_groups(model_pair, base_x, prefix, nodes)
        B = base_x.shape[0]
        stats = None
        if (categorical_metric == Categorical_Metric.KL and model_pair.hl_model.is_categorical()
                and _reduced_logits(model_pair) and hl_reduced and base_hl_out.dim() == 2):
            stats = target_stats(base_hl_out)  # the HL pmf side of every node's KL, once per batch
        for L, pos in groups:
            srcs = {p: cache[nodes[p].name] for p in pos}
            ll_all = prefix.forward_rows(base_x, L, len(pos), _group_plan(model_pair, nodes, pos, srcs, B))
            for i, p in enumerate(pos):
                scores[p] = _resample_score(model_pair, base_in, ablation_in, ll_all[i * B:(i + 1) * B], base_hl_out,
                                            hl_reduced, atol, verbose, nodes[p], categorical_metric,
                                            stats).float().reshape(())
        for p in single:
            node = nodes[p]
            plan = RunPlan.with_splices([(node.name, node.index, cache[node.name])],
                                        logits=model_pair.ll_logits_mode())
            ll_out = prefix.forward(base_x, node, plan)
            scores[p] = _resample_score(model_pair, base_in, ablation_in, ll_out, base_hl_out, hl_reduced, atol,
                                        verbose, node, categorical_metric, stats).float().reshape(())
        return torch.stack(scores)


def resample_ablate_nodes(model_pair, base_in, ablation_in, nodes, results: Dict, atol: float = 5e-2,
                          verbose: bool = False, categorical_metric: Categorical_Metric = Categorical_Metric.KL) -> None:
    """Native batched form of :func:`resample_ablate_node` over ``nodes`` (adds into ``results``)."""
    s = _resample_scores(model_pair, base_in, ablation_in, nodes, atol, verbose, categorical_metric)
    for i, node in enumerate(nodes):
        results[node] = results[node] + s[i]


_EVAL_GRAPHS_DEFAULT = "1"  # validated on MI355X in round 4 (tests/test_eval_graphs_gpu.py: graphed sweeps equal the eager ones)


class _SweepGraph:
    """A sweep's per-batch body (``fn(*batch) -> [n] scores``) run as ONE captured HIP graph per batch shape.

    The node loop of a sweep is a fixed kernel sequence for a given batch shape (one source capture, one HL
    forward, one spliced forward + score per node), so after one eager batch (settling lazily built state: GEMM
    decisions, weight mirrors) the body is captured with the batch in static buffers and the running sums
    accumulated in place on device; each later batch is a copy into the buffers and one replay -- no per-node
    Python or launch overhead (23 ms per spliced B=256 forward eagerly).  Sums are added in the
    same order as the eager loop, so the results are the eager ones bit for bit.  Batches of another shape (an
    epoch tail) and bodies that cannot be captured run eagerly into the same accumulator.  ``IIT_EVAL_GRAPHS=1|0``
    turns capture on / off."""

    def __init__(self, fn, n: int, device):
        self.fn = fn
        self.acc = torch.zeros(n, dtype=torch.float32, device=device)
        self.enabled = (device.type == "cuda" and torch.cuda.is_available()
                        and os.environ.get("IIT_EVAL_GRAPHS", _EVAL_GRAPHS_DEFAULT) == "1")
        self.static = None
        self.sig = None
        self.graph = None
        self.eager_runs = 0
        self.replays = 0

    @staticmethod
    def _flat(batch):
        return [t for part in batch for t in (part if isinstance(part, (tuple, list)) else (part,))
                if isinstance(t, torch.Tensor)]

    def _rebuild(self, batch, flat_static):
        it = iter(flat_static)
        out = []
        for part in batch:
            if isinstance(part, (tuple, list)):
                out.append(type(part)(next(it) if isinstance(t, torch.Tensor) else t for t in part))
            else:
                out.append(next(it) if isinstance(part, torch.Tensor) else part)
        return out

    def __call__(self, *batch) -> None:
        flat = self._flat(batch)
        sig = tuple((tuple(t.shape), t.dtype) for t in flat)
        if not self.enabled or (self.sig is not None and sig != self.sig):
            self.acc.add_(self.fn(*batch))
            return
        if self.static is None:
            self.static = [t.clone() for t in flat]
            self.sig = sig
        for d, s_ in zip(self.static, flat):
            d.copy_(s_, non_blocking=True)
        sbatch = self._rebuild(batch, self.static)
        if self.graph is None and self.eager_runs < 1:
            self.eager_runs += 1
            self.acc.add_(self.fn(*sbatch))
            return
        if self.graph is None:
            import gc
            from ..engine.graphs import _CAPTURE_MODE
            g = torch.cuda.CUDAGraph()
            gc.collect()
            try:
                with torch.cuda.graph(g, capture_error_mode=_CAPTURE_MODE):
                    self.acc.add_(self.fn(*sbatch))
            except Exception as e:  # noqa: BLE001 - not capturable: eager from now on
                print(f"[iit eval] sweep body not captured ({type(e).__name__}: {str(e)[:120]}); eager")
                torch.cuda.synchronize()
                self.enabled = False
                self.acc.add_(self.fn(*batch))
                return
            self.graph = g
        self.graph.replay()
        self.replays += 1

    def sums(self) -> torch.Tensor:
        return self.acc


def check_causal_effect(model_pair, dataset, batch_size: int = 256, node_type: str = "a", verbose: bool = False,
                        categorical_metric: Categorical_Metric = Categorical_Metric.KL) -> Dict[LLNode, float]:
    """Mean resample-ablation score per node over the dataset (``eval_ablations.py:128-161``)."""
    nodes = _nodes(model_pair, node_type)
    native = _native(model_pair)
    hookers = {} if native else {n: model_pair.make_ll_ablation_hook(n) for n in nodes}
    results = {n: 0 for n in nodes}
    loader = dataset.make_loader(batch_size=batch_size, num_workers=0)
    nb = 0
    sweep = None
    if native and not verbose and nodes:
        dev = next(model_pair.ll_model.parameters()).device
        sweep = _SweepGraph(lambda b, a: _resample_scores(model_pair, b, a, nodes,
                                                          categorical_metric=categorical_metric), len(nodes), dev)
    for base_in, ablation_in in progress(loader, desc="resample ablation"):
        nb += 1
        if sweep is not None:
            sweep(base_in, ablation_in)
            continue
        if native:
            resample_ablate_nodes(model_pair, base_in, ablation_in, nodes, results, verbose=verbose,
                                  categorical_metric=categorical_metric)
            continue
        for node in nodes:
            resample_ablate_node(model_pair, base_in, ablation_in, node, results, hookers.get(node), verbose=verbose,
                                 categorical_metric=categorical_metric)
    if sweep is not None:
        sums = sweep.sums().tolist()  # one host read for the whole sweep
        return {n: float(sums[i]) / max(nb, 1) for i, n in enumerate(nodes)}
    return {n: float(v) / max(nb, 1) for n, v in results.items()}


# ----------------------------------------------------------------------------- mean / zero ablation
def get_mean_cache(model_pair, dataset, batch_size: int = 8, names=None) -> Dict[str, torch.Tensor]:
    """Dataset mean of every (or the named) LL hook activation, shape [1, ...] (``eval_ablations.py:164-173``)."""
    loader = dataset.make_loader(batch_size=batch_size, num_workers=0)
    n = len(loader)
    mean_cache: Dict[str, torch.Tensor] = {}
    model = model_pair.ll_model
    with torch.no_grad():
        for batch in progress(loader, desc="mean cache"):
            x = batch[0]
            if _native(model_pair):
                wanted = names if names is not None else list(model.hook_dict.keys())
                cache = model.run_capture(x, sorted(wanted))
            else:
                _, cache = model.run_with_cache(x)
            for name, t in cache.items():
                m = t.float().mean(dim=0, keepdim=True) / n
                mean_cache[name] = mean_cache[name] + m if name in mean_cache else m
    return mean_cache


def make_ablation_hook(node: LLNode, mean_cache: Optional[Dict[str, torch.Tensor]], use_mean_cache: bool = True
                       ) -> Callable[[torch.Tensor, HookPoint], torch.Tensor]:
    if node.subspace is not None:
        raise NotImplementedError("Subspace not supported yet.")
    index = node.index if node.index is not None else EVERYTHING

    def zero_hook(act: torch.Tensor, hook: HookPoint) -> torch.Tensor:
        act[index.as_index] = 0
        return act

    def mean_hook(act: torch.Tensor, hook: HookPoint) -> torch.Tensor:
        act[index.as_index] = mean_cache[node.name][index.as_index].to(act.dtype)
        return act

    return mean_hook if use_mean_cache else zero_hook


def _ablation_value(node: LLNode, mean_cache, use_mean_cache: bool, like: torch.Tensor) -> torch.Tensor:
    if use_mean_cache:
        return mean_cache[node.name].to(like.dtype).expand_as(like)
    return torch.zeros_like(like)


def _ablation_score(model_pair, ll_out, base_ll_out, base_hl_out, hl_reduced, atol: float = 5e-2):
    reduced = _reduced_logits(model_pair)
    if model_pair.hl_model.is_categorical():
        label_idx = model_pair.get_label_idxs()
        ll_pred = torch.argmax(_at(ll_out.squeeze() if not reduced else ll_out, label_idx, reduced), dim=-1)
        hl_pred = torch.argmax(_at(base_hl_out.squeeze() if not hl_reduced else base_hl_out, label_idx, hl_reduced),
                               dim=-1)
        base_pred = torch.argmax(_at(base_ll_out.squeeze() if not reduced else base_ll_out, label_idx, reduced),
                                 dim=-1)
        accuracy = (base_pred == hl_pred).float()
        changed = (ll_pred != hl_pred).float() * accuracy
    else:
        ll_unchanged = torch.isclose(ll_out.float().squeeze(), base_hl_out.float().squeeze(), atol=atol)
        accuracy = torch.isclose(base_ll_out.float().squeeze(), base_hl_out.float().squeeze(), atol=atol).float()
        changed = (~ll_unchanged).float() * accuracy
    return changed.sum() / (accuracy.sum() + 1e-6)


def ablate_node(model_pair, base_in, node: LLNode, results: Dict, hook: Optional[Callable] = None, atol: float = 5e-2,
                verbose: bool = False, mean_cache=None, use_mean_cache: bool = True, shapes=None) -> None:
    base_x = base_in[0]
    model = model_pair.ll_model
    with torch.no_grad():
        if _native(model_pair):
            like = shapes[node.name] if shapes is not None else model.run_capture(base_x, [node.name])[node.name]
            if like.shape[0] != base_x.shape[0]:
                like = like[:1].expand(base_x.shape[0], *like.shape[1:])
            val = _ablation_value(node, mean_cache, use_mean_cache, like)
            plan = RunPlan.with_splices([(node.name, node.index, val)], logits=model_pair.ll_logits_mode())
            ll_out = model(base_x, plan=plan)
            base_ll_out = model_pair.ll_forward(base_x)
        else:
            ll_out = model.run_with_hooks(base_x, fwd_hooks=[(node.name, hook)])
            base_ll_out = model(base_x)
        base_hl_out, hl_reduced = _hl_out(model_pair, base_in)
    results[node] = results[node] + _ablation_score(model_pair, ll_out, base_ll_out, base_hl_out, hl_reduced, atol)


def _ablation_scores(model_pair, base_in, nodes, values: Dict[str, torch.Tensor], atol: float = 5e-2) -> torch.Tensor:
    """One batch of the native mean / zero ablation sweep: one unablated base forward and one HL base output, then
    one spliced forward per node with its [1, ...] ablation value broadcast over the batch; scores as a vector."""
    model = model_pair.ll_model
    base_x = base_in[0]
    with torch.no_grad():
        base_ll_out = model_pair.ll_forward(base_x)
        base_hl_out, hl_reduced = _hl_out(model_pair, base_in)
        B = base_x.shape[0]
        prefix = _BasePrefix(model_pair, base_x, nodes)
        scores = [None] * len(nodes)
        groups, single = _node_groups(model_pair, base_x, prefix, nodes)
        for L, pos in groups:
            srcs = {p: values[nodes[p].name] for p in pos}  # [1, ...] values broadcast per row group
            ll_all = prefix.forward_rows(base_x, L, len(pos), _group_plan(model_pair, nodes, pos, srcs, B))
            for i, p in enumerate(pos):
                scores[p] = _ablation_score(model_pair, ll_all[i * B:(i + 1) * B], base_ll_out, base_hl_out,
                                            hl_reduced, atol).float().reshape(())
        for p in single:
            node = nodes[p]
            v = values[node.name]
            v = v.expand(B, *v.shape[1:]) if v.shape[0] != B else v  # a view: no per-batch copy
            plan = RunPlan.with_splices([(node.name, node.index, v)], logits=model_pair.ll_logits_mode())
            ll_out = prefix.forward(base_x, node, plan)
            scores[p] = _ablation_score(model_pair, ll_out, base_ll_out, base_hl_out, hl_reduced,
                                        atol).float().reshape(())
        return torch.stack(scores)


def ablate_nodes(model_pair, base_in, nodes, results: Dict, values: Dict[str, torch.Tensor], atol: float = 5e-2) -> None:
    """Native batched form of :func:`ablate_node` over ``nodes`` (adds into ``results``)."""
    s = _ablation_scores(model_pair, base_in, nodes, values, atol)
    for i, node in enumerate(nodes):
        results[node] = results[node] + s[i]


def check_causal_effect_on_ablation(model_pair, dataset, batch_size: int = 256, node_type: str = "a",
                                    mean_cache: Optional[Dict[str, torch.Tensor]] = None, verbose: bool = False
                                    ) -> Dict[LLNode, float]:
    """Mean (or zero) ablation effect per node (``eval_ablations.py:262-295``)."""
    use_mean_cache = bool(mean_cache)
    nodes = _nodes(model_pair, node_type, with_suffixes=True)
    native = _native(model_pair)
    hookers = {} if native else {n: make_ablation_hook(n, mean_cache, use_mean_cache) for n in nodes}
    results = {n: 0 for n in nodes}
    loader = dataset.make_loader(batch_size=batch_size, num_workers=0)
    nb = 0
    values = None
    sweep = None
    for base_in in progress(loader, desc="ablation"):
        nb += 1
        if native:
            if values is None:  # [1, ...] ablation values, broadcast over every batch (shapes probed once)
                names = sorted({n.name for n in nodes})
                if use_mean_cache and all(nm in mean_cache for nm in names):
                    values = {nm: mean_cache[nm] for nm in names}
                else:
                    with torch.no_grad():
                        probe = model_pair.ll_model.run_capture(base_in[0][:1], names)
                    values = {nm: (mean_cache[nm] if use_mean_cache else torch.zeros_like(probe[nm]))
                              for nm in names}
                if nodes and not verbose:
                    dev = next(model_pair.ll_model.parameters()).device
                    sweep = _SweepGraph(lambda b: _ablation_scores(model_pair, b, nodes, values), len(nodes), dev)
            if sweep is not None:
                sweep(base_in)
            else:
                ablate_nodes(model_pair, base_in, nodes, results, values)
            continue
        for node in nodes:
            ablate_node(model_pair, base_in, node, results, hookers.get(node), verbose=verbose, mean_cache=mean_cache,
                        use_mean_cache=use_mean_cache)
    if sweep is not None:
        sums = sweep.sums().tolist()
        return {n: float(sums[i]) / max(nb, 1) for i, n in enumerate(nodes)}
    return {n: float(v) / max(nb, 1) for n, v in results.items()}


def get_causal_effects_for_all_nodes(model_pair, uni_test_set, batch_size: int = 256, use_mean_cache: bool = True):
    mean_cache = get_mean_cache(model_pair, uni_test_set, batch_size=batch_size) if use_mean_cache else None
    za_not = check_causal_effect_on_ablation(model_pair, uni_test_set, batch_size=batch_size, node_type="n",
                                             mean_cache=mean_cache)
    za_in = check_causal_effect_on_ablation(model_pair, uni_test_set, batch_size=batch_size, node_type="c",
                                            mean_cache=mean_cache)
    return za_not, za_in


# ----------------------------------------------------------------------------- reporting
def _node_label(node: LLNode) -> str:
    if "mlp" in node.name:
        return node.name
    if node.index is not None and node.index != EVERYTHING:
        return f"{node.name}, head {str(node.index).split(',')[-2]}"
    return f"{node.name}, head [:]"


def make_dataframe_of_results(result_not_in_circuit, result_in_circuit):
    import pandas as pd
    df = pd.DataFrame({
        "node": [_node_label(n) for n in result_not_in_circuit] + [_node_label(n) for n in result_in_circuit],
        "status": ["not_in_circuit"] * len(result_not_in_circuit) + ["in_circuit"] * len(result_in_circuit),
        "causal effect": list(result_not_in_circuit.values()) + list(result_in_circuit.values()),
    })
    return df.sort_values("status", ascending=False)


def make_combined_dataframe_of_results(result_not_in_circuit, result_in_circuit, za_result_not_in_circuit,
                                       za_result_in_circuit, use_mean_cache: bool = False):
    df = make_dataframe_of_results(result_not_in_circuit, result_in_circuit)
    df2 = make_dataframe_of_results(za_result_not_in_circuit, za_result_in_circuit)
    df["resample_ablate_effect"] = df.pop("causal effect")
    df["mean_ablate_effect" if use_mean_cache else "zero_ablate_effect"] = df2.pop("causal effect")
    return df


def save_result(df, save_dir: str, model_pair=None) -> None:
    """``results.csv`` (+ ``results.png`` table render, + ``meta.log`` training args) under ``save_dir``."""
    os.makedirs(save_dir, exist_ok=True)
    try:
        _render_table_png(df, os.path.join(save_dir, "results.png"))
    except Exception as e:  # rendering is best-effort, as in the reference
        print(f"Error exporting dataframe to image: {e}")
    df.to_csv(os.path.join(save_dir, "results.csv"))
    if model_pair is None:
        return
    with open(os.path.join(save_dir, "meta.log"), "w") as f:
        f.write(str(model_pair.training_args))


def _render_table_png(df, path: str) -> None:
    import matplotlib
    matplotlib.use("Agg")
    import matplotlib.pyplot as plt
    fig, ax = plt.subplots(figsize=(min(20, 2 + 2.2 * len(df.columns)), 0.4 + 0.3 * len(df)))
    ax.axis("off")
    cells = [[f"{v:.4f}" if isinstance(v, float) else str(v) for v in row] for row in df.itertuples(index=False)]
    ax.table(cellText=cells, colLabels=list(df.columns), loc="center")
    fig.savefig(path, bbox_inches="tight", dpi=120)
    plt.close(fig)
