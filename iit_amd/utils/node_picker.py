"""Circuit algebra over LL nodes and parameters.

Parity: ``/root/reference/iit/utils/node_picker.py:9-170``.  Candidate LL nodes
are, per layer, one node per head ``Ix[:, :, h, :]`` on the attention hook plus
one whole-tensor MLP node; the rest is set algebra against the correspondence
and the mapping from activation nodes to TL parameter slices (reproducing the
reference's d_head-axis indexing quirk Q8 for API parity).  Q20 fixed:
``get_post_nodes_not_in_circuit`` never leaves the hook name unbound.
"""
from __future__ import annotations

from typing import Dict, Iterable, List

import torch

from ..core.correspondence import DEFAULT_SUFFIXES, Correspondence
from ..core.index import EVERYTHING, Ix, TorchIndex
from ..core.nodes import LLNode

LLParamNode = LLNode


def _cfg(model):
    cfg = getattr(model, "cfg", None)
    if cfg is None and hasattr(model, "model"):
        cfg = model.model.cfg
    return cfg


def get_all_nodes(model, suffixes: Dict[str, str] = None) -> List[LLNode]:
    suffixes = DEFAULT_SUFFIXES if suffixes is None else suffixes
    cfg = _cfg(model)
    nodes = []
    for layer in range(cfg.n_layers):
        attn_hook = f"blocks.{layer}.{suffixes['attn']}"
        nodes.extend(LLNode(attn_hook, Ix[:, :, h, :]) for h in range(cfg.n_heads))
        if not getattr(cfg, "attn_only", False):
            nodes.append(LLNode(f"blocks.{layer}.{suffixes['mlp']}", Ix[[None]]))
    return nodes


def _corr_values(corr) -> Iterable[LLNode]:
    for v in corr.values():
        if isinstance(v, LLNode):
            yield v
        else:
            yield from v


def get_nodes_in_circuit(hl_ll_corr) -> List[LLNode]:
    # sorted (the reference returns set order, which varies with PYTHONHASHSEED and
    # would desynchronise ranks / result tables)
    return sorted(set(_corr_values(hl_ll_corr)), key=lambda n: (n.name, repr(n.index)))


def nodes_intersect(a: LLNode, b: LLNode) -> bool:
    return a.name == b.name and a.index.intersects(b.index)


def get_nodes_not_in_circuit(ll_model, hl_ll_corr) -> List[LLNode]:
    suffixes = hl_ll_corr.get_suffixes() if hasattr(hl_ll_corr, "get_suffixes") else DEFAULT_SUFFIXES
    in_circuit = get_nodes_in_circuit(hl_ll_corr)
    return [n for n in get_all_nodes(ll_model, suffixes) if not any(nodes_intersect(n, c) for c in in_circuit)]


def get_post_nodes_not_in_circuit(ll_model, hl_ll_corr) -> List[LLNode]:
    """Whole-hook nodes of every layer component that has a non-circuit node."""
    suffixes = hl_ll_corr.get_suffixes() if hasattr(hl_ll_corr, "get_suffixes") else DEFAULT_SUFFIXES
    out: List[LLNode] = []
    seen = set()
    for node in get_nodes_not_in_circuit(ll_model, hl_ll_corr):
        layer = int(node.name.split(".")[1])
        kind = "attn" if ("attn" in node.name and "attn" in suffixes) else "mlp"
        name = f"blocks.{layer}.{suffixes[kind]}"
        if name not in seen:
            seen.add(name)
            out.append(LLNode(name, Ix[[None]]))
    return out


def _get_param_idx(name: str, param: torch.Tensor, node: LLNode) -> TorchIndex:
    kind = name.split(".")[-1]
    idx = node.index
    if node.subspace is not None:
        raise NotImplementedError("Subspaces are not supported")
    if idx == EVERYTHING or kind == "b_O":
        pidx = EVERYTHING
    elif kind in ("W_Q", "W_K", "W_V"):
        pidx = TorchIndex(list(idx.as_index[:-1]))
    elif kind == "W_O":
        t = list(idx.as_index[:-1])
        pidx = TorchIndex([t[0], t[2], t[1]])
    elif kind in ("b_Q", "b_K", "b_V"):
        t = list(idx.as_index[:-1])
        pidx = TorchIndex([slice(None), t[2]])
    else:
        raise NotImplementedError(f"Param of type '{kind}' is expected to have index {EVERYTHING}, but got {idx}")
    try:
        param[pidx.as_index]
    except IndexError as e:
        raise IndexError(f"Index {pidx} is out of bounds for param {name}") from e
    return pidx


def get_activation_idx(node: LLParamNode) -> TorchIndex:
    kind = node.name.split(".")[-1]
    t = node.index.as_index
    if kind in ("W_Q", "W_K", "W_V"):
        return TorchIndex([slice(None), *t])
    if kind in ("b_Q", "b_K", "b_V"):
        return TorchIndex([slice(None), *t, slice(None)])
    if kind == "W_O":
        return TorchIndex([t[0], t[2], t[1], slice(None)])
    return EVERYTHING


def _named_parameters(model):
    inner = getattr(model, "model", None)
    if inner is not None and not isinstance(model, torch.nn.Module):
        return inner.named_parameters()
    return model.named_parameters()


def get_params_in_circuit(hl_ll_corr, ll_model) -> List[LLParamNode]:
    in_circuit = get_nodes_in_circuit(hl_ll_corr)
    out = []
    for name, param in _named_parameters(ll_model):
        prefix = name.rsplit(".", 1)[0]
        for node in in_circuit:
            if node.name.rsplit(".", 1)[0] == prefix:
                out.append(LLParamNode(name, _get_param_idx(name, param, node)))
    return out


def get_all_params(ll_model) -> List[LLParamNode]:
    cfg = _cfg(ll_model)
    out = []
    for name, param in _named_parameters(ll_model):
        kind = name.split(".")[-1]
        if kind in ("W_Q", "W_K", "W_V", "W_O", "b_Q", "b_K", "b_V"):
            for h in range(cfg.n_heads):
                out.append(LLParamNode(name, _get_param_idx(name, param, LLParamNode(name, Ix[:, :, h, :]))))
        else:
            out.append(LLParamNode(name, EVERYTHING))
    return out


def get_params_not_in_circuit(hl_ll_corr, ll_model, filter_out_embed: bool = True) -> List[LLParamNode]:
    in_circuit = get_nodes_in_circuit(hl_ll_corr)
    out = []
    for p in get_all_params(ll_model):
        if filter_out_embed and "embed" in p.name:
            continue
        if not any(nodes_intersect(p, c) for c in in_circuit):
            out.append(p)
    return out
