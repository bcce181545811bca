"""The HL -> LL correspondence map (the paper's Pi).

Parity target: ``/root/reference/iit/utils/correspondence.py:3-70``.

Decisions:
  * item assignment is validated (key must be an ``HLNode`` or ``str``; values an
    ``LLNode`` or a set of them).  A bare ``LLNode`` value is accepted and stored
    as-is for parity with ``tests/test_corr.py`` in the reference.
  * ``make_corr_from_dict`` defaults ``suffixes`` instead of asserting on ``None``.
"""
from __future__ import annotations

from typing import Dict, Iterable, Optional

from .nodes import HLNode, LLNode

DEFAULT_SUFFIXES = {"attn": "attn.hook_result", "mlp": "mlp.hook_post"}


class Correspondence(dict):
    def __init__(self, *args, suffixes: Optional[Dict[str, str]] = None, **kwargs):
        super().__init__()
        self.suffixes = dict(DEFAULT_SUFFIXES if suffixes is None else suffixes)
        for k, v in dict(*args, **kwargs).items():
            self[k] = v

    def __setattr__(self, key, value):
        if key == "suffixes" and not isinstance(value, dict):
            raise TypeError(f"suffixes must be a dict, got {type(value)}")
        super().__setattr__(key, value)

    def __setitem__(self, key, value):
        if isinstance(key, str) and not isinstance(key, HLNode):
            key = HLNode(key, -1)
        if not isinstance(key, HLNode):
            raise TypeError(f"key must be of type HLNode, got {type(key)}")
        if isinstance(value, (list, tuple, frozenset)):
            value = set(value)
        if isinstance(value, set):
            bad = [v for v in value if not isinstance(v, LLNode)]
            if bad:
                raise TypeError(f"value contains non-LLNode elements: {bad}")
        elif not isinstance(value, LLNode):
            raise TypeError(f"value must be a set of LLNode, got {type(value)}")
        super().__setitem__(key, value)

    def get_suffixes(self) -> Dict[str, str]:
        return self.suffixes

    def ll_nodes(self, hl_node) -> Iterable[LLNode]:
        v = self[hl_node]
        return [v] if isinstance(v, LLNode) else sorted(v, key=lambda n: (n.name, repr(n.index)))

    @staticmethod
    def get_hook_suffix(corr: Dict[HLNode, Iterable[LLNode]]) -> Dict[str, str]:
        """Infer the per-block hook suffix (text after ``blocks.<l>.``) of attn / mlp nodes."""
        found: Dict[str, str] = {}
        for _, ll_nodes in corr.items():
            if isinstance(ll_nodes, LLNode):
                ll_nodes = [ll_nodes]
            for node in ll_nodes:
                suffix = ".".join(node.name.split(".")[2:])
                if "attn" in node.name:
                    kind = "attn"
                elif "mlp" in node.name:
                    kind = "mlp"
                else:
                    raise ValueError(f"Unknown node type {node.name}")
                if kind in found and found[kind] != suffix:
                    raise ValueError(
                        f"Multiple {kind} suffixes found: {found[kind]} and {suffix}; "
                        f"multiple {kind} hook locations are not supported"
                    )
                found[kind] = suffix
        return found

    @classmethod
    def make_corr_from_dict(cls, d, suffixes=None, make_suffixes_from_corr: bool = False):
        mapping = {
            HLNode(k, -1): {LLNode(name=n, index=None) for n in names} for k, names in d.items()
        }
        if make_suffixes_from_corr:
            suffixes = cls.get_hook_suffix(mapping)
        return cls(mapping, suffixes=suffixes)

    def to_name_dict(self) -> Dict[str, list]:
        """Inverse of ``make_corr_from_dict`` for whole-tensor nodes (``corr.json`` layout)."""
        out = {}
        for k, v in self.items():
            nodes = [v] if isinstance(v, LLNode) else list(v)
            out[k.name] = sorted(n.name for n in nodes)
        return out
