"""High-level / low-level node descriptors.

Parity target: ``/root/reference/iit/model_pairs/nodes.py:10-56``.

* ``HLNode`` hashes by name and compares equal to a plain ``str`` of that name,
  so ``corr["hook_x"]`` works on a correspondence keyed by ``HLNode``.
* ``LLNode`` hashes / compares on ``(name, index, subspace)``.
* A ``None`` index is normalised to ``Ix[[None]]`` (whole tensor).
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Any, Optional

import torch

from .index import EVERYTHING, Ix, TorchIndex

HookName = str
HLCache = dict  # dict[HookName, torch.Tensor]


@dataclass(eq=False)
class HLNode:
    name: HookName
    num_classes: int
    index: Optional[TorchIndex] = field(default_factory=lambda: Ix[[None]])

    def __post_init__(self):
        if self.index is None:
            self.index = Ix[[None]]

    def __hash__(self) -> int:
        return hash(self.name)

    def __eq__(self, other) -> bool:
        if isinstance(other, HLNode):
            return self.name == other.name
        if isinstance(other, str):
            return self.name == other
        return False

    def __str__(self) -> str:
        return self.name

    def __repr__(self) -> str:
        return self.name


@dataclass(eq=False)
class LLNode:
    name: HookName
    index: Optional[TorchIndex]
    subspace: Optional[Any] = None

    def __post_init__(self):
        if self.index is None:
            self.index = Ix[[None]]

    def _key(self):
        sub = self.subspace
        if isinstance(sub, torch.Tensor):
            sub = ("tensor", sub.data_ptr(), tuple(sub.shape))
        return (self.name, self.index, sub)

    def __eq__(self, other) -> bool:
        return isinstance(other, LLNode) and self._key() == other._key()

    def __hash__(self) -> int:
        return hash(self._key())

    def __repr__(self) -> str:
        return f"LLNode(name={self.name!r}, index={self.index!r}, subspace={self.subspace!r})"

    def get_index(self):
        return self.index.as_index

    @property
    def is_whole(self) -> bool:
        return self.index == EVERYTHING or self.index.is_everything()


# names used throughout the package
__all__ = ["HLNode", "LLNode", "HookName", "HLCache"]
