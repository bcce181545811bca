"""Hashable tensor indices (``TorchIndex`` / ``Ix``).

Parity target: ``/root/reference/iit/utils/index.py:9-122`` (originally from ACDC).
A ``TorchIndex`` describes *which part* of a hook tensor a node covers.  Each
entry of the tuple is one of ``None`` (whole dimension), ``int``, ``slice`` or
``list[int]``.  ``Ix[[None]]`` is the canonical "everything" index.

Behavioural decisions:
  * ``graphviz_index`` works (the reference passes a kwarg ``__repr__`` does not take).
  * ``intersects`` handles half-open slices with mixed ``None`` bounds instead of
    raising ``TypeError`` on ``max(None, int)``.
  * comparing with a non-``TorchIndex`` returns ``False`` instead of raising.

Besides the reference API this module exposes ``to_ranges``, which lowers an
index to the compact per-dimension range table (up to 8 half-open ranges per
dimension) that the HIP splice / gradient-mask / scale kernel consumes
(``csrc/splice.hip`` through :mod:`iit_amd.ops.splice`, used by
:class:`iit_amd.engine.plan.Splice` and the StopGrad sites of the hooked
transformer), and ``to_mask_spec`` (the same selection as per-dimension lists).
"""
from __future__ import annotations

from typing import Iterable, Optional, Tuple, Union

import torch

IndexAtom = Union[None, int, slice, list]


def _is_int(x) -> bool:
    return isinstance(x, int) and not isinstance(x, bool)


def _freeze(atom: IndexAtom):
    """Hashable representation of one index atom (slices are unhashable < py3.12)."""
    if isinstance(atom, slice):
        return ("slice", atom.start, atom.stop, atom.step)
    if isinstance(atom, list):
        return ("list", tuple(atom))
    return atom


class TorchIndex:
    """A hashable, intersectable tensor index."""

    __slots__ = ("as_index", "hashable_tuple", "_atoms", "_dev", "_iit_specs")

    def __init__(self, list_of_things_in_tuple: Iterable[IndexAtom]):
        if not isinstance(list_of_things_in_tuple, (tuple, list)):
            list_of_things_in_tuple = (list_of_things_in_tuple,)
        atoms = tuple(list_of_things_in_tuple)
        for a in atoms:
            if a is None or _is_int(a) or isinstance(a, slice):
                continue
            if not (isinstance(a, list) and all(_is_int(v) for v in a)):
                raise TypeError(f"unsupported index atom {a!r} (allowed: None, int, slice, list[int])")
        self._atoms = atoms
        self.as_index: Tuple = tuple(slice(None) if a is None else a for a in atoms)
        self.hashable_tuple = tuple(_freeze(a) for a in atoms)
        self._dev = None
        self._iit_specs = None  # packed splice range tables per (hook shape, source strides), see iit_amd.ops.splice

    def on(self, device) -> Tuple:
        """``as_index`` with list atoms as cached int64 tensors on ``device``: indexing a GPU tensor with a Python
        list copies the list host-to-device on every call, which a captured HIP graph cannot contain (and which
        costs a sync-free but real copy per splice).  The first call per device builds the tensors."""
        if not any(isinstance(a, list) for a in self._atoms):
            return self.as_index
        device = torch.device(device)
        if self._dev is None:
            self._dev = {}
        ix = self._dev.get(device)
        if ix is None:
            ix = self._dev[device] = tuple(torch.tensor(a, dtype=torch.long, device=device) if isinstance(a, list)
                                           else a for a in self.as_index)
        return ix

    # -- identity -----------------------------------------------------------
    def __hash__(self) -> int:
        return hash(self.hashable_tuple)

    def __eq__(self, other) -> bool:
        if not isinstance(other, TorchIndex):
            return False
        return self.hashable_tuple == other.hashable_tuple

    def __ne__(self, other) -> bool:
        return not self.__eq__(other)

    def __len__(self) -> int:
        return len(self._atoms)

    # -- printing -----------------------------------------------------------
    def _fmt(self, colon: str = ":") -> str:
        parts = []
        for a in self._atoms:
            if a is None:
                parts.append(colon)
            elif _is_int(a):
                parts.append(str(a))
            elif isinstance(a, slice):
                if a.step is not None:
                    raise ValueError("Step is not supported")
                lo = "" if a.start is None else str(a.start)
                hi = "" if a.stop is None else str(a.stop)
                parts.append(f"{lo}{colon}{hi}")
            else:
                parts.append(str(list(a)))
        return "[" + ", ".join(parts) + "]"

    def __repr__(self) -> str:
        return self._fmt(":")

    def graphviz_index(self, use_actual_colon: bool = True) -> str:
        return self._fmt(":" if use_actual_colon else "COLON")

    # -- algebra ------------------------------------------------------------
    def is_everything(self) -> bool:
        """True for indices that select the whole tensor (``Ix[[None]]``, ``Ix[:, :]``...)."""
        return all(a is None or (isinstance(a, slice) and a == slice(None)) for a in self._atoms)

    def intersects(self, other: Optional["TorchIndex"]) -> bool:
        if other is None or self == EVERYTHING or other == EVERYTHING:
            return True
        if len(self.as_index) != len(other.as_index):
            raise ValueError("Cannot compare indices of different lengths")
        for a, b in zip(self.as_index, other.as_index):
            if not _atoms_overlap(a, b):
                return False
        return True

    def to_ranges(self, shape: Tuple[int, ...], max_ranges: int = 8):
        """Per-dimension lists of half-open ``(lo, hi)`` ranges selecting the same elements of a tensor of ``shape``
        as ``t[self.as_index]`` -- the splice kernel's patch spec -- or None when the index is not such a
        per-dimension product: more than one list atom (torch pairs list atoms up instead of crossing them), a
        stepped slice, more atoms than dimensions, or a dimension needing more than ``max_ranges`` runs.
        Negative ints / slice bounds are normalised; list atoms are sorted and merged into runs (a splice writes
        the same value whatever the order or multiplicity)."""
        atoms = self.as_index
        if len(atoms) > len(shape) or sum(isinstance(a, list) for a in atoms) > 1:
            return None
        out = []
        for d, n in enumerate(shape):
            a = atoms[d] if d < len(atoms) else slice(None)
            if isinstance(a, slice):
                if a.step not in (None, 1):
                    return None
                lo, hi, _ = a.indices(n)
                runs = [(lo, hi)] if hi > lo else []
            elif _is_int(a):
                if not -n <= a < n:
                    return None
                v = a % n
                runs = [(v, v + 1)]
            else:
                if any(not -n <= v < n for v in a):
                    return None  # out of range: the generic path raises torch's IndexError
                vals = sorted({v % n for v in a})
                runs = []
                for v in vals:
                    if runs and runs[-1][1] == v:
                        runs[-1] = (runs[-1][0], v + 1)
                    else:
                        runs.append((v, v + 1))
            if len(runs) > max_ranges:
                return None
            out.append(runs)
        return out

    def to_mask_spec(self, shape: Tuple[int, ...]):
        """Per-dimension list of selected positions (None = whole dim) for ``shape``.

        Used by the engine to build splice masks.  Trailing dims not named by
        the index are whole.
        """
        spec = []
        for d, n in enumerate(shape):
            a = self.as_index[d] if d < len(self.as_index) else slice(None)
            if isinstance(a, slice):
                if a == slice(None):
                    spec.append(None)
                else:
                    spec.append(list(range(n))[a])
            elif _is_int(a):
                spec.append([a % n])
            else:
                spec.append([v % n for v in a])
        return spec


def _slice_bounds(s: slice):
    lo = 0 if s.start is None else s.start
    hi = float("inf") if s.stop is None else s.stop
    return lo, hi


def _atoms_overlap(a, b) -> bool:
    if a == slice(None) or b == slice(None):
        return True
    if _is_int(a) and _is_int(b):
        return a == b
    if isinstance(a, list) or isinstance(b, list):
        la = a if isinstance(a, list) else None
        lb = b if isinstance(b, list) else None
        if la is not None and lb is not None:
            return bool(set(la) & set(lb))
        lst, other = (la, b) if la is not None else (lb, a)
        return any(_atoms_overlap(v, other) for v in lst)
    if isinstance(a, slice) and isinstance(b, slice):
        alo, ahi = _slice_bounds(a)
        blo, bhi = _slice_bounds(b)
        return max(alo, blo) < min(ahi, bhi)
    s, i = (a, b) if isinstance(a, slice) else (b, a)
    lo, hi = _slice_bounds(s)
    return lo <= i < hi


class Index:
    """Syntactic sugar: ``Ix[:, :, 3]`` -> ``TorchIndex((slice(None), slice(None), 3))``."""

    def __getitem__(self, index) -> TorchIndex:
        return TorchIndex(index)


Ix = Index()
EVERYTHING = TorchIndex([None])
