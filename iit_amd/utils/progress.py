"""Progress bars (tqdm when available, silent otherwise)."""
from __future__ import annotations


def progress(iterable, total=None, disable: bool = False, leave: bool = True, desc=None):
    if disable:
        return iterable
    try:
        from tqdm import tqdm
    except ImportError:  # pragma: no cover
        return iterable
    return tqdm(iterable, total=total, leave=leave, desc=desc)
