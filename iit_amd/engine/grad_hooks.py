"""Notification channel for gradients written directly by fused kernels.

The HIP op backend accumulates weight gradients straight into ``param.grad``
(inside the GEMM epilogue) instead of returning them to autograd, so torch's
post-accumulate-grad hooks never fire for those parameters.  Kernels call
``notify(param)`` after the write; the data-parallel reducer listens here to
launch bucket all-reduces as soon as a bucket's gradients are final.
"""
from __future__ import annotations

from typing import Callable, List

_listeners: List[Callable] = []


def add_listener(fn: Callable) -> Callable:
    _listeners.append(fn)
    return fn


def remove_listener(fn: Callable) -> None:
    if fn in _listeners:
        _listeners.remove(fn)


def notify(p) -> None:
    for fn in _listeners:
        fn(p)
