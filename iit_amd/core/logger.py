"""Change-tracking dict (parity: ``/root/reference/iit/utils/logger.py:7-52``).

Writes the first value and every change of each key to
``logs/log_<%m-%d_%H-%M>.log``.  Unlike the reference, importing this module
has no numpy print-option side effect, and the log directory is configurable.
"""
from __future__ import annotations

import os
import time

import numpy as np


def _same(x, y) -> bool:
    try:
        import torch
        if isinstance(x, torch.Tensor) or isinstance(y, torch.Tensor):
            return (isinstance(x, torch.Tensor) and isinstance(y, torch.Tensor) and x.shape == y.shape
                    and bool((x == y).all()))
    except ImportError:  # pragma: no cover
        pass
    if isinstance(x, np.ndarray):
        return isinstance(y, np.ndarray) and x.shape == y.shape and bool((x == y).all())
    if isinstance(x, (list, tuple)):
        return isinstance(y, (list, tuple)) and len(x) == len(y) and all(_same(a, b) for a, b in zip(x, y))
    return x == y


class LoggingDict(dict):
    def __init__(self, *args, log_dir: str = "logs", **kwargs):
        os.makedirs(log_dir, exist_ok=True)
        self._log_filename = os.path.join(log_dir, f"log_{time.strftime('%m-%d_%H-%M')}.log")
        super().__init__(*args, **kwargs)

    compare = staticmethod(_same)

    @staticmethod
    def convert_tensor_to_numpy(x):
        try:
            import torch
            if isinstance(x, torch.Tensor):
                return x.detach().cpu().numpy()
        except ImportError:  # pragma: no cover
            pass
        return x

    def __setitem__(self, key, value):
        if key not in self:
            msg = f"{key}\n initial value: {value}\n"
        elif not _same(self[key], value):
            msg = f"{key}\n changed from {self[key]} to {value}\n"
        else:
            msg = None
        if msg:
            with open(self._log_filename, "a") as f:
                f.write(msg)
        super().__setitem__(key, value)
