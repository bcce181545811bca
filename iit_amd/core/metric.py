"""Per-epoch metric accumulation.

Parity target: ``/root/reference/iit/utils/metric.py:5-88``.  Each train/eval
step returns ``{name: value}``; ``MetricStoreCollection.update`` appends them;
an epoch value is the mean (x100 for ``ACCURACY``) or, for
``PerTokenMetricStore``, the per-position mean.

Differences (documented): no global numpy print-option side
effects; formatting precision is per-store.  Values may be python floats,
numpy arrays or *device tensors*: tensors are kept on device and only reduced
(one host sync) when ``get_value`` is called, so a training epoch does not pay
one ``.item()`` per step.
"""
from __future__ import annotations

from enum import Enum
from typing import Dict, List

import numpy as np


class MetricType(Enum):
    ACCURACY = 1
    LOSS = 2
    LOG = 3


def _to_numpy_list(store):
    """Materialise a list that may contain device tensors with a single host transfer."""
    try:
        import torch
    except ImportError:  # pragma: no cover
        return [np.asarray(v) for v in store]
    tensors = [i for i, v in enumerate(store) if isinstance(v, torch.Tensor)]
    if not tensors:
        return store
    out = list(store)
    stacked = torch.stack([store[i].detach().float().reshape(-1) for i in tensors]).cpu().numpy()
    for row, i in enumerate(tensors):
        v = stacked[row]
        out[i] = v[0] if v.size == 1 and store[i].dim() == 0 else v
    return out


class MetricStore:
    def __init__(self, name: str, metric_type: MetricType):
        if not isinstance(metric_type, MetricType):
            raise AssertionError(f"Invalid metric type {metric_type}")
        self._name = name
        self.type = metric_type
        self._store: list = []

    def append(self, metric):
        self._store.append(metric)

    def _values(self):
        if len(self._store) == 0:
            raise ValueError("No values in metric store!")
        self._store = _to_numpy_list(self._store)
        return self._store

    def get_value(self):
        vals = self._values()
        m = float(np.mean(vals))
        return m * 100 if self.type == MetricType.ACCURACY else m

    def get_name(self) -> str:
        return self._name

    def __str__(self) -> str:
        if self.type == MetricType.ACCURACY:
            return f"{self._name}: {float(self.get_value()):.2f}%"
        return f"{self._name}: {self.get_value():.4f}"

    __repr__ = __str__

    def __len__(self) -> int:
        return len(self._store)


class PerTokenMetricStore(MetricStore):
    def __init__(self, name: str, precision: int = 3, **kwargs):
        super().__init__(name, metric_type=MetricType.LOG)
        self.precision = precision

    def get_value(self):
        return np.mean(np.stack([np.asarray(v, dtype=np.float64) for v in self._values()]), axis=0)

    def __str__(self) -> str:
        return f"{self._name}: {np.array2string(self.get_value(), precision=self.precision)}"

    __repr__ = __str__


class MetricStoreCollection:
    def __init__(self, list_of_metric_stores: List[MetricStore]):
        self.metrics = list_of_metric_stores

    def _by_name(self, name):
        for m in self.metrics:
            if m.get_name() == name:
                return m
        return None

    def update(self, metrics: Dict[str, object]):
        for k, v in metrics.items():
            store = self._by_name(k)
            if store is None:
                raise AssertionError(f"Key {k} not found in metric stores!")
            store.append(v)
        lengths = {len(m) for m in self.metrics}
        if len(lengths) > 1:
            raise AssertionError(
                f"All metric stores should have the same length after update!, got lengths: "
                f"{[len(m) for m in self.metrics]}"
            )

    def create_metric_store(self, name: str, metric_type: MetricType) -> MetricStore:
        if any(len(m) for m in self.metrics):
            raise AssertionError("All metric stores should be empty before creating a new one!")
        store = MetricStore(name, metric_type)
        self.metrics.append(store)
        return store

    def __str__(self) -> str:
        return "\n".join(str(m) for m in self.metrics)

    def to_dict(self) -> Dict[str, object]:
        return {m.get_name(): m.get_value() for m in self.metrics}
