"""Metric kernels for the causal-effect sweeps (parity: ``/root/reference/iit/utils/eval_metrics.py:4-32``).

``kl_div(a, b, label_idx)`` is KL(b || a) per row at the label index, where either
input is softmaxed unless its rows already sum to one.  ``accuracy_affected``
is the fraction of changed-label samples whose argmax prediction flipped.
Both are sync-free (return device tensors).
"""
from __future__ import annotations

import torch

from ..core.index import TorchIndex


def _as_pmf(x: torch.Tensor) -> torch.Tensor:
    x = x.float()
    s = x.sum(dim=-1)
    # rows that are already probability vectors are used as-is (reference: allclose(sum, 1))
    is_pmf = torch.isclose(s, torch.ones_like(s), rtol=1e-5, atol=1e-8).all()
    return torch.where(is_pmf, x, torch.softmax(x, dim=-1))


def kl_div(a: torch.Tensor, b: torch.Tensor, label_idx: TorchIndex) -> torch.Tensor:
    """KL(b || a) over the last dim at ``label_idx`` (``a`` = intervened LL output, ``b`` = HL target)."""
    a_pmf = _as_pmf(a[label_idx.as_index])
    b_pmf = _as_pmf(b[label_idx.as_index])
    return torch.nn.functional.kl_div(a_pmf.log(), b_pmf, reduction="none", log_target=False).sum(dim=-1)


def accuracy_affected(a: torch.Tensor, b: torch.Tensor, label_unchanged: torch.Tensor,
                      label_idx: TorchIndex) -> torch.Tensor:
    a_lab = torch.argmax(a[label_idx.as_index], dim=-1)
    b_lab = torch.argmax(b[label_idx.as_index], dim=-1)
    changed = (a_lab != b_lab).float() * (~label_unchanged).float()
    return changed.sum() / (~label_unchanged).float().sum()
