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


def target_stats(b: torch.Tensor):
    """What :func:`kl_div_from_stats` needs of a 2-D HL output ``b`` (computed once per batch, shared by every node
    of a sweep): its pmf (``_as_pmf``), the per-row sum of ``b log b`` (0 log 0 = 0) and the per-row pmf sum."""
    bp = _as_pmf(b).contiguous()
    return bp, torch.special.xlogy(bp, bp).sum(-1), bp.sum(-1)


def kl_div_from_stats(a: torch.Tensor, stats) -> torch.Tensor:
    """``kl_div(a, b, EVERYTHING)`` per row for a 2-D LL output ``a`` and ``stats = target_stats(b)``.

    On the GPU one kernel pass over ``a`` and the pmf (``hip_kernels.kl_rows``) gives sum(a), logsumexp(a),
    sum(b a) and sum(b log a); then KL = sum b log b - (sum b a - lse(a) sum b) when ``a`` is read as logits
    (log softmax = a - lse) and sum b log b - sum b log a when every row of ``a`` already sums to one, the
    reference's two readings (``_as_pmf``) without materialising softmax / log / kl_div tensors."""
    bp, ent, bsum = stats
    if (a.is_cuda and a.dim() == 2 and a.dtype == torch.float32 and a.stride(1) == 1 and bp.shape == a.shape):
        from ..ops import hip_kernels
        o = hip_kernels.kl_rows(a, bp)
        is_pmf = torch.isclose(o[:, 0], torch.ones_like(o[:, 0]), rtol=1e-5, atol=1e-8).all()
        return torch.where(is_pmf, ent - o[:, 3], ent - (o[:, 2] - o[:, 1] * bsum))
    a_pmf = _as_pmf(a)
    return torch.nn.functional.kl_div(a_pmf.log(), bp, reduction="none", log_target=False).sum(dim=-1)


def accuracy_affected(a: torch.Tensor, b: torch.Tensor, label_unchanged: torch.Tensor,
                      label_idx: TorchIndex) -> torch.Tensor:
    a_lab = torch.argmax(a[label_idx.as_index], dim=-1)
    b_lab = torch.argmax(b[label_idx.as_index], dim=-1)
    changed = (a_lab != b_lab).float() * (~label_unchanged).float()
    return changed.sum() / (~label_unchanged).float().sum()
