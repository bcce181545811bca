"""Staged backward: gradient all-reduce overlapped with a graph-captured backward.

Collectives are never captured into HIP graphs (every rank must issue the same
RCCL sequence, and a captured RCCL call cannot be validated on a one-GPU box),
so a data-parallel phase replays ``graph(forward + backward)`` and reduces the
gradient arena between graphs.  Done naively the whole all-reduce waits for the
whole backward.  :class:`StagedBackward` cuts the LL model's residual stream at
a few block boundaries (``HookedTransformer._grad_cuts``): the forward stores a
detached leaf there, so ``loss.backward()`` stops at the top cut and each lower
stage resumes with ``torch.autograd.backward(resid, leaf.grad)`` as its own
captured graph.  The flat arena is in module order (embeddings, block 0 ... block
L-1, final norm, unembed), so each stage's parameter gradients are one contiguous
arena range; the host launches that range's bucketed RCCL all-reduce right after
the stage's graph and the next stage's graph runs on the compute stream while
RCCL moves it over xGMI::

    compute: [fwd + bwd top] [bwd stage 2] [bwd stage 1] [bwd stage 0]   wait  [clip + Adam]
    RCCL:                    [reduce top ] [reduce 2   ] [reduce 1   ] [reduce 0]

Only the bottom stage's reduction is exposed.  The cut is exact: the gradient
reaching ``resid`` through the leaf is the one plain autograd would pass.
("bucketed all-reduce on a comm stream overlapped with backward".)
"""
from __future__ import annotations

from typing import List, Optional, Tuple

import torch


class StagedBackward:
    def __init__(self, model, n_stages: int = 6):
        self.model = model
        L = len(getattr(model, "blocks", []))
        n_stages = max(1, min(int(n_stages), L))
        self.cuts: List[int] = sorted({round(L * i / n_stages) for i in range(1, n_stages)} - {0, L})
        flat = getattr(model, "_flat_params", None)
        self.flat = flat
        self.edges: List[int] = []
        if flat is not None and self.cuts:
            for k in self.cuts:
                offs = [flat.offset_of(p) for p in model.blocks[k].parameters() if p.requires_grad and flat.owns(p)]
                self.edges.append(min(offs) if offs else flat.numel)
        self.active = bool(self.cuts) and flat is not None and all(
            a < b for a, b in zip(self.edges, self.edges[1:]))

    # ------------------------------------------------------------------ forward side
    def arm(self) -> None:
        self.model._grad_cuts = frozenset(self.cuts)
        self.model._cut_log = []

    def disarm(self) -> None:
        self.model.__dict__.pop("_grad_cuts", None)

    # ------------------------------------------------------------------ backward side
    def stages(self) -> List[int]:
        """Cut layers in backward order (top first)."""
        return sorted(self.cuts, reverse=True)

    def run_stage(self, k: int) -> None:
        """Resume the backward below cut ``k`` for every grad-enabled forward that crossed it."""
        for li, resid, leaf in list(getattr(self.model, "_cut_log", [])):
            if li == k and leaf.grad is not None and resid.requires_grad:
                torch.autograd.backward(resid, leaf.grad)

    def release(self) -> None:
        self.model._cut_log = []

    def ranges(self) -> List[Tuple[int, int]]:
        """Arena range per backward unit: [top, stage for each cut descending ..., bottom]."""
        n = self.flat.numel
        edges = self.edges
        out = [(edges[-1], n)]
        for i in range(len(edges) - 1, 0, -1):
            out.append((edges[i - 1], edges[i]))
        out.append((0, edges[0]))
        return out


def staged_for(pair, n_stages: Optional[int] = None) -> Optional[StagedBackward]:
    """A StagedBackward for the pair's LL model, or None when it does not apply."""
    import os
    n = int(os.environ.get("IIT_DP_STAGES", "6")) if n_stages is None else n_stages
    model = pair._ll_module() if hasattr(pair, "_ll_module") else getattr(pair, "ll_model", None)
    if n <= 1 or model is None or not hasattr(model, "blocks"):
        return None
    st = StagedBackward(model, n)
    return st if st.active else None
