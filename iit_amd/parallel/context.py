"""Context parallelism: attention over a sequence sharded across ranks (SURVEY.md §5.7 seam).

The reference has no long-context path: IOI prompts are 16 tokens, and TL's attention is dense and eager.
This module is the seam that SURVEY.md §5.7 asks for. A sequence of ``S`` tokens is split into contiguous
shards of ``S / P`` tokens, one per rank of a process group. :func:`context_parallel_attention` computes exact
causal (or bidirectional) attention for the local queries, and autograd carries the gradient back to every
rank's K/V shard.

Design (MI355X): the K/V shards are **all-gathered** once per layer, then each rank attends with its local
queries. This is the all-gather form of context parallelism. It suits a fully connected xGMI mesh: one large
collective per layer runs on all 7 links, with no P2P ring of P - 1 dependent hops. At 288 GB per GPU the full
K/V of a long sequence fits. The backward reduce-scatters the K/V gradient: ``reduce_scatter_tensor`` on RCCL,
and all-reduce + slice on gloo, which has no reduce-scatter. Heads may be grouped (GQA): ``k``/``v`` carry
``H_kv`` heads, and ``H_kv`` must divide ``H``.

Layout follows the engine's hooks: ``[batch, seq, heads, d_head]`` (``hook_q`` / ``hook_k`` / ``hook_v``).
"""
from __future__ import annotations

import math
from typing import Optional

import torch
import torch.distributed as dist


def _group_size(group) -> int:
    return dist.get_world_size(group) if dist.is_initialized() else 1


def _group_rank(group) -> int:
    return dist.get_rank(group) if dist.is_initialized() else 0


def shard_sequence(x: torch.Tensor, dim: int = 1, group=None) -> torch.Tensor:
    """This rank's contiguous shard of ``x`` along ``dim`` (the length must divide evenly)."""
    p = _group_size(group)
    if p == 1:
        return x
    n = x.shape[dim]
    if n % p:
        raise ValueError(f"sequence length {n} is not divisible by the context-parallel group size {p}")
    return x.narrow(dim, _group_rank(group) * (n // p), n // p)


class _GatherSeq(torch.autograd.Function):
    """All-gather along ``dim``; the backward returns this rank's slice of the summed gradient."""

    @staticmethod
    def forward(ctx, x, dim, group):
        ctx.dim, ctx.group = dim, group
        p = _group_size(group)
        parts = [torch.empty_like(x) for _ in range(p)]
        dist.all_gather(parts, x.contiguous(), group=group)
        return torch.cat(parts, dim=dim)

    @staticmethod
    def backward(ctx, g):
        p, r, dim = _group_size(ctx.group), _group_rank(ctx.group), ctx.dim
        n = g.shape[dim] // p
        if dist.get_backend(ctx.group) == "nccl":
            chunks = g.movedim(dim, 0).contiguous()  # shards contiguous along the leading axis
            out = torch.empty_like(chunks[:n])
            dist.reduce_scatter_tensor(out, chunks, group=ctx.group)
            return out.movedim(0, dim), None, None
        g = g.clone(memory_format=torch.contiguous_format)  # never reduce in place into an autograd-owned buffer
        dist.all_reduce(g, group=ctx.group)  # gloo: no reduce-scatter
        return g.narrow(dim, r * n, n), None, None


def gather_sequence(x: torch.Tensor, dim: int = 1, group=None) -> torch.Tensor:
    """Differentiable all-gather of sequence shards along ``dim`` (identity on one rank)."""
    if _group_size(group) == 1:
        return x
    return _GatherSeq.apply(x, dim, group)


def context_parallel_attention(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, *, causal: bool = True,
                               group=None, scale: Optional[float] = None) -> torch.Tensor:
    """Exact attention for the local query shard against the whole (gathered) sequence.

    ``q``: ``[B, S_loc, H, D]``; ``k``, ``v``: ``[B, S_loc, H_kv, D]``, the rank's shards of one sequence, rank ``r``
    holding positions ``[r * S_loc, (r + 1) * S_loc)``. Returns ``z`` ``[B, S_loc, H, D]`` (``hook_z`` layout).
    Scores and softmax are in fp32 or wider, and the output is in ``q``'s dtype."""
    B, S_loc, H, D = q.shape
    Hkv = k.shape[2]
    if H % Hkv:
        raise ValueError(f"{H} query heads are not a multiple of {Hkv} key/value heads")
    K = gather_sequence(k, 1, group)
    V = gather_sequence(v, 1, group)
    if Hkv != H:
        K = K.repeat_interleave(H // Hkv, dim=2)
        V = V.repeat_interleave(H // Hkv, dim=2)
    S = K.shape[1]
    scale = 1.0 / math.sqrt(D) if scale is None else scale
    acc = torch.promote_types(q.dtype, torch.float32)  # fp32 scores / softmax (fp64 inputs stay fp64)
    scores = torch.einsum("bqhd,bkhd->bhqk", q.to(acc), K.to(acc)) * scale
    if causal:
        q_pos = _group_rank(group) * S_loc + torch.arange(S_loc, device=q.device)
        k_pos = torch.arange(S, device=q.device)
        scores = scores.masked_fill(k_pos[None, :] > q_pos[:, None], float("-inf"))
    p = torch.softmax(scores, dim=-1)
    return torch.einsum("bhqk,bkhd->bqhd", p, V.to(acc)).to(q.dtype)
