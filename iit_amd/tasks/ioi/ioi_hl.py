"""IOI high-level causal model (parity: ``/root/reference/iit/tasks/ioi/ioi_hl.py:16-130``).

Hooks: ``all_nodes_hook`` (input tokens), ``hook_duplicate``, ``hook_previous``
(registered, unused), ``hook_s_inhibition``, ``hook_name_mover``.

All heads are **sync-free** (SURVEY.md §2.3 K16): the reference's
``positions.nonzero()`` scatter (a device->host sync per call) becomes a masked
max over earlier positions, and the name-mover's CPU ``meshgrid`` index becomes
a device scatter.  Semantics are identical, including the "last duplicate wins"
write order of the reference.

``forward(args, last_only=True)`` computes the name-mover logits only at the last
position (``[B, V]`` instead of ``[B, S, V]``) – everything the IOI losses and
IIA read – so the HL side of a training step never materialises 823 MB of fp32
logits.  Both runs of an intervention must use the same mode.
"""
from __future__ import annotations

import torch
from torch import nn

from ...hooks.hook_points import HookedRootModule, HookPoint
from ..hl_model import HLModel


class DuplicateHead(nn.Module):
    def forward(self, tokens: torch.Tensor) -> torch.Tensor:
        """At each position, the latest earlier position holding the same token (else -1)."""
        S = tokens.shape[-1]
        same = tokens[..., :, None] == tokens[..., None, :]  # [.., i, j]
        pos = torch.arange(S, device=tokens.device)
        earlier = pos[:, None] < pos[None, :]  # i < j
        cand = torch.where(same & earlier, pos[:, None].expand(S, S), torch.full_like(same, -1, dtype=torch.long))
        return cand.max(dim=-2).values.to(tokens.dtype)


class PreviousHead(nn.Module):
    def forward(self, tokens: torch.Tensor) -> torch.Tensor:
        out = torch.full_like(tokens, -1)
        out[..., 1:] = tokens[..., :-1]
        return out


class InductionHead(nn.Module):
    """Omitted in IOI (redundant with duplicate heads), kept for API parity."""


class SInhibitionHead(nn.Module):
    def forward(self, tokens: torch.Tensor, duplicate: torch.Tensor) -> torch.Tensor:
        return torch.where(duplicate == -1, torch.full_like(tokens, -1), tokens)


class NameMoverHead(nn.Module):
    def __init__(self, names, d_vocab: int = 40):
        super().__init__()
        self.d_vocab_out = d_vocab
        names = torch.as_tensor(names)
        self.register_buffer("names", names.clone(), persistent=False)
        # vocab-sized membership table: a gather instead of torch.isin (sort-based, not graph-capturable)
        table = torch.zeros(max(d_vocab, int(names.max()) + 1 if names.numel() else 1), dtype=torch.float32)
        table[names.long()] = 1.0
        self.register_buffer("name_table", table, persistent=False)

    def deltas(self, tokens: torch.Tensor, s_inhibition: torch.Tensor):
        """Per-position logit increments: +10 at each name token, -15 at each inhibited token."""
        is_name = self.name_table.to(tokens.device)[tokens]
        inhibited = s_inhibition.ne(-1).float()
        return 10.0 * is_name, -15.0 * inhibited

    def forward(self, tokens: torch.Tensor, s_inhibition: torch.Tensor, last_only: bool = False) -> torch.Tensor:
        B, S = tokens.shape
        V = self.d_vocab_out
        up, down = self.deltas(tokens, s_inhibition)
        inh_idx = torch.where(s_inhibition.ne(-1), s_inhibition, torch.full_like(s_inhibition, V - 1))
        if last_only:
            out = torch.zeros(B, V, device=tokens.device)
            out.scatter_add_(1, tokens, up)
            out.scatter_add_(1, inh_idx, down)
            return out
        out = torch.zeros(B, S, V, device=tokens.device)
        out.scatter_add_(2, tokens[..., None], up[..., None])
        out.scatter_add_(2, inh_idx[..., None], down[..., None])
        return torch.cumsum(out, dim=1)


class IOI_HL(HookedRootModule, HLModel):
    supports_last_only = True

    def __init__(self, d_vocab: int, names):
        super().__init__()
        self.all_nodes_hook = HookPoint()
        self.duplicate_head = DuplicateHead()
        self.hook_duplicate = HookPoint()
        self.hook_previous = HookPoint()
        self.s_inhibition_head = SInhibitionHead()
        self.hook_s_inhibition = HookPoint()
        self.name_mover_head = NameMoverHead(names, d_vocab)
        self.hook_name_mover = HookPoint()
        self.d_vocab = d_vocab
        self.setup()

    def is_categorical(self) -> bool:
        return True

    def forward(self, args, verbose: bool = False, last_only: bool = False):
        tokens = args[0]
        single = tokens.dim() == 1
        if single:
            tokens = tokens[None]
        tokens = self.all_nodes_hook(tokens)
        dup = self.hook_duplicate(self.duplicate_head(tokens))
        s_inh = self.hook_s_inhibition(self.s_inhibition_head(tokens, dup))
        out = self.hook_name_mover(self.name_mover_head(tokens, s_inh, last_only=last_only))
        if verbose:
            print(f"duplicate: {dup}\ns_inhibition: {s_inh}")
        return out[0] if single else out
