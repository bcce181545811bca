"""Docstring-completion HL circuit (parity: ``/root/reference/iit/tasks/docstring/docstring_hl.py:13-142``).

Heads are dense, sync-free tensor programs (no ``nonzero`` / numpy round trip):

* ``InductionHead(tokens, prev_tok_out)``: at position ``a2`` copy ``tokens[b1]``
  where ``prev_tok_out[b1] == tokens[a2]`` and ``b1 < a2`` (latest such ``b1``,
  the deterministic choice the reference's TODO asks for; -1 if none);
* ``ArgMoverHead``: for each target position ``s2``, every earlier position
  ``s1`` with ``def_patterns[s1] == induction_output[s2]`` except the last such
  ``s1`` raises ``logits[s2, tokens[s1]]`` by ``logit_increase`` (once per token,
  like the reference's indexed ``+=``);
* ``Docstring_HL`` wires previous-token heads, induction and arg mover with hooks
  ``hook_pre, hook_prev1, hook_prev2, hook_prev_doc, hook_induction, hook_arg_mover``.
  Unlike the reference it calls ``setup()`` (so ``hook_dict`` is populated and it
  can be used in a model pair) and its debug prints are behind ``verbose``.
"""
from __future__ import annotations

import torch
from torch import nn

from ...hooks.hook_points import HookedRootModule, HookPoint
from ..hl_model import HLModel
from ..ioi.ioi_hl import PreviousHead


class InductionHead(nn.Module):
    def forward(self, tokens: torch.Tensor, prev_tok_out: torch.Tensor) -> torch.Tensor:
        S = tokens.shape[-1]
        matches = prev_tok_out[..., :, None] == tokens[..., None, :]  # [b, s1, s2]
        matches = torch.triu(matches, diagonal=1)
        pos = torch.arange(S, device=tokens.device)
        last_s1 = torch.where(matches, pos[:, None], torch.full_like(pos[:, None], -1)).max(dim=-2).values  # [b, s2]
        copied = tokens.gather(-1, last_s1.clamp(min=0))
        return torch.where(last_s1 >= 0, copied, torch.full_like(tokens, -1))


class ArgMoverHead(nn.Module):
    def __init__(self, d_vocab: int = 40, logit_increase: float = 50):
        super().__init__()
        self.d_vocab_out = d_vocab
        self.logit_increase = logit_increase

    def forward(self, tokens: torch.Tensor, def_patterns: torch.Tensor, induction_output: torch.Tensor) -> torch.Tensor:
        S = tokens.shape[-1]
        eq = induction_output[..., None, :] == def_patterns[..., :, None]  # [b, s1, s2]
        eq = torch.triu(eq, diagonal=1)
        pos = torch.arange(S, device=tokens.device)
        last = torch.where(eq, pos[:, None], torch.full_like(pos[:, None], -1)).max(dim=-2, keepdim=True).values
        keep = eq & (pos[:, None] != last)  # drop the last appearance of each (b, s2) group
        onehot = torch.nn.functional.one_hot(tokens.long(), self.d_vocab_out).float()  # [b, s1, V]
        hit = torch.einsum("bst,bsv->btv", keep.float(), onehot) > 0
        return hit.float() * self.logit_increase


class Docstring_HL(HookedRootModule, HLModel):
    def __init__(self, d_vocab: int = 40, logit_increase: float = 50):
        super().__init__()
        self.hook_pre = HookPoint()
        self.prev_def1 = PreviousHead()
        self.hook_prev1 = HookPoint()
        self.prev_def2 = PreviousHead()
        self.hook_prev2 = HookPoint()
        self.prev_doc = PreviousHead()
        self.hook_prev_doc = HookPoint()
        self.induction = InductionHead()
        self.hook_induction = HookPoint()
        self.arg_mover = ArgMoverHead(d_vocab, logit_increase)
        self.hook_arg_mover = HookPoint()
        self.setup()

    def is_categorical(self) -> bool:
        return True

    def forward(self, args, verbose: bool = False):
        tokens_in = args[0]
        assert tokens_in.dim() == 2, f"Expected input to be batch seq, got {tokens_in.shape}"
        tokens = self.hook_pre(tokens_in)
        prev1 = self.hook_prev1(self.prev_def1(tokens))
        prev2 = self.hook_prev2(self.prev_def2(prev1))
        prev_doc = self.hook_prev_doc(self.prev_doc(tokens))
        induction_out = self.hook_induction(self.induction(tokens, prev_doc))
        if verbose:
            print(f"{tokens=}\n{prev_doc=}\n{prev2=}\n{induction_out=}")
        return self.hook_arg_mover(self.arg_mover(tokens, prev2, induction_out))
