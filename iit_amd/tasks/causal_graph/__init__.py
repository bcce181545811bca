"""Eight-node arithmetic causal graph (the HL side of ``BASELINE.json`` config 5).

Input ``[BOS, a, b, c, d, =]`` (digit tokens), the answer token is predicted at the
last position; ``seq_len > 6`` puts a context of random filler tokens between BOS and
the operands (long-context runs: the operands stay the last five positions).  HL
graph, 8 hooked nodes::

    a   b   c   d            leaves   (hook_a .. hook_d)
     \\ /     \\ /
      s1      s2             s1 = (a + b) % 10, s2 = (c + d) % 10
        \\    /
          p                  p   = (s1 * s2) % 10
          |   a
          out                out = (p + a) % 10

:func:`make_causal_graph_corr` aligns it with any hooked transformer (Llama or
GPT-2 family): leaves -> ``hook_embed`` at their positions, ``s1`` / ``s2`` ->
the two halves of the heads of an early layer's ``attn.hook_z`` at the last
position, ``p`` / ``out`` -> MLP neurons (``mlp.hook_post``) of later layers at the
last position.  :class:`CausalGraphModelPair` trains Strict IIT on it with
last-position logits.
"""
from __future__ import annotations

from typing import Dict, Optional

import numpy as np
import torch
import torch.nn.functional as F

from ...config import DEVICE
from ...core.correspondence import Correspondence
from ...core.index import Ix
from ...core.metric import MetricStore, MetricStoreCollection, MetricType
from ...core.nodes import HLNode, LLNode
from ...hooks.hook_points import HookedRootModule, HookPoint
from ...model_pairs.strict_iit_model_pair import StrictIITModelPair
from ..hl_model import HLModel

BOS, EQ, DIGIT0 = 1, 2, 10
FILLER = (3, 10)  # filler token range of long-context prompts (never a digit, BOS or "=")
NODES = ("hook_a", "hook_b", "hook_c", "hook_d", "hook_s1", "hook_s2", "hook_p", "hook_out")
SEQ = 6


class CausalGraphHL(HookedRootModule, HLModel):
    def __init__(self, d_vocab: int):
        super().__init__()
        self.d_vocab = d_vocab
        for n in NODES:
            setattr(self, n, HookPoint())
        self.setup()

    def is_categorical(self) -> bool:
        return True

    def get_idx_to_intermediate(self, name: str):
        i = NODES.index(name)
        return lambda iv: iv[:, i]

    def forward(self, args):
        x = args[0]
        # the operands are the four positions before the final "=" (positions 1..4 of the 6-token prompt)
        a, b, c, d = (self.hook_a(x[:, -5] - DIGIT0), self.hook_b(x[:, -4] - DIGIT0), self.hook_c(x[:, -3] - DIGIT0),
                      self.hook_d(x[:, -2] - DIGIT0))
        s1 = self.hook_s1((a + b) % 10)
        s2 = self.hook_s2((c + d) % 10)
        p = self.hook_p((s1 * s2) % 10)
        out = self.hook_out((p + a) % 10)
        return F.one_hot(out + DIGIT0, self.d_vocab).float() * 10.0  # [B, V] logits of the answer token


class CausalGraphDataset(torch.utils.data.Dataset):
    """``(x [seq_len], y, iv [8])`` items; all 10^4 operand tuples are distinct, ``n`` of them drawn by ``seed``;
    ``seq_len > 6`` inserts ``seq_len - 6`` random filler tokens after BOS."""

    def __init__(self, n: int = 10000, seed: int = 0, device=None, seq_len: int = SEQ):
        if seq_len < SEQ:
            raise ValueError(f"seq_len must be >= {SEQ}")
        rng = np.random.default_rng(seed)
        codes = rng.permutation(10 ** 4)[:n] if n <= 10 ** 4 else rng.integers(0, 10 ** 4, n)
        dig = np.stack([(codes // 10 ** k) % 10 for k in (3, 2, 1, 0)], axis=1)
        a, b, c, d = (torch.as_tensor(dig[:, i]) for i in range(4))
        s1, s2 = (a + b) % 10, (c + d) % 10
        p = (s1 * s2) % 10
        out = (p + a) % 10
        dev = torch.device(device) if device is not None else torch.device(DEVICE)
        x = torch.stack([torch.full_like(a, BOS), a + DIGIT0, b + DIGIT0, c + DIGIT0, d + DIGIT0,
                         torch.full_like(a, EQ)], dim=1)
        if seq_len > SEQ:
            fill = torch.as_tensor(rng.integers(FILLER[0], FILLER[1], (x.shape[0], seq_len - SEQ)))
            x = torch.cat([x[:, :1], fill, x[:, 1:]], dim=1)
        self.x = x.long().to(dev)
        self.y = (out + DIGIT0).long().to(dev)
        self.iv = torch.stack([a, b, c, d, s1, s2, p, out], dim=1).long().to(dev)

    def __len__(self) -> int:
        return self.x.shape[0]

    def __getitem__(self, i):
        return self.x[i], self.y[i], self.iv[i]

    def gather(self, idx: torch.Tensor):
        idx = idx.to(self.x.device)
        return self.x.index_select(0, idx), self.y.index_select(0, idx), self.iv.index_select(0, idx)

    def token_ids(self) -> torch.Tensor:
        return torch.unique(self.x)


def make_causal_graph_corr(n_layers: int, n_heads: int, d_mlp: int, seq_len: int = SEQ) -> Correspondence:
    """Default alignment of the 8 HL nodes with an ``n_layers`` hooked transformer (prompts of ``seq_len``)."""
    early = max(0, n_layers // 4)
    mid = min(n_layers - 1, max(early + 1, n_layers // 2)) if n_layers > 1 else 0
    last = n_layers - 1
    h = max(1, n_heads // 2)
    corr: Dict[HLNode, set] = {}
    for i, n in enumerate(NODES[:4]):
        corr[HLNode(n, 10)] = {LLNode("hook_embed", Ix[:, seq_len - 5 + i])}
    corr[HLNode("hook_s1", 10)] = {LLNode(f"blocks.{early}.attn.hook_z", Ix[:, -1, :h, :])}
    corr[HLNode("hook_s2", 10)] = {LLNode(f"blocks.{early}.attn.hook_z", Ix[:, -1, h:, :])}
    if mid == last:  # shallow models: p and out share the last MLP, split by neurons
        half = d_mlp // 2
        corr[HLNode("hook_p", 10)] = {LLNode(f"blocks.{mid}.mlp.hook_post", Ix[:, -1, :half])}
        corr[HLNode("hook_out", 10)] = {LLNode(f"blocks.{last}.mlp.hook_post", Ix[:, -1, half:])}
    else:
        corr[HLNode("hook_p", 10)] = {LLNode(f"blocks.{mid}.mlp.hook_post", Ix[:, -1])}
        corr[HLNode("hook_out", 10)] = {LLNode(f"blocks.{last}.mlp.hook_post", Ix[:, -1])}
    return Correspondence(corr, suffixes={"attn": "attn.hook_z", "mlp": "mlp.hook_post"})


class CausalGraphModelPair(StrictIITModelPair):
    """Strict IIT + behaviour on the causal-graph task; every loss reads the last position only."""

    def ll_logits_mode(self) -> str:
        return "last" if self.native() else "full"

    @staticmethod
    def get_label_idxs():
        return Ix[:, -1]

    @staticmethod
    def _last(out):
        return out[:, -1] if out.dim() == 3 else out

    @property
    def loss_fn(self):
        if self._loss_fn_override is not None:
            return self._loss_fn_override

        def ce(output, target):
            output = self._last(output).float()
            if target.dtype.is_floating_point:
                target = self._last(target).argmax(-1)
            elif target.dim() == 2:
                target = target[:, -1]
            from ...ops import cross_entropy
            return cross_entropy(output, target)
        return ce

    @loss_fn.setter
    def loss_fn(self, value):
        self._loss_fn_override = value

    @staticmethod
    def make_test_metrics():
        return MetricStoreCollection([MetricStore("val/iit_loss", MetricType.LOSS),
                                      MetricStore("val/IIA", MetricType.ACCURACY),
                                      MetricStore("val/accuracy", MetricType.ACCURACY)])

    def run_eval_step(self, base_input, ablation_input, loss_fn):
        hl_node = self.sample_hl_name()
        hl_output, ll_output = self.do_intervention(base_input, ablation_input, hl_node)
        ll_last = self._last(ll_output)
        label = hl_output.argmax(-1)
        iia = (ll_last.argmax(-1) == label).float().mean()
        out = self._last(self.ll_forward(base_input[0]))
        acc = (out.argmax(-1) == base_input[1]).float().mean()
        return {"val/iit_loss": loss_fn(ll_last, hl_output).detach(), "val/IIA": iia, "val/accuracy": acc}


def make_causal_graph_task(ll_model, n_samples: int = 10000, seed: int = 0, device=None, seq_len: int = SEQ):
    """(dataset, HL model, corr) for a hooked-transformer LL model."""
    cfg = ll_model.cfg
    ds = CausalGraphDataset(n_samples, seed, device=device, seq_len=seq_len)
    hl = CausalGraphHL(cfg.d_vocab_out)
    corr = make_causal_graph_corr(cfg.n_layers, cfg.n_heads, cfg.d_mlp, seq_len=seq_len)
    return ds, hl, corr
