"""MQNLI-style natural-language inference causal model (``BASELINE.json`` config 4: MQNLI <-> BERT-base).

Offline, synthetic and self-consistent (no dataset download): sentences follow the
MQNLI template ``Q (Adj) N (not) (Adv) V`` for premise and hypothesis; the label
is produced by a compositional natural-logic causal model whose composition
tables are model-checked (:mod:`.natural_logic`).  HL causal graph (10 hooked
nodes)::

    q      adj   noun      neg     adv   verb            (lexical, per aligned word pair)
     \\        \\  /          |        \\  /
      \\        np           |         vp
       \\        \\           \\        /
        \\        \\            negvp
         \\        \\          /
          `-------- rel -----'                          rel = Q_table[q_p, q_h, np, negvp]
                     |
                   label (entailment / contradiction / neutral)

Input layout (BERT sentence pair, 15 tokens)::

    0 [CLS] | 1 Q 2 Adj 3 N 4 Neg 5 Adv 6 V | 7 [SEP] | 8 Q 9 Adj 10 N 11 Neg 12 Adv 13 V | 14 [SEP]

:func:`make_mqnli_corr` aligns each HL node with the aligned premise/hypothesis
positions of one encoder layer's ``hook_normalized_resid_post`` (lexical nodes
early, np / vp middle, negvp later, the final relation on [CLS] in the last
layer), in the spirit of Geiger et al.'s BERT <-> MQNLI alignment.
"""
from __future__ import annotations

from typing import Dict

import numpy as np
import torch

from ...config import DEVICE
from ...core.correspondence import Correspondence
from ...core.index import Ix
from ...core.nodes import HLNode, LLNode
from ...hooks.hook_points import HookedRootModule, HookPoint
from ..hl_model import HLModel
from . import natural_logic as nl

PAD, CLS, SEP, EMPTY = 0, 1, 2, 3
Q0 = 4                      # some, every, no, not every -> 4..7
NOT = 8
ADJ0, N_ADJ = 9, 8          # 9..16
NOUN0, N_NOUN = 17, 8       # 17..24
ADV0, N_ADV = 25, 4         # 25..28
VERB0, N_VERB = 29, 8       # 29..36
VOCAB = 37
SEQ = 15
P_POS = {"q": 1, "adj": 2, "noun": 3, "neg": 4, "adv": 5, "verb": 6}
H_POS = {k: v + 7 for k, v in P_POS.items()}
NODES = ("hook_q", "hook_adj", "hook_noun", "hook_neg", "hook_adv", "hook_verb", "hook_np", "hook_vp", "hook_negvp",
         "hook_rel")
N_CLASSES = {"hook_q": 16, "hook_neg": 4, "hook_rel": 7}


def _modifier_relation(mp: torch.Tensor, mh: torch.Tensor) -> torch.Tensor:
    """Intersective modifier pair -> relation (EMPTY = no modifier)."""
    out = torch.full_like(mp, nl.IND)
    out = torch.where(mp == mh, torch.full_like(mp, nl.EQ), out)
    out = torch.where((mp != EMPTY) & (mh == EMPTY), torch.full_like(mp, nl.FWD), out)
    out = torch.where((mp == EMPTY) & (mh != EMPTY), torch.full_like(mp, nl.REV), out)
    return out


class MQNLI_HL(HookedRootModule, HLModel):
    """The natural-logic causal model; forward returns 3-way label logits ``[B, 3]``."""

    def __init__(self):
        super().__init__()
        for n in NODES:
            setattr(self, n, HookPoint())
        self.register_buffer("T_int", torch.as_tensor(nl.intersective_table()), persistent=False)
        self.register_buffer("T_neg", torch.as_tensor(nl.negation_table()), persistent=False)
        self.register_buffer("T_q", torch.as_tensor(nl.quantifier_table()), persistent=False)
        self.register_buffer("label_of", torch.tensor([nl.label_of(r) for r in range(7)]), persistent=False)
        self.setup()

    def is_categorical(self) -> bool:
        return True

    def forward(self, args):
        x = args[0]
        T_int, T_neg, T_q, lab = self._tables(x.device)
        tok = lambda side, k: x[:, (P_POS if side == "p" else H_POS)[k]]  # noqa: E731
        q = self.hook_q((tok("p", "q") - Q0) * 4 + (tok("h", "q") - Q0))
        adj = self.hook_adj(_modifier_relation(tok("p", "adj"), tok("h", "adj")))
        noun = self.hook_noun(torch.where(tok("p", "noun") == tok("h", "noun"), nl.EQ, nl.IND))
        neg = self.hook_neg((tok("p", "neg") == NOT).long() * 2 + (tok("h", "neg") == NOT).long())
        adv = self.hook_adv(_modifier_relation(tok("p", "adv"), tok("h", "adv")))
        verb = self.hook_verb(torch.where(tok("p", "verb") == tok("h", "verb"), nl.EQ, nl.IND))
        np_rel = self.hook_np(T_int[adj, noun])
        vp_rel = self.hook_vp(T_int[adv, verb])
        negvp = self.hook_negvp(T_neg[neg // 2, neg % 2, vp_rel])
        rel = self.hook_rel(T_q[q // 4, q % 4, np_rel, negvp])
        return torch.nn.functional.one_hot(lab[rel], 3).float() * 10.0

    def _tables(self, dev):
        """Composition tables on ``dev`` (cached: the first, eager call copies them; graph replays never do)."""
        cache = self.__dict__.setdefault("_dev_tables", {})
        if dev not in cache:
            cache[dev] = tuple(t.to(dev) for t in (self.T_int, self.T_neg, self.T_q, self.label_of))
        return cache[dev]

    def get_idx_to_intermediate(self, name: str):
        i = NODES.index(name)
        return lambda iv: iv[:, i]


class MQNLIDataset(torch.utils.data.Dataset):
    """Premise / hypothesis pairs; each hypothesis slot copies the premise word with probability ``p_same``.
    Labels (3-way) and every HL node value come from :class:`MQNLI_HL`; classes are rebalanced."""

    def __init__(self, n: int = 20000, seed: int = 0, p_same: float = 0.6, balance: bool = True, device=None):
        rng = np.random.default_rng(seed)
        dev = torch.device(device) if device is not None else torch.device(DEVICE)
        hl = MQNLI_HL()
        keep_x = []
        counts = np.zeros(3, dtype=np.int64)
        target = n // 3 + 1
        while sum(len(k) for k in keep_x) < n:
            m = max(4 * n, 1024)
            x = self._sample(rng, m, p_same)
            with torch.no_grad():
                y = hl((torch.as_tensor(x), None, None)).argmax(-1).numpy()
            if balance:
                sel = []
                for i, c in enumerate(y):
                    if counts[c] < target:
                        counts[c] += 1
                        sel.append(i)
                x = x[sel]
            keep_x.append(x)
            if not balance:
                break
        x = torch.as_tensor(np.concatenate(keep_x)[:n])
        with torch.no_grad():
            y, cache = hl.run_with_cache((x, None, None))
        self.x = x.long().to(dev)
        self.y = y.argmax(-1).long().to(dev)
        self.iv = torch.stack([cache[name] for name in NODES], dim=1).long().to(dev)

    @staticmethod
    def _sample(rng, m: int, p_same: float) -> np.ndarray:
        def word(base, k, optional):
            w = base + rng.integers(0, k, m)
            if optional:
                w = np.where(rng.random(m) < 0.5, EMPTY, w)
            return w

        def prem():
            return {"q": Q0 + rng.integers(0, 4, m), "adj": word(ADJ0, N_ADJ, True), "noun": word(NOUN0, N_NOUN, False),
                    "neg": np.where(rng.random(m) < 0.5, NOT, EMPTY), "adv": word(ADV0, N_ADV, True),
                    "verb": word(VERB0, N_VERB, False)}

        p, alt = prem(), prem()
        h = {k: np.where(rng.random(m) < p_same, p[k], alt[k]) for k in p}
        x = np.zeros((m, SEQ), dtype=np.int64)
        x[:, 0], x[:, 7], x[:, 14] = CLS, SEP, SEP
        for k in P_POS:
            x[:, P_POS[k]] = p[k]
            x[:, H_POS[k]] = h[k]
        return x

    def __len__(self) -> int:
        return self.x.shape[0]

    def __getitem__(self, i):
        return self.x[i], self.y[i], self.iv[i]

    def gather(self, idx: torch.Tensor):
        idx = idx.to(self.x.device)
        return self.x.index_select(0, idx), self.y.index_select(0, idx), self.iv.index_select(0, idx)

    def token_ids(self) -> torch.Tensor:
        return torch.unique(self.x)


def make_mqnli_corr(n_layers: int) -> Correspondence:
    early = max(0, n_layers // 4)
    mid = min(n_layers - 1, max(early + 1, n_layers // 2))
    late = min(n_layers - 1, max(mid + 1, (3 * n_layers) // 4))
    last = n_layers - 1
    site = "blocks.{}.hook_normalized_resid_post"
    pos = lambda *ks: [P_POS[k] for k in ks] + [H_POS[k] for k in ks]  # noqa: E731
    corr: Dict[HLNode, set] = {}
    for k in ("q", "adj", "noun", "neg", "adv", "verb"):
        corr[HLNode(f"hook_{k}", N_CLASSES.get(f"hook_{k}", 7))] = {LLNode(site.format(early), Ix[:, pos(k)])}
    corr[HLNode("hook_np", 7)] = {LLNode(site.format(mid), Ix[:, pos("adj", "noun")])}
    corr[HLNode("hook_vp", 7)] = {LLNode(site.format(mid), Ix[:, pos("adv", "verb")])}
    corr[HLNode("hook_negvp", 7)] = {LLNode(site.format(late), Ix[:, pos("neg")])}
    corr[HLNode("hook_rel", 7)] = {LLNode(site.format(last), Ix[:, [0]])}
    return Correspondence(corr, suffixes={"attn": "attn.hook_z", "mlp": "mlp.hook_post"})


def make_mqnli_task(ll_model, n_samples: int = 20000, seed: int = 0, device=None):
    """(dataset, HL model, corr) for a :class:`iit_amd.models.bert.HookedEncoder` with ``n_classes=3``."""
    ll_model.sep_token_id = SEP
    ds = MQNLIDataset(n_samples, seed, device=device)
    return ds, MQNLI_HL(), make_mqnli_corr(ll_model.cfg.n_layers)
