"""Synthetic IOI dataset (parity: ``/root/reference/iit/tasks/ioi/ioi_dataset_tl.py:171-377``).

Sample generation follows the reference: ``random.seed(seed)``; per sample a
template is drawn, every noun slot is filled, two distinct names are drawn,
``[A]`` <- names[0], ``[B]`` <- names[1]; ``IO = " " + names[0]``, ``S = " " + names[1]``.

Design differences (SURVEY.md §2.7 Q18, §3.1 hot loop 3):
* prompts are tokenised **once** into a device-resident ``[N, S+1]`` int tensor;
  items are views, and ``gather(idx)`` assembles a whole batch with one
  ``index_select`` (no per-sample tokenisation / H2D copies / one-hot);
* labels default to **index** form ``[S]`` (next token ids).  ``label_format="onehot"``
  reproduces the reference's dense ``[S, vocab]`` float one-hot;
* prompts are left unpadded (BOS + 16 tokens), so the last target is the IO name
  ("Padding caveat").
"""
from __future__ import annotations

import random
from typing import Dict, List, Optional, Sequence

import torch
from torch.utils.data import Dataset

from ...config import DEVICE
from .ioi_config import NAMES, NOUNS, TEMPLATES, vocabulary_words
from .tokenizer import SyntheticTokenizer


def default_tokenizer() -> SyntheticTokenizer:
    return SyntheticTokenizer(vocabulary_words())


class IOIDataset(Dataset):
    def __init__(self, tokenizer=None, templates: Optional[List[str]] = None, names: Optional[List[str]] = None,
                 nouns: Optional[Dict[str, List[str]]] = None, num_samples: int = 1000, symmetric: bool = False,
                 prepend_bos: bool = True, seed: int = 42, device=None):
        self.tokenizer = tokenizer if tokenizer is not None else default_tokenizer()
        self.prepend_bos = prepend_bos
        self.templates = list(templates) if templates is not None else list(TEMPLATES)
        self.names = list(names) if names is not None else list(NAMES)
        self.nouns = dict(nouns) if nouns is not None else {k: list(v) for k, v in NOUNS.items()}
        self.device = torch.device(device) if device is not None else DEVICE
        self.samples: List[Dict[str, str]] = []
        random.seed(seed)
        for _ in range(num_samples // 2 if symmetric else num_samples):
            self.samples.extend(self._draw(symmetric))
        self._build_tensors()

    def _draw(self, symmetric: bool):
        template = random.choice(self.templates)
        for slot, options in self.nouns.items():
            template = template.replace(f"[{slot}]", random.choice(options))
        a, b = random.sample(self.names, 2)
        out = [{"text": template.replace("[A]", a).replace("[B]", b), "IO": " " + a, "S": " " + b}]
        if symmetric:
            out.append({"text": template.replace("[A]", b).replace("[B]", a), "IO": " " + b, "S": " " + a})
        return out

    def _build_tensors(self):
        tok = self.tokenizer
        rows = []
        for s in self.samples:
            ids = tok.encode(s["text"])
            rows.append(([tok.bos_token_id] if self.prepend_bos else []) + ids)
        width = max(len(r) for r in rows) if rows else 0
        if any(len(r) != width for r in rows):
            rows = [r + [tok.pad_token_id] * (width - len(r)) for r in rows]
        self.prompts = torch.tensor(rows, dtype=torch.long).to(self.device)
        self.io_ids = torch.tensor([tok.encode(s["IO"])[0] for s in self.samples], dtype=torch.long).to(self.device)
        self.s_ids = torch.tensor([tok.encode(s["S"])[0] for s in self.samples], dtype=torch.long).to(self.device)

    def __len__(self) -> int:
        return len(self.samples)

    def __getitem__(self, idx):
        return {
            "prompt": self.prompts[idx],
            "IO": self.io_ids[idx:idx + 1],
            "S": self.s_ids[idx:idx + 1],
            "idx_to_ablate": int(self.prompts.shape[1]) - 2,
        }

    @staticmethod
    def get_default_names():
        return list(NAMES)

    @staticmethod
    def get_default_templates():
        return list(TEMPLATES)

    @staticmethod
    def get_default_nouns():
        return {k: list(v) for k, v in NOUNS.items()}


class IOIDatasetWrapper(IOIDataset):
    """Yields ``(x, y, iv)`` = ``(prompt[:-1], next-token labels, IO token)`` per sample."""

    def __init__(self, *args, label_format: str = "index", **kwargs):
        if label_format not in ("index", "onehot"):
            raise ValueError("label_format must be 'index' or 'onehot'")
        self.label_format = label_format
        super().__init__(*args, **kwargs)

    def _labels(self, y: torch.Tensor) -> torch.Tensor:
        if self.label_format == "onehot":
            return torch.nn.functional.one_hot(y, num_classes=self.tokenizer.vocab_size).float()
        return y

    def __getitem__(self, idx):
        p = self.prompts[idx]
        return p[:-1], self._labels(p[1:]), self.io_ids[idx:idx + 1]

    def token_ids(self) -> torch.Tensor:
        """Distinct input token ids (the only embedding rows that can receive gradient)."""
        return torch.unique(self.prompts[:, :-1])

    def gather(self, idx: torch.Tensor):
        """Batched ``__getitem__``: one device gather for a whole batch of indices."""
        p = self.prompts.index_select(0, idx.to(self.prompts.device))
        return p[:, :-1], self._labels(p[:, 1:]), self.io_ids.index_select(0, idx.to(self.prompts.device))[:, None]
