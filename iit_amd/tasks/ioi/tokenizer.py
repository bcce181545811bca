"""Offline GPT-2-shaped word tokenizer for the synthetic IOI task.

The reference tokenizes IOI prompts with the HF GPT-2 BPE tokenizer
(``/root/reference/iit/tasks/ioi/ioi_dataset_tl.py:219,234-244``), which is not
available without network access.  This
tokenizer keeps the tensor contract instead: a 50,257-entry vocabulary,
``bos == eos == pad == 50256``, and GPT-2-style pre-tokenisation (a word carries
its leading space, punctuation is its own token), so every name and template
word is exactly one token and an IOI prompt is BOS + 16 tokens.

Ids are stable across processes: known words are registered in a fixed order and
hashed (crc32) into the id space with deterministic linear probing.
"""
from __future__ import annotations

import re
import zlib
from typing import Dict, Iterable, List, Optional

_PIECE_RE = re.compile(r" ?[A-Za-z]+| ?[0-9]+| ?[^\sA-Za-z0-9]+|\s+")


class SyntheticTokenizer:
    vocab_size = 50257

    def __init__(self, known_words: Iterable[str] = (), reserved: int = 256):
        self.bos_token_id = 50256
        self.eos_token_id = 50256
        self.pad_token_id = 50256
        self.padding_side = "right"
        self._reserved = reserved
        self._piece_to_id: Dict[str, int] = {}
        self._id_to_piece: Dict[int, str] = {self.bos_token_id: "<|endoftext|>"}
        for w in known_words:
            self._register(w)

    # -- vocabulary -------------------------------------------------------------
    def _hash_id(self, piece: str) -> int:
        span = self.bos_token_id - self._reserved
        return self._reserved + zlib.crc32(piece.encode("utf-8")) % span

    def _register(self, piece: str) -> int:
        if piece in self._piece_to_id:
            return self._piece_to_id[piece]
        i = self._hash_id(piece)
        span = self.bos_token_id - self._reserved
        while i in self._id_to_piece:
            i = self._reserved + (i - self._reserved + 1) % span
        self._piece_to_id[piece] = i
        self._id_to_piece[i] = piece
        return i

    def token_id(self, piece: str) -> int:
        i = self._piece_to_id.get(piece)
        return self._hash_id(piece) if i is None else i

    # -- HF-like API ------------------------------------------------------------
    def tokenize(self, text: str) -> List[str]:
        return [p for p in _PIECE_RE.findall(text) if p.strip() or p == " "]

    def encode(self, text: str) -> List[int]:
        return [self.token_id(p) for p in self.tokenize(text)]

    def decode(self, ids, clean_up_tokenization_spaces: bool = True) -> str:
        if isinstance(ids, int) or (hasattr(ids, "dim") and ids.dim() == 0):
            ids = [int(ids)]
        return "".join(self._id_to_piece.get(int(i), f"<{int(i)}>") for i in ids)

    def __call__(self, text, **kwargs):
        if isinstance(text, str):
            return {"input_ids": self.encode(text)}
        return {"input_ids": [self.encode(t) for t in text]}

    def __len__(self) -> int:
        return self.vocab_size
