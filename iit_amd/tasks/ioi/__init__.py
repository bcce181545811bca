"""IOI task wiring (parity: ``/root/reference/iit/tasks/ioi/__init__.py:8-37`` and ``utils.py:4-29``).

``corr_dict`` / ``corr`` / ``suffixes`` / ``ioi_cfg`` match the reference exactly for
the 6-layer LL model.  ``make_ioi_corr_dict(n_layers)`` generalises the mapping
to deeper LL models (e.g. the 12-layer GPT-2-small config of ``BASELINE.json``)
by stretching each reference layer over ``n_layers/6`` consecutive layers.
"""
from __future__ import annotations

from typing import Dict, List

import torch

from ...config import DEVICE
from ...core.correspondence import Correspondence
from ...core.nodes import HLNode, LLNode
from .ioi_config import NAMES, NOUNS, TEMPLATES
from .ioi_dataset import IOIDataset, IOIDatasetWrapper, default_tokenizer
from .ioi_hl import IOI_HL, DuplicateHead, InductionHead, NameMoverHead, PreviousHead, SInhibitionHead
from .tokenizer import SyntheticTokenizer

n_layers = 6
n_heads = 4
d_model = 64
d_head = d_model // n_heads
ioi_cfg = {"n_layers": n_layers, "n_heads": n_heads, "d_model": d_model, "d_head": d_head}

suffixes = {"attn": "attn.hook_z", "mlp": "mlp.hook_post"}


def _attn(i):
    return f"blocks.{i}.attn.hook_z"


def _mlp(i):
    return f"blocks.{i}.mlp.hook_post"


def make_ioi_corr_dict(num_layers: int = 6, attn_only: bool = False) -> Dict[str, List[str]]:
    """Reference mapping for 6 layers; deeper models stretch each reference layer over
    ``num_layers/6`` layers, shallower ones map reference layer ``l`` to ``l*num_layers//6``.
    Attention-only models map the input-token node to ``hook_embed``."""
    if num_layers % 6 == 0:
        r = num_layers // 6

        def span(ref_layers):
            return [l * r + j for l in ref_layers for j in range(r)]
    else:
        def span(ref_layers):
            return sorted({l * num_layers // 6 for l in ref_layers})

    return {
        "hook_duplicate": [_attn(i) for i in span([0])],
        "hook_s_inhibition": [_attn(i) for i in span([2, 3])],
        "hook_name_mover": [_attn(i) for i in span([4, 5])],
        "all_nodes_hook": ["hook_embed"] if attn_only else [_mlp(i) for i in span([0, 1])],
    }


all_attns = [_attn(i) for i in range(n_layers)]
all_mlps = [_mlp(i) for i in range(n_layers)]
corr_dict = make_ioi_corr_dict(n_layers)
corr = Correspondence.make_corr_from_dict(corr_dict, suffixes=suffixes, make_suffixes_from_corr=False)


def make_ioi_corr(num_layers: int = 6, attn_only: bool = False) -> Correspondence:
    return Correspondence.make_corr_from_dict(make_ioi_corr_dict(num_layers, attn_only), suffixes=suffixes)


def make_ioi_dataset_and_hl(num_samples: int, ll_model, NAMES=NAMES, verbose: bool = False, device=None,
                            label_format: str = "index", seed: int = 42):
    """Build the IOI dataset wrapper and the HL model whose name set is every IO token seen."""
    device = device if device is not None else DEVICE
    tokenizer = getattr(ll_model, "tokenizer", None)
    if tokenizer is None:
        tokenizer = default_tokenizer()
        if ll_model is not None:
            ll_model.tokenizer = tokenizer
    ds = IOIDatasetWrapper(tokenizer=tokenizer, names=NAMES, num_samples=num_samples, device=device,
                           label_format=label_format, seed=seed)
    names = torch.unique(ds.io_ids).to(device)
    d_vocab = ll_model.cfg.d_vocab_out if ll_model is not None else tokenizer.vocab_size
    hl_model = IOI_HL(d_vocab=d_vocab, names=names).to(device)
    if verbose:
        p = ds.prompts[0]
        print(p.tolist(), [tokenizer.decode(int(i)) for i in p])
    return ds, hl_model
