"""What each IOI HL interchange does to the IIT label (the data side of the IIA ceiling).

For every HL node and every held-out (base, source) pair of the synthetic IOI split used in training (12k samples,
80/20, random_state 42): does the intervened HL label equal the base label, the source label, and are the node's HL
values identical for base and source?  Pure HL computation (``IOI_HL``, /root/reference/iit/tasks/ioi/ioi_hl.py),
CPU is enough.

    python scripts/ioi_hl_label_stats.py
"""
from __future__ import annotations

import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from iit_amd.data.iit_dataset import IITDataset, train_test_split
    from iit_amd.model_pairs import IOI_ModelPair
    from iit_amd.models.config import gpt2_config_dict
    from iit_amd.models.transformer import HookedTransformer
    from iit_amd.tasks.ioi import NAMES, make_ioi_corr, make_ioi_dataset_and_hl

    cfg = gpt2_config_dict()
    cfg.update(n_layers=6, d_model=32, n_heads=4, d_head=8, d_mlp=64, device="cpu")  # LL only supplies the tokenizer
    ll = HookedTransformer(cfg)
    ds, hl = make_ioi_dataset_and_hl(12000, ll, NAMES, device="cpu")
    _, te = train_test_split(ds, test_size=0.2, random_state=42)
    test = IITDataset(te, te, seed=0, device="cpu")
    pair = IOI_ModelPair(hl, ll, make_ioi_corr(6), training_args={"lr_scheduler": None})
    out = {}
    for node in pair.corr.keys():
        c = {"label==base_label": 0, "label==source_label": 0, "base_label==source_label": 0,
             "hl_value_identical": 0}
        n = 0
        for base, abl in test.make_loader(512, 0, shuffle=False):
            with torch.no_grad():
                _, src_cache = hl.run_with_cache(abl, last_only=True)
                _, base_cache = hl.run_with_cache(base, last_only=True)
                pair.hl_cache = src_cache
                y = hl.run_with_hooks(base, fwd_hooks=[(node.name, pair.make_hl_ablation_hook(node))],
                                      last_only=True)
                yb = hl(base, last_only=True)
                ys = hl(abl, last_only=True)
            lab, lb, ls = y.argmax(-1), yb.argmax(-1), ys.argmax(-1)
            c["label==base_label"] += int((lab == lb).sum())
            c["label==source_label"] += int((lab == ls).sum())
            c["base_label==source_label"] += int((lb == ls).sum())
            sv, bv = src_cache[node.name], base_cache[node.name]
            c["hl_value_identical"] += int((sv == bv).reshape(sv.shape[0], -1).all(-1).sum())
            n += lab.shape[0]
        out[node.name] = {k: round(100.0 * v / n, 2) for k, v in c.items()}
        print(node.name, json.dumps(out[node.name]), flush=True)
    print(json.dumps({"ioi_hl_label_stats_pct": out, "held_out_pairs": n}))


if __name__ == "__main__":
    main()
