"""Add the evaluation sweeps' GEMM shapes to the shipped decision table (cold ``eval_ioi.py`` runs skip the autotune).

The node-batched sweeps (``iit_amd/utils/eval_ablations.py``) run GEMMs at M = nodes x B rows that the training step
never sees; the dispatcher times every candidate for each such key on first use (8-12 s of a cold sweep).  This script
runs the sweeps once on GPT-2-small and the reference 6L model (random init, synthetic IOI prompts), then writes the
shipped table plus every key decided here that the table does not hold yet (isolated timings; the in-context entries
of the training step stay as they are).

    python scripts/tune_eval_shapes.py --out gpurun_out/table_with_eval.json
"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def sweep(model_name: str, samples: int = 1024):
    from iit_amd.data.iit_dataset import IITDataset, IITUniqueDataset
    from iit_amd.model_pairs import IOI_ModelPair
    from iit_amd.models.config import gpt2_config_dict
    from iit_amd.models.transformer import HookedTransformer
    from iit_amd.tasks.ioi import ioi_cfg, make_ioi_corr, make_ioi_dataset_and_hl
    from iit_amd.utils import eval_ablations as ea
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    cfg = gpt2_config_dict()
    if model_name == "ioi-6l":
        cfg.update(ioi_cfg)
    cfg.update(device="cuda:0", dtype=torch.bfloat16)
    ll = HookedTransformer(cfg)
    ll.set_op_backend("hip")
    ds, hl = make_ioi_dataset_and_hl(samples, ll, device=dev)
    pair = IOI_ModelPair(hl, ll, make_ioi_corr(cfg["n_layers"]), training_args={"batch_size": 256, "lr_scheduler": None})
    test = IITDataset(ds, ds, seed=0, device=dev)
    uni = IITUniqueDataset(ds, ds, seed=0, device=dev)
    for t in ("n", "c"):
        ea.check_causal_effect(pair, test, batch_size=256, node_type=t)
    ea.get_causal_effects_for_all_nodes(pair, uni, batch_size=512, use_mean_cache=True)
    pair._run_eval_epoch(test.make_loader(512, 0), pair.loss_fn)
    torch.cuda.synchronize()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "table_with_eval.json"))
    a = ap.parse_args()
    from iit_amd.ops import gemm_dispatch as gd
    shipped_path = gd._TABLE_PATH
    with open(shipped_path) as f:
        table = json.load(f)
    for m in ("gpt2-small", "ioi-6l"):
        sweep(m)
        print(f"[tune-eval] {m}: {len(gd.DECISIONS)} single / {len(gd.DUAL_DECISIONS)} dual keys decided so far",
              flush=True)
    added = 0
    for key, (choice, times) in {**gd.DECISIONS, **gd.DUAL_DECISIONS}.items():
        k = repr(key)
        if k not in table["decisions"] and choice is not None:
            table["decisions"][k] = choice
            added += 1
    table["method"] = table.get("method", "") + "; eval-sweep shapes: isolated autotune (scripts/tune_eval_shapes.py)"
    with open(a.out, "w") as f:
        json.dump(table, f, indent=0, sort_keys=True)
    print(f"[tune-eval] added {added} keys -> {a.out} ({len(table['decisions'])} total)")


if __name__ == "__main__":
    main()
