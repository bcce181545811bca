"""Where the IOI evaluation sweeps spend device time (GPT-2-small, random-init weights, synthetic IOI prompts).

    IIT_EVAL_GRAPHS=0 python scripts/profile_eval.py > gpurun_out/eval_profile.txt

Prints the node schedule of the resample sweeps (nodes per block, grouped forwards), the warm wall time of each
sweep, then a torch.profiler table (device time per kernel) of one warm resample + mean-ablation pass.  Eager mode
(``IIT_EVAL_GRAPHS=0``) so the profiler sees every kernel; the graphed sweeps replay the same kernels.
"""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main(samples=4608, bs=256):
    from collections import Counter

    from iit_amd.data.iit_dataset import IITDataset, IITUniqueDataset
    from iit_amd.model_pairs import IOI_ModelPair
    from iit_amd.models.config import gpt2_config_dict
    from iit_amd.models.transformer import HookedTransformer
    from iit_amd.tasks.ioi import make_ioi_corr, make_ioi_dataset_and_hl
    from iit_amd.utils import eval_ablations as ea
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    cfg = gpt2_config_dict()
    cfg.update(device="cuda:0", dtype=torch.bfloat16)
    ll = HookedTransformer(cfg)
    ll.set_op_backend("hip")
    ds, hl = make_ioi_dataset_and_hl(samples, ll, device=dev)
    pair = IOI_ModelPair(hl, ll, make_ioi_corr(cfg["n_layers"]), training_args={"batch_size": bs, "lr_scheduler": None})
    test = IITDataset(ds, ds, seed=0, device=dev)
    uni = IITUniqueDataset(ds, ds, seed=0, device=dev)
    for t in ("n", "c"):
        nodes = ea._nodes(pair, t)
        print(f"[eval] sweep {t}: {len(nodes)} nodes, per block {sorted(Counter(ea._node_layer(n.name) for n in nodes).items(), key=lambda kv: (kv[0] is None, kv[0] or 0))}")

    def sweeps():
        ea.check_causal_effect(pair, test, batch_size=bs, node_type="n")
        ea.check_causal_effect(pair, test, batch_size=bs, node_type="c")
        ea.get_causal_effects_for_all_nodes(pair, uni, batch_size=512, use_mean_cache=True)

    for rep in range(2):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for t in ("n", "c"):
            t1 = time.perf_counter()
            ea.check_causal_effect(pair, test, batch_size=bs, node_type=t)
            torch.cuda.synchronize()
            print(f"[eval] rep {rep} resample {t}: {time.perf_counter() - t1:.3f} s")
        t1 = time.perf_counter()
        ea.get_causal_effects_for_all_nodes(pair, uni, batch_size=512, use_mean_cache=True)
        torch.cuda.synchronize()
        print(f"[eval] rep {rep} mean ablation: {time.perf_counter() - t1:.3f} s; total {time.perf_counter() - t0:.3f} s",
              flush=True)
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as prof:
        sweeps()
        torch.cuda.synchronize()
    print(prof.key_averages().table(sort_by="self_cuda_time_total", row_limit=40, max_name_column_width=90))


if __name__ == "__main__":
    main()
