"""Evaluate a trained IOI model pair: resample / mean(zero) ablation sweeps + IIT eval epoch.

Parity: ``/root/reference/eval_ioi.py:1-75`` (flags ``-w -m -c -b``, 18k samples,
seeds, ``models/ioi/{class}/{weights}`` layout, ``results/`` outputs).  The
reference's ``-m`` is ``type=bool`` (any non-empty string is True, Q11); here
``-m`` accepts ``true/false/1/0``.

    python eval_ioi.py -w 100_100_40 -c IOI_ModelPair
"""
from __future__ import annotations

import argparse
import json
import os
import time

import numpy as np
import torch

from iit_amd import model_pairs as mp
from iit_amd.data.iit_dataset import IITDataset, IITUniqueDataset
from iit_amd.models.config import gpt2_config_dict
from iit_amd.models.transformer import HookedTransformer
from iit_amd.tasks.ioi import NAMES, ioi_cfg, make_ioi_corr, make_ioi_dataset_and_hl, suffixes
from iit_amd.utils import checkpoint as ck
from iit_amd.utils import eval_ablations as ea


def _bool(s: str) -> bool:
    return str(s).lower() in ("1", "true", "yes", "y", "t")


def parse(argv=None):
    ap = argparse.ArgumentParser(description="IIT evaluation")
    ap.add_argument("-w", "--weights", type=str, default="100_100_0", help="IIT_behavior_strict weights")
    ap.add_argument("-m", "--mean", type=_bool, default=True, help="Use mean cache")
    ap.add_argument("-c", "--class_name", type=str, default="IOI_ModelPair", help="Model pair class to use")
    ap.add_argument("-b", "--batch_size", type=int, default=512,
                    help="Batch size for making mean cache (if using mean ablation)")
    ap.add_argument("--root", default="models/ioi")
    ap.add_argument("--num-samples", type=int, default=18000)
    ap.add_argument("--model", default="ioi-6l", choices=["ioi-6l", "gpt2-small"])
    ap.add_argument("--resample-batch-size", type=int, default=256)
    ap.add_argument("--backend", default="auto", choices=["auto", "hip", "torch"],
                    help="auto: the fused HIP engine (bf16 compute, fp32 weights) on a GPU, the fp32 torch-op backend "
                         "elsewhere; torch: fp32 reference precision")
    ap.add_argument("--timing-repeats", type=int, default=1,
                    help="run the three sweeps this many times; the timing JSON reports the first (cold: GEMM "
                         "autotuning, graph captures) and the last (warm) run")
    return ap.parse_args(argv)


def main(argv=None):
    args = parse(argv)
    dev = torch.device("cuda") if torch.cuda.is_available() else torch.device("cpu")
    save_dir = os.path.join(args.root, args.class_name, args.weights)
    ll_cfg = gpt2_config_dict()
    if args.model == "ioi-6l":
        ll_cfg.update(ioi_cfg)
    backend = args.backend if args.backend != "auto" else ("hip" if dev.type == "cuda" else "torch")
    ll_cfg.update(device=str(dev), dtype=torch.bfloat16 if backend == "hip" else torch.float32)
    ll_model = HookedTransformer(ll_cfg)
    ll_model.set_op_backend(backend)
    ck.load_ll_model(save_dir, ll_model)
    corr = ck.load_corr(save_dir, suffixes=suffixes, default=make_ioi_corr(ll_cfg["n_layers"]))

    ioi_dataset, hl_model = make_ioi_dataset_and_hl(args.num_samples, ll_model, NAMES, verbose=True, device=dev)
    test_set = IITDataset(ioi_dataset, ioi_dataset, seed=0, device=dev)
    pair_cls = getattr(mp, args.class_name)
    model_pair = pair_cls(ll_model=ll_model, hl_model=hl_model, corr=corr)

    bs = args.resample_batch_size
    uni_test_set = IITUniqueDataset(ioi_dataset, ioi_dataset, seed=0, device=dev)

    def _sync():
        if dev.type == "cuda":
            torch.cuda.synchronize()

    runs = []
    for _ in range(max(1, args.timing_repeats)):
        np.random.seed(0)
        torch.manual_seed(0)
        times = {}
        _sync()
        t0 = time.perf_counter()
        result_not_in_circuit = ea.check_causal_effect(model_pair, test_set, batch_size=bs, node_type="n")
        result_in_circuit = ea.check_causal_effect(model_pair, test_set, batch_size=bs, node_type="c")
        _sync()
        times["resample_ablation_s"] = time.perf_counter() - t0
        t0 = time.perf_counter()
        metric_collection = model_pair._run_eval_epoch(test_set.make_loader(args.batch_size, 0), model_pair.loss_fn)
        _sync()
        times["eval_epoch_s"] = time.perf_counter() - t0
        t0 = time.perf_counter()
        za_not, za_in = ea.get_causal_effects_for_all_nodes(model_pair, uni_test_set, batch_size=args.batch_size,
                                                            use_mean_cache=args.mean)
        _sync()
        times["mean_ablation_s"] = time.perf_counter() - t0
        runs.append(times)
    df = ea.make_combined_dataframe_of_results(result_not_in_circuit, result_in_circuit, za_not, za_in,
                                               use_mean_cache=args.mean)
    out_dir = os.path.join(save_dir, "results")
    ea.save_result(df, out_dir, model_pair)
    with open(os.path.join(out_dir, "metric_collection.log"), "w") as f:
        f.write(str(metric_collection))
    print("Results saved at", out_dir)
    print(metric_collection)
    timing = {k: round(v, 3) for k, v in runs[0].items()}
    if len(runs) > 1:
        timing["warm"] = {k: round(v, 3) for k, v in runs[-1].items()}
    print(json.dumps({"eval_ioi_timing": timing, "backend": backend, "model": args.model,
                      "samples": args.num_samples}))
    return df


if __name__ == "__main__":
    main()
