"""Time the PVR leakiness sweep variants on a random-init ResNet-18 (timing does not depend on the weights):
the per-node path and the restructured sweep at several node-chunk sizes, a few hook points each.

    python scripts/time_eval_causality.py [--test-size 10000] [--hooks N]
"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--test-size", type=int, default=10000)
    ap.add_argument("--hooks", type=int, default=4)
    ap.add_argument("--chunks", nargs="*", type=int, default=[1, 2, 4, 12])
    args = ap.parse_args()
    from iit_amd.entry.eval_causality import evaluate_model_on_ablations
    from iit_amd.hooks.wrapper import get_hook_points
    from iit_amd.tasks.task_loader import get_alignment, get_dataset
    torch.manual_seed(0)
    _, leaky = get_dataset("pvr_leaky", dataset_config={"train_size": 1, "test_size": args.test_size})
    ll, _, _ = get_alignment("mnist_pvr", config={"input_shape": leaky.base_data.get_input_shape()})
    ll.eval()
    hps = get_hook_points(ll)
    hps = [hps[i] for i in sorted({int(j * (len(hps) - 1) / max(args.hooks - 1, 1)) for j in range(args.hooks)})]
    print("hook points:", hps, flush=True)
    variants = [("pernode", {"fast": False})] + [(f"chunk{c}", {"node_chunk": c}) for c in args.chunks]
    for rep in range(2):  # second round: MIOpen solutions / allocator warm
        for name, ea in variants:
            _, leaky = get_dataset("pvr_leaky", dataset_config={"train_size": 1, "test_size": args.test_size})
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            evaluate_model_on_ablations(ll, "pvr_leaky", leaky.base_data, {"batch_size": 1024, **ea}, hook_points=hps)
            torch.cuda.synchronize()
            print(f"[time] round {rep} {name}: {time.perf_counter() - t0:.2f} s", flush=True)


if __name__ == "__main__":
    main()
