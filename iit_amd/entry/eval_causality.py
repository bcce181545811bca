"""PVR leakiness by input-space resample ablation, per conv hook point (parity: ``/root/reference/eval_causality.py``).

For every conv hook point of the LL ResNet and every leaky HL node
``hook_{i}_leaked_to_{j}``: patch quadrant ``i`` of the input with a digit of a
different class, intervene at quadrant ``j``'s slice of the hook, and measure how
often the LL still predicts the HL output on label-changing samples.  The
reference script is broken (4-argument ``patch_batch_at_hl`` call);
this implements its evident semantics.  Writes ``plots/{time}_ablation_stats.png``.

    python eval_causality.py --weights weights/ll_model/mnist_pvr.pt
"""
from __future__ import annotations

import argparse
from datetime import datetime

import torch

from iit_amd.config import DEVICE
from iit_amd.hooks.wrapper import get_hook_points
from iit_amd.model_pairs import IITProbeSequentialPair
from iit_amd.tasks.task_loader import get_alignment, get_dataset
from iit_amd.utils.plotter import plot_ablation_stats
from iit_amd.utils.progress import progress


def evaluate_model_on_ablations(ll_model, task: str, test_set, eval_args: dict, verbose: bool = False,
                                hook_points=None):
    stats_per_layer = {}
    for hook_point in progress(hook_points or get_hook_points(ll_model), desc="Hook points"):
        _, hl_model, corr = get_alignment(task, config={"hook_point": hook_point,
                                                        "input_shape": test_set.get_input_shape()})
        pair = IITProbeSequentialPair(ll_model=ll_model, hl_model=hl_model, corr=corr,
                                      training_args={"engine": eval_args.get("engine", "native")})
        stats = {hl_node: torch.zeros((), device=DEVICE) for hl_node in pair.corr}
        n = len(test_set)
        bs = eval_args["batch_size"]
        nb = 0
        with torch.no_grad():
            for s in range(0, n, bs):
                nb += 1
                base_input = test_set.gather(torch.arange(s, min(n, s + bs), device=DEVICE))
                for hl_node in pair.corr:
                    # same draws, one device pass per batch (the reference engine keeps the reference's per-sample loop)
                    if hasattr(test_set, "patch_batch_tensor") and eval_args.get("engine", "native") != "reference":
                        ablated = test_set.patch_batch_tensor(base_input[0], base_input[2], hl_node)
                    else:
                        xs, ys, ivs = test_set.patch_batch_at_hl(list(base_input[0]), list(base_input[2]), hl_node)
                        ablated = (torch.stack(xs), torch.stack([torch.as_tensor(y) for y in ys]).to(DEVICE),
                                   torch.stack(ivs))
                    hl_output, ll_output = pair.do_intervention(base_input, ablated, hl_node)
                    changed = (ablated[1] != base_input[1]).float()
                    acc = (torch.argmax(ll_output, dim=1) == hl_output).float() * changed
                    stats[hl_node] += acc.sum() / (changed.sum() + 1e-10)
        out = {k.name: float(v) / max(nb, 1) for k, v in stats.items()}
        for k, v in out.items():
            assert 0 <= v <= 1, f"{k}: {v}"
        stats_per_layer[hook_point] = out
        if verbose:
            print(hook_point, out)
    return stats_per_layer


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--weights", default=None, help="LL state_dict (train.py --save); random init if omitted")
    ap.add_argument("--test-size", type=int, default=10000)
    ap.add_argument("--batch-size", type=int, default=1024)
    ap.add_argument("--hook-points", nargs="*", default=None)
    ap.add_argument("--out-dir", default="plots")
    ap.add_argument("--wandb", action="store_true")
    args = ap.parse_args(argv)
    _, leaky_test = get_dataset("pvr_leaky", dataset_config={"train_size": 1, "test_size": args.test_size})
    ll_model, _, _ = get_alignment("mnist_pvr", config={"input_shape": leaky_test.base_data.get_input_shape()})
    if args.weights:
        ll_model.load_state_dict(torch.load(args.weights, map_location=DEVICE, weights_only=True))
    ll_model.eval()
    stats = evaluate_model_on_ablations(ll_model, "pvr_leaky", leaky_test.base_data,
                                        {"batch_size": args.batch_size, "num_workers": 0},
                                        hook_points=args.hook_points)
    prefix = datetime.now().strftime("%d_%m_%Y_%H_%M_%S")
    plot_ablation_stats(stats, prefix=prefix, use_wandb=args.wandb, out_dir=args.out_dir)
    return stats


if __name__ == "__main__":
    main()
