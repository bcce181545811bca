"""PVR probe correctness / leakiness per conv hook point (parity: ``/root/reference/eval_information.py``).

Trains an ``IITProbeSequentialPair`` (IIT + behaviour + linear probes), then for
every conv hook point trains fresh probes for the correctness HL (quadrant digit
at its own location) and the leaky HL (digit ``i`` at quadrant ``j``'s location)
and plots the accuracy heatmaps (``plots/{time}_probe_stats.png``,
``plots/{time}_leaky_accs_all.png``).  Probes can be saved as
``weights/probes/{task}/{hook_point}/{hl_node}.pt`` state_dicts.

    python eval_information.py --train-size 4096 --test-size 1024 --epochs 1
"""
from __future__ import annotations

import argparse
import os
import time
from datetime import datetime

import torch
from torch import nn

from iit_amd.hooks.wrapper import get_hook_points
from iit_amd.model_pairs import IITProbeSequentialPair
from iit_amd.tasks.task_loader import get_alignment, get_dataset
from iit_amd.utils.plotter import plot_probe_stats
from iit_amd.utils.probes import ActivationBank, evaluate_probe, train_probes_on_model_pair
from iit_amd.utils.progress import progress


def evaluate_model_on_probes(ll_model, task: str, probe_training_args: dict, train_set, test_set,
                             use_wandb: bool = False, verbose: bool = False, save_probes: bool = False,
                             hook_points=None):
    stats = {}
    hps = hook_points or get_hook_points(ll_model)
    banks = (None, None)
    timing = os.environ.get("IIT_PROBE_TIMING") == "1"
    clock = {"bank": 0.0, "train": 0.0, "eval": 0.0}

    def tick(key, t0):
        if timing:
            if torch.cuda.is_available():
                torch.cuda.synchronize()
            clock[key] += time.perf_counter() - t0
        return time.perf_counter()

    t0 = time.perf_counter()
    if (probe_training_args.get("engine", "native") == "native" and getattr(ll_model, "supports_run_plan", False)
            and hasattr(train_set, "gather") and hasattr(test_set, "gather")
            and os.environ.get("IIT_PROBE_BANK", "1") != "0"
            and ActivationBank.fits(ll_model, (train_set, test_set), hps)):
        # every hook point's activations of every train / test sample, captured once (ActivationBank): the
        # per-hook-point loop below then trains and evaluates its probes from gathers instead of forwards
        banks = (ActivationBank(ll_model, train_set, hps, probe_training_args["batch_size"]),
                 ActivationBank(ll_model, test_set, hps, 256))
    t0 = tick("bank", t0)
    for hook_point in progress(hps, desc="Hook points"):
        _, hl_model, corr = get_alignment(task, config={"hook_point": hook_point,
                                                        "input_shape": test_set.get_input_shape()})
        pair = IITProbeSequentialPair(ll_model=ll_model, hl_model=hl_model, corr=corr,
                                      training_args=probe_training_args)  # ("engine": "reference" = hook path)
        t0 = time.perf_counter()
        out = train_probes_on_model_pair(pair, train_set.get_input_shape(), train_set, probe_training_args,
                                         bank=banks[0])
        t0 = tick("train", t0)
        if save_probes:
            d = os.path.join("weights", "probes", task, hook_point)
            os.makedirs(d, exist_ok=True)
            for k, v in out["probes"].items():
                torch.save(v.state_dict(), os.path.join(d, f"{k}.pt"))
        out.update(evaluate_probe(out["probes"], pair, test_set, nn.CrossEntropyLoss(), bank=banks[1]))
        tick("eval", t0)
        if verbose:
            print(hook_point, out["test accuracy"])
        stats[hook_point] = out
    if timing:
        print(f"[probe timing] {task} engine={probe_training_args.get('engine', 'native')} bank={banks[0] is not None}: "
              + ", ".join(f"{k} {v:.2f} s" for k, v in clock.items()), flush=True)
    return stats


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--train-size", type=int, default=60000)
    ap.add_argument("--test-size", type=int, default=10000)
    ap.add_argument("--epochs", type=int, default=1)
    ap.add_argument("--batch-size", type=int, default=512)
    ap.add_argument("--probe-batch-size", type=int, default=1024)
    ap.add_argument("--probe-epochs", type=int, default=1)
    ap.add_argument("--reduction", default="max", choices=["max", "mean", "median"])
    ap.add_argument("--hook-points", nargs="*", default=None)
    ap.add_argument("--out-dir", default="plots")
    ap.add_argument("--save-weights", action="store_true")
    args = ap.parse_args(argv)
    cfg = {"train_size": args.train_size, "test_size": args.test_size}
    train_set, test_set = get_dataset("mnist_pvr", dataset_config=cfg)
    ll_model, hl_model, corr = get_alignment("mnist_pvr", config={"input_shape": test_set.base_data.get_input_shape()})
    training_args = {"batch_size": args.batch_size, "lr": 1e-3, "num_workers": 0, "epochs": args.epochs}
    pair = IITProbeSequentialPair(ll_model=ll_model, hl_model=hl_model, corr=corr, training_args=training_args)
    pair.train(train_set, test_set, epochs=args.epochs)
    ll_model.eval()
    if args.save_weights:
        os.makedirs(os.path.join("weights", "ll_model"), exist_ok=True)
        torch.save({k: v.detach().clone() for k, v in ll_model.state_dict().items()},
                   os.path.join("weights", "ll_model", "mnist_pvr.pt"))
    probe_args = {"batch_size": args.probe_batch_size, "lr": 1e-3, "num_workers": 0, "epochs": args.probe_epochs}
    leaky_train, leaky_test = get_dataset("pvr_leaky", dataset_config=cfg)
    correct = evaluate_model_on_probes(ll_model, "mnist_pvr", probe_args, train_set.base_data, test_set.base_data,
                                       save_probes=args.save_weights, hook_points=args.hook_points)
    leaky = evaluate_model_on_probes(ll_model, "pvr_leaky", probe_args, leaky_train.base_data, leaky_test.base_data,
                                     save_probes=args.save_weights, hook_points=args.hook_points)
    prefix = datetime.now().strftime("%d_%m_%Y_%H_%M_%S")
    return plot_probe_stats(correct, leaky, reduction=args.reduction, prefix=prefix, out_dir=args.out_dir)


if __name__ == "__main__":
    main()
