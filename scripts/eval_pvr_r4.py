"""The PVR evaluation scripts at the reference's configuration on one MI355X, native engine vs the fp32 oracle path.

1. Train the LL ResNet-18 with ``train.py``'s configuration (60k / 10k, lr 1e-3, IITBehaviorModelPair, early stop).
2. ``eval_causality``: input-space leaky resample ablation at every conv hook point (17) x 12 leaky HL nodes, test
   set of ``--test-size``; once with the native plan engine and once with ``engine="reference"`` (hook closures),
   timed; the two heatmap arrays compared entry by entry.
3. ``eval_information``: probes for the correctness and the leaky HL at every conv hook point, native capture vs the
   reference ``run_with_cache`` path, same seeds; accuracy arrays compared.
Prints one summary block (the profiles/eval_pvr_r4.txt record).
"""
import argparse
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--train-size", type=int, default=60000)
    ap.add_argument("--test-size", type=int, default=10000)
    ap.add_argument("--epochs", type=int, default=10)
    ap.add_argument("--probe-train", type=int, default=10000)
    ap.add_argument("--hook-points", nargs="*", default=None)
    ap.add_argument("--engines", nargs="*", default=["native", "reference"],
                    help="native (restructured sweep), native_pernode (one do_intervention per node), reference")
    ap.add_argument("--skip-info", action="store_true", help="skip eval_information")
    ap.add_argument("--skip-causality", action="store_true", help="skip eval_causality")
    ap.add_argument("--info-engines", nargs="*", default=["native", "reference"],
                    help="eval_information engines: native (activation bank), native_nobank, reference")
    args = ap.parse_args()
    from iit_amd.entry import train as train_entry
    from iit_amd.entry.eval_causality import evaluate_model_on_ablations
    from iit_amd.entry.eval_information import evaluate_model_on_probes
    from iit_amd.hooks.wrapper import get_hook_points
    from iit_amd.tasks.task_loader import get_dataset

    t0 = time.perf_counter()
    pair = train_entry.main(["--train-size", str(args.train_size), "--test-size", str(args.test_size),
                             "--epochs", str(args.epochs)])
    torch.cuda.synchronize()
    t_train = time.perf_counter() - t0
    ll = pair.ll_model
    ll.eval()
    hps = args.hook_points or get_hook_points(ll)
    print(f"[pvr] trained in {t_train:.1f} s; {len(hps)} conv hook points", flush=True)

    _, leaky_test = get_dataset("pvr_leaky", dataset_config={"train_size": 1, "test_size": args.test_size})
    res = {}
    for eng in ([] if args.skip_causality else args.engines):
        torch.manual_seed(0)
        # a fresh dataset object per engine: every engine starts from the same patch-draw RNG state
        _, leaky_test = get_dataset("pvr_leaky", dataset_config={"train_size": 1, "test_size": args.test_size})
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ea = {"batch_size": 1024, "engine": "native" if eng.startswith("native") else eng,
              "fast": eng != "native_pernode"}
        res[eng] = evaluate_model_on_ablations(ll, "pvr_leaky", leaky_test.base_data, ea, hook_points=hps)
        torch.cuda.synchronize()
        res[eng + "_s"] = time.perf_counter() - t0
        print(f"[pvr] eval_causality {eng}: {res[eng + '_s']:.2f} s", flush=True)
    first = args.engines[0]
    keys = [(h, k) for h in hps for k in sorted(res[first][h])] if not args.skip_causality else []
    a = np.array([res[first][h][k] for h, k in keys])
    for other in ([] if args.skip_causality else args.engines[1:]):
        b = np.array([res[other][h][k] for h, k in keys])
        print(f"[pvr] eval_causality: {len(keys)} (hook, HL node) cells; max |{first} - {other}| = "
              f"{np.abs(a - b).max():.3g}; {first} range [{a.min():.3f}, {a.max():.3f}]; {first} is "
              f"{res[other + '_s'] / res[first + '_s']:.2f}x faster than {other}", flush=True)
    if args.skip_info:
        return

    tr, te = get_dataset("mnist_pvr", dataset_config={"train_size": args.probe_train, "test_size": args.test_size})
    ltr, lte = get_dataset("pvr_leaky", dataset_config={"train_size": args.probe_train, "test_size": args.test_size})
    probe_res = {}
    # untimed warm-up: one pass of every engine over the deepest hook point (every conv at every batch size the
    # timed passes use), so MIOpen's first-call / find cost for those shapes is paid by none of the timed engines
    for eng in args.info_engines:
        os.environ["IIT_PROBE_BANK"] = "0" if eng == "native_nobank" else "1"
        pargs = {"batch_size": 1024, "lr": 1e-3, "num_workers": 0, "epochs": 1,
                 "engine": "native" if eng.startswith("native") else eng}
        evaluate_model_on_probes(ll, "mnist_pvr", pargs, tr.base_data, te.base_data, hook_points=hps[-1:])
    for eng in args.info_engines:
        # native_nobank: the native engine without the activation bank (one capture per hook point and batch)
        os.environ["IIT_PROBE_BANK"] = "0" if eng == "native_nobank" else "1"
        pargs = {"batch_size": 1024, "lr": 1e-3, "num_workers": 0, "epochs": 1,
                 "engine": "native" if eng.startswith("native") else eng}
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        torch.manual_seed(0)
        c = evaluate_model_on_probes(ll, "mnist_pvr", pargs, tr.base_data, te.base_data, hook_points=hps)
        torch.manual_seed(0)
        lk = evaluate_model_on_probes(ll, "pvr_leaky", pargs, ltr.base_data, lte.base_data, hook_points=hps)
        torch.cuda.synchronize()
        probe_res[eng] = (c, lk, time.perf_counter() - t0)
        print(f"[pvr] eval_information {eng}: {probe_res[eng][2]:.2f} s", flush=True)
    diffs = []
    for i in (0, 1):
        for h in hps:
            for k, v in probe_res["native"][i][h]["test accuracy"].items():
                diffs.append(abs(v - probe_res["reference"][i][h]["test accuracy"][k]))
    accs = [v for h in hps for v in probe_res["native"][0][h]["test accuracy"].values()]
    print(f"[pvr] eval_information: {len(diffs)} probe accuracies; max |native - reference| = {max(diffs):.3g}; "
          f"correctness-probe accuracy range [{min(accs):.3f}, {max(accs):.3f}]; speedup "
          f"{probe_res['reference'][2] / probe_res['native'][2]:.2f}x", flush=True)
    best = max(hps, key=lambda h: np.mean(list(probe_res["native"][0][h]["test accuracy"].values())))
    print(f"[pvr] best correctness-probe hook point: {best}", flush=True)


if __name__ == "__main__":
    main()
