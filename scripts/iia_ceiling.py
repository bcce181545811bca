"""Where the IOI val/IIA ceiling comes from.

1. **Ties.**  For every held-out (base, source) pair and every HL node, the HL's intervened last-position logits
   (``IOI_HL``, /root/reference/iit/tasks/ioi/ioi_hl.py:54-68) are checked for a tied maximum: with a tie the IIT
   label is the first maximal vocabulary index (torch.argmax), a deterministic but token-order-dependent target.
2. **Per-node IIA.**  The reference's eval epoch samples ONE HL node per batch from the pair's RNG
   (/root/reference/iit/model_pairs/ioi_model_pair.py:71-92), so an epoch's val/IIA is a mix of ~10 node draws.  Every
   ``--every`` epochs this script also evaluates every HL node on the whole validation split, and logs which nodes
   the epoch's own eval drew, so an epoch-to-epoch swing can be attributed to the node mix (data / evaluation) or to
   the model (optimizer).

Training is ``train_ioi.py``'s configuration (BaseModelPair.train: 12k samples, 80/20, batch 256, Adam 1e-4,
iit/behaviour/strict 1/1/0.4, clip 1.0) on the headline GPT-2-small model.  Prints one JSON line at the end.

    python scripts/iia_ceiling.py --epochs 70 --every 5

3. **Control: ``--control zero-wo``.**  ``W_O`` of every block that hosts ``hook_duplicate``'s
   LL sites is zeroed and frozen, so the duplicate splice provably cannot reach the output: the intervened LL output
   IS the base output.  The HL label of a duplicate intervention is the base's IO name for every pair, so a correct
   pipeline (dataset, HL model, site mapping, splice plan, IIA metric) must report ``IIA(hook_duplicate)`` equal to
   the behaviour accuracy on the same pairs -- exactly, element for element.  The script asserts it at every
   evaluation and prints both.
"""
from __future__ import annotations

import argparse
import collections
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def tie_stats(pair, test_set, batch: int = 512):
    """Fraction of held-out pairs whose intervened HL last-position max is tied, per HL node."""
    hl = pair.hl_model
    out = {}
    for node in pair.corr.keys():
        ties = total = 0
        for base, abl in test_set.make_loader(batch, 0, shuffle=False):
            with torch.no_grad():
                _, pair.hl_cache = hl.run_with_cache(abl, **pair.hl_run_kwargs())
                y = hl.run_with_hooks(base, fwd_hooks=[(node.name, pair.make_hl_ablation_hook(node))],
                                      **pair.hl_run_kwargs())
            y = y[:, -1] if y.dim() == 3 else y
            top = y.max(dim=-1, keepdim=True).values
            ties += int(((y == top).sum(dim=-1) > 1).sum())
            total += y.shape[0]
        out[node.name] = ties / max(total, 1)
    return out


def per_node_iia(pair, test_set, batch: int = 512):
    """val/IIA of every HL node over the whole validation split (the pair's own eval draws one node per batch)."""
    res, losses = {}, {}
    pair._ll_module().eval()
    for node in pair.corr.keys():
        hits = n = 0
        loss = 0.0
        for base, abl in test_set.make_loader(batch, 0, shuffle=False):
            with torch.no_grad():
                hl_out, ll_out = pair.do_intervention(base, abl, node)
            hl_last = hl_out[:, -1] if hl_out.dim() == 3 else hl_out
            ll_last = ll_out[:, -1] if ll_out.dim() == 3 else ll_out
            hits += int((ll_last.argmax(-1) == hl_last.argmax(-1)).sum())
            loss += float(torch.nn.functional.cross_entropy(ll_last.float(), hl_last.argmax(-1), reduction="sum"))
            n += hl_last.shape[0]
        res[node.name] = 100.0 * hits / max(n, 1)
        losses[node.name] = loss / max(n, 1)
    return res, losses


def behaviour_accuracy(pair, test_set, node, batch: int = 512):
    """Accuracy of the un-intervened LL on the base inputs against the HL's base label, through the same code path
    as :func:`per_node_iia` (an intervention whose source is the base itself is the identity), plus the per-pair
    agreement with the duplicate-intervened run."""
    hits = n = same = 0
    pair._ll_module().eval()
    for base, abl in test_set.make_loader(batch, 0, shuffle=False):
        with torch.no_grad():
            hl_b, ll_b = pair.do_intervention(base, base, node)
            hl_i, ll_i = pair.do_intervention(base, abl, node)
        last = (lambda t: t[:, -1] if t.dim() == 3 else t)
        pred_b, pred_i = last(ll_b).argmax(-1), last(ll_i).argmax(-1)
        hits += int((pred_b == last(hl_b).argmax(-1)).sum())
        same += int(((pred_b == pred_i) & (last(hl_b).argmax(-1) == last(hl_i).argmax(-1))).sum())
        n += pred_b.shape[0]
    return 100.0 * hits / max(n, 1), 100.0 * same / max(n, 1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="gpt2-small", choices=["gpt2-small", "ioi-6l"])
    ap.add_argument("--epochs", type=int, default=70)
    ap.add_argument("--every", type=int, default=5)
    ap.add_argument("--num-samples", type=int, default=12000)
    ap.add_argument("--lr", type=float, default=1e-4)
    ap.add_argument("--graphs", type=int, default=1, help="0: eager phases (no HIP graphs)")
    ap.add_argument("--backend", default="hip", choices=["hip", "torch", "torch-bf16"],
                    help="torch: the fp32 torch-op oracle backend on the same device; torch-bf16: the torch-op backend "
                         "computing in bf16 (separates bf16 precision from the HIP kernels)")
    ap.add_argument("--train-nodes", default="",
                    help="comma list of HL node names the TRAINING steps sample from (default: all, as the reference)")
    ap.add_argument("--seed", type=int, default=0, help="model-initialisation seed (torch / numpy)")
    ap.add_argument("--plain-adam", action="store_true",
                    help="torch.optim.Adam on the module's own parameters: no flat arena, no bf16 mirror, no fused "
                         "clip norm (separates the fused-optimizer machinery from compute precision)")
    ap.add_argument("--control", default="", choices=["", "zero-wo"],
                    help="zero-wo: zero and freeze W_O of the blocks hosting hook_duplicate (see the docstring)")
    args = ap.parse_args()

    from iit_amd.data.iit_dataset import IITDataset, train_test_split
    from iit_amd.model_pairs import IOI_ModelPair
    from iit_amd.models.config import gpt2_config_dict
    from iit_amd.models.transformer import HookedTransformer
    from iit_amd.tasks.ioi import NAMES, ioi_cfg, make_ioi_corr, make_ioi_dataset_and_hl

    dev = torch.device("cuda") if torch.cuda.is_available() else torch.device("cpu")
    torch.manual_seed(args.seed)
    np.random.seed(args.seed)
    cfg = gpt2_config_dict()
    if args.model == "ioi-6l":
        cfg.update(ioi_cfg)
    fast = dev.type == "cuda" and args.backend == "hip"
    bf16 = fast or (dev.type == "cuda" and args.backend == "torch-bf16")
    cfg.update(init_weights=True, device=str(dev), dtype=torch.bfloat16 if bf16 else torch.float32)
    ll = HookedTransformer(cfg)
    if not fast:
        ll.set_op_backend("torch")
    control_layers = []
    if args.control == "zero-wo":
        from iit_amd.tasks.ioi import make_ioi_corr_dict
        control_layers = sorted({int(s.split(".")[1]) for s in make_ioi_corr_dict(cfg["n_layers"])["hook_duplicate"]})
        with torch.no_grad():
            for l in control_layers:
                ll.blocks[l].attn.W_O.zero_()
                ll.blocks[l].attn.W_O.requires_grad_(False)
        ll.mark_weights_changed()
        print(f"[control] W_O zeroed and frozen in blocks {control_layers}", flush=True)
    ds, hl = make_ioi_dataset_and_hl(args.num_samples, ll, NAMES, device=dev)
    train_ds, test_ds = train_test_split(ds, test_size=0.2, random_state=42)
    train_set = IITDataset(train_ds, train_ds, seed=0, device=dev)
    test_set = IITDataset(test_ds, test_ds, seed=0, device=dev)
    training_args = {"batch_size": 256, "lr": args.lr, "iit_weight": 1.0, "behavior_weight": 1.0, "strict_weight": 0.4,
                     "next_token": False, "lr_scheduler": None, "clip_grad_norm": 1.0, "early_stop": False,
                     "use_single_loss": False, "graphs": bool(args.graphs)}
    if args.plain_adam:
        training_args["fused_optimizer"] = False
    pair = IOI_ModelPair(ll_model=ll, hl_model=hl, corr=make_ioi_corr(cfg["n_layers"]), training_args=training_args)

    if args.train_nodes:  # learnability probe: train on a subset of nodes, still evaluate every node
        keep = [n for n in pair.corr.keys() if n.name in args.train_nodes.split(",")]
        assert keep, args.train_nodes
        pair.sample_hl_name = lambda: keep[int(pair.rng.integers(len(keep)))]

    ties = tie_stats(pair, test_set)
    print("tied HL maxima per node (fraction of held-out pairs):", json.dumps(ties), flush=True)

    # record the HL node each eval batch draws (the reference's one-node-per-batch eval)
    drawn = []
    orig_eval = pair.run_eval_step

    def eval_step(base, abl, loss_fn):
        train_sampler = pair.__dict__.get("sample_hl_name")
        orig_sample = type(pair).sample_hl_name.__get__(pair)

        def sample():
            n = orig_sample()
            drawn.append(n.name)
            return n
        pair.sample_hl_name = sample
        try:
            return orig_eval(base, abl, loss_fn)
        finally:
            if train_sampler is None:
                del pair.sample_hl_name
            else:
                pair.sample_hl_name = train_sampler
    pair.run_eval_step = eval_step
    pair.training_args["eval_graphs"] = False  # the draws must go through the recording sampler

    rows = []
    orig_log = pair._print_and_log_metrics
    t0 = time.perf_counter()
    t_eval = [0.0]   # wall spent in this script's whole-split per-node evaluations (not the reference's epoch loop)
    first95 = {}     # first evaluated epoch where EVERY node's whole-split IIA >= 95 %: epoch, training wall

    def log(epoch, metrics, sink=None):
        vals = {m.get_name(): m.get_value() for m in metrics if m.get_name() != "val/per_token_accuracy"}
        mix = collections.Counter(drawn)
        drawn.clear()
        row = {"epoch": epoch, "val/IIA": round(float(vals["val/IIA"]), 2), "eval_node_draws": dict(mix)}
        if epoch % args.every == 0 or epoch == args.epochs - 1:
            rng_state = pair.rng.bit_generator.state
            te = time.perf_counter()
            iia, ce = per_node_iia(pair, test_set)
            t_eval[0] += time.perf_counter() - te
            if not first95 and min(iia.values()) >= 95.0:
                first95.update(epoch=epoch, train_wall_s=round(te - t0 - (t_eval[0] - (time.perf_counter() - te)), 1))
            row["per_node_IIA"] = {k: round(v, 2) for k, v in iia.items()}
            row["per_node_IIT_loss"] = {k: round(v, 4) for k, v in ce.items()}
            if control_layers:
                dup = next(n for n in pair.corr.keys() if n.name == "hook_duplicate")
                acc, agree = behaviour_accuracy(pair, test_set, dup)
                row["control"] = {"behaviour_acc": round(acc, 2), "dup_IIA": row["per_node_IIA"]["hook_duplicate"],
                                  "pairs_with_identical_prediction_and_label": round(agree, 2),
                                  "W_O_absmax": max(float(ll.blocks[l].attn.W_O.abs().max()) for l in control_layers)}
                assert row["control"]["W_O_absmax"] == 0.0, row
                assert abs(iia["hook_duplicate"] - acc) < 1e-9 and agree == 100.0, row
            pair.rng.bit_generator.state = rng_state  # per-node evaluation draws nothing; keep the RNG anyway
            pair._ll_module().train()
            orig_log(epoch, metrics, sink)
            print(json.dumps(row), flush=True)
        rows.append(row)
    pair._print_and_log_metrics = log
    pair.train(train_set, test_set, epochs=args.epochs)
    wall = time.perf_counter() - t0
    best = max(rows, key=lambda r: r["val/IIA"])
    print(json.dumps({"metric": "IOI val/IIA ceiling analysis", "model": args.model, "epochs": args.epochs,
                      "train_nodes": args.train_nodes or "all", "control": args.control or None, "graphs": args.graphs, "backend": args.backend, "plain_adam": args.plain_adam,
                      "fused_norm": os.environ.get("IIT_FUSED_NORM", "1"), "lr": args.lr,
                      "wall_s": round(wall, 1), "seed": args.seed,
                      "first_eval_all_nodes_IIA_ge_95": first95 or None, "tie_fraction_per_node": ties,
                      "best_epoch_val_IIA": best["val/IIA"], "best_epoch": best["epoch"],
                      "final_per_node_IIA": rows[-1].get("per_node_IIA"), "final_control": rows[-1].get("control")}))


if __name__ == "__main__":
    main()
