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


def _resnet_site(hook_point: str):
    """``mod.conv1.hook_point`` -> (0, 0, "stem"); ``mod.layer{L}.mod.{i}.mod.conv{c}.hook_point`` -> (L, i, "conv{c}");
    None for any other hook."""
    parts = hook_point.split(".")
    if parts == ["mod", "conv1", "hook_point"]:
        return 0, 0, "stem"
    if len(parts) == 7 and parts[0] == "mod" and parts[1].startswith("layer") and parts[4] == "mod" \
            and parts[5] in ("conv1", "conv2") and parts[6] == "hook_point":
        return int(parts[1][5:]), int(parts[3]), parts[5]
    return None


def _block_input_name(L: int, i: int) -> str:
    if i > 0:
        return f"mod.layer{L}.mod.{i - 1}.hook_point"
    return "mod.maxpool.hook_point" if L == 1 else f"mod.layer{L - 1}.hook_point"


def _resnet_suffix(res, L: int, i: int, which: str, act: torch.Tensor, identity) -> torch.Tensor:
    """The rest of the ResNet forward from the output of conv hook (L, i, which) -- ``act`` is that conv's output
    (spliced), ``identity`` the block's shortcut (``downsample(block input)`` or the block input) -- to the logits."""
    if which == "stem":
        x = res.maxpool(res.relu(res.bn1(act)))
        L, i = 1, 0
    else:
        bb = getattr(res, f"layer{L}").mod[i].mod
        out = bb.bn2(bb.conv2(bb.relu(bb.bn1(act)))) if which == "conv1" else bb.bn2(act)
        x = bb.relu(out + identity)
        i += 1
    for layer in range(L, 5):
        blocks = getattr(res, f"layer{layer}").mod
        for k in range(i if layer == L else 0, len(blocks)):
            x = blocks[k](x)
    return res.fc(torch.flatten(res.avgpool(x), 1))


def _fast_resample_sweep(ll_model, test_set, hook_points, bs: int, node_chunk: int = 1):
    """The leakiness sweep of :func:`evaluate_model_on_ablations` for the PVR ResNet, restructured for the device
    (the IOI sweeps' machinery, ``iit_amd.utils.eval_ablations``):

    * **node batching** (``node_chunk`` nodes per launch sequence, default 1): stacking the twelve patched source
      batches into one [12 B] batch measured slower on MI355X -- every new convolution batch size pays MIOpen's
      first-encounter cost (124 s vs 7.4 s for four hook points) and the warm difference is within 12 %
      (profiles/eval_causality_r5.txt) -- so the convolutions keep the reference's batch;
    * **truncated source runs**: the source forward stops at the hook point (``run_capture``);
    * **shared base prefix**: the base batch runs ONCE per (hook point, batch), up to the hook point, capturing the
      hook's activation and the enclosing block's shortcut input; each node's spliced run then starts AT the hook
      (:func:`_resnet_suffix`) from the base activation with the node's quadrant replaced by the source's -- the
      reference re-runs the whole base forward per node;
    * the HL output of ``hook_{i}_leaked_to_{j}`` is the patched batch's label (the HL intervention replaces
      quadrant i's class by the source's, which is exactly what the patch changed; asserted against the HL model
      in tests/test_eval_causality_fast.py).

    The patch draws are the reference loop's, in its order (hook point, batch, node): ``draw_patch_digits``
    consumes ``test_set.rng`` exactly as ``patch_batch_at_hl`` does; the loop never synchronises (the draws' host
    inputs are read once up front), so the host draws of one (hook, batch) overlap the GPU work of the previous.  Cells equal the per-node path up to fp32 batch-size effects in the convolutions."""
    from iit_amd.tasks.mnist_pvr.pvr_check_leaky_hl import corr_for_shape
    res = ll_model.mod
    n = len(test_set)
    dev = next(ll_model.parameters()).device
    batches = [test_set.gather(torch.arange(s, min(n, s + bs), device=dev)) for s in range(0, n, bs)]
    curs = [iv.cpu().numpy() for _, _, iv in batches]  # the draws' host inputs, read once: the loop never syncs
    # every hook's output shape from one capture at the sweep's own batch size (no extra convolution shapes)
    shapes = {h: t.shape for h, t in ll_model.run_capture(batches[0][0], list(hook_points)).items()}
    out = {}
    with torch.no_grad():
        for hp in hook_points:
            L, i, which = _resnet_site(hp)
            corr = corr_for_shape(hp, shapes[hp])
            nodes = list(corr.keys())
            lidx = [next(iter(corr[nd])).index for nd in nodes]
            shortcut = None if which == "stem" else _block_input_name(L, i)
            acc = torch.zeros(len(nodes), dtype=torch.float64, device=dev)
            for (x, y, iv), cur in zip(batches, curs):
                B = x.shape[0]
                srcs, ys = [], []
                for nd in nodes:
                    _, k = test_set.get_idx_and_intermediate(nd)
                    js = test_set.draw_patch_digits(cur[:, k])
                    xs, yk, _ = test_set.apply_patch_digits(x, iv, nd, js)
                    srcs.append(xs)
                    ys.append(yk)
                names = [hp] if shortcut is None else [hp, shortcut]
                base = ll_model.run_capture(x, names)
                ident = None
                if shortcut is not None:
                    bb = getattr(res, f"layer{L}").mod[i].mod
                    ident = base[shortcut] if bb.downsample is None else bb.downsample(base[shortcut])
                preds = []
                for c0 in range(0, len(nodes), node_chunk):  # node_chunk nodes per launch sequence
                    cn = min(node_chunk, len(nodes) - c0)
                    a_src = ll_model.run_capture(torch.cat(srcs[c0:c0 + cn]), [hp])[hp]
                    a = base[hp].repeat(cn, *([1] * (base[hp].dim() - 1)))
                    for t in range(cn):
                        sl = (slice(t * B, (t + 1) * B),) + tuple(lidx[c0 + t].as_index)[1:]
                        a[sl] = a_src[sl]
                    idc = None if ident is None else ident.repeat(cn, *([1] * (ident.dim() - 1)))
                    preds.append(_resnet_suffix(res, L, i, which, a, idc).argmax(dim=1).view(cn, B))
                pred = torch.cat(preds)
                hl = torch.stack(ys)
                changed = (hl != y.unsqueeze(0)).float()
                hit = (pred == hl).float() * changed
                acc += (hit.sum(1) / (changed.sum(1) + 1e-10)).double()
            vals = (acc / max(len(batches), 1)).tolist()
            out[hp] = {nd.name: float(v) for nd, v in zip(nodes, vals)}
            for k, v in out[hp].items():
                assert 0 <= v <= 1, f"{k}: {v}"
    return out


def evaluate_model_on_ablations(ll_model, task: str, test_set, eval_args: dict, verbose: bool = False,
                                hook_points=None):
    hps = hook_points or get_hook_points(ll_model)
    if (eval_args.get("engine", "native") == "native" and eval_args.get("fast", True) and task == "pvr_leaky"
            and hasattr(test_set, "draw_patch_digits") and hasattr(getattr(ll_model, "mod", None), "layer4")
            and not ll_model.training and all(_resnet_site(h) is not None for h in hps)):
        stats = _fast_resample_sweep(ll_model, test_set, hps, eval_args["batch_size"],
                                     node_chunk=int(eval_args.get("node_chunk", 1)))
        if verbose:
            for h, v in stats.items():
                print(h, v)
        return stats
    stats_per_layer = {}
    for hook_point in progress(hps, desc="Hook points"):
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
