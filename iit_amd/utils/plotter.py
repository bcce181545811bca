"""Probe / ablation heatmaps (parity: ``/root/reference/iit/utils/plotter.py:8-152``).

Writes ``plots/{prefix}_probe_stats.png``, ``plots/{prefix}_leaky_accs_all.png``,
``plots/{prefix}_ablation_stats.png`` and the raw matrices under ``plots/bin/``
(``out_dir`` overrides ``plots``); optional wandb image logging.  Headless
(matplotlib Agg backend).
"""
from __future__ import annotations

import os
from typing import Dict, List

import numpy as np

from ..core.nodes import HLNode

_REDUCTIONS = {"mean": np.mean, "max": np.max, "median": np.median}


def _plt():
    import matplotlib
    matplotlib.use("Agg")
    import matplotlib.pyplot as plt
    return plt


def get_hookpoint_labels(hookpoints: List[str]) -> List[str]:
    return [h.replace("mod.", "").replace(".hook_point", "").replace(".", " ") for h in hookpoints]


def get_leaky_hlnode_labels(hl_nodes) -> List[str]:
    if isinstance(hl_nodes[0], HLNode):
        hl_nodes = [n.name for n in hl_nodes]
    elif not isinstance(hl_nodes[0], str):
        raise ValueError(f"hl_nodes must be a list of str or HLNode, got {type(hl_nodes[0])}")
    return [f"{n.split('_')[1]} -> {n.split('_')[-1]}" for n in hl_nodes]


def _wandb_image(key: str, path: str) -> None:
    try:
        import wandb
        wandb.log({key: wandb.Image(path)})
    except Exception as e:  # optional sink
        print(f"wandb logging skipped: {e}")


def probe_matrices(correctness_stats_per_layer: Dict, leaky_stats_per_layer: Dict, reduction: str = "max"):
    """(correctness_acc [hooks x hl], leaky_acc [hooks x hl] reduced over leak sources, leaky_accs_all)."""
    if reduction not in _REDUCTIONS:
        raise AssertionError(f"reduction must be one of 'mean', 'max', or 'median', got {reduction}")
    red = _REDUCTIONS[reduction]
    hookpoints = list(correctness_stats_per_layer)
    hl_nodes = list(correctness_stats_per_layer[hookpoints[0]]["probes"].keys())
    leaky_nodes = list(leaky_stats_per_layer[hookpoints[0]]["probes"].keys())
    correct = np.array([[correctness_stats_per_layer[h]["test accuracy"][n] for n in hl_nodes] for h in hookpoints])
    leaky = np.zeros((len(hookpoints), len(hl_nodes)))
    leaky_all = np.zeros((len(hookpoints), len(leaky_nodes)))
    pos = {n: i for i, n in enumerate(hl_nodes)}
    for i, h in enumerate(hookpoints):
        accs = np.zeros((len(hl_nodes), len(hl_nodes)))  # rows: leaked from, cols: leaked to
        for j, n in enumerate(leaky_nodes):
            a = leaky_stats_per_layer[h]["test accuracy"][n]
            accs[pos["hook_" + n.split("_")[1]], pos["hook_" + n.split("_")[-1]]] = a
            leaky_all[i, j] = a
        leaky[i] = red(accs, axis=0)
    return correct, leaky, leaky_all, hookpoints, hl_nodes, leaky_nodes


def plot_probe_stats(correctness_stats_per_layer, leaky_stats_per_layer, reduction: str = "max", prefix: str = "",
                     use_wandb: bool = False, out_dir: str = "plots"):
    plt = _plt()
    correct, leaky, leaky_all, hookpoints, hl_nodes, leaky_nodes = probe_matrices(
        correctness_stats_per_layer, leaky_stats_per_layer, reduction)
    os.makedirs(os.path.join(out_dir, "bin"), exist_ok=True)
    np.save(os.path.join(out_dir, "bin", "correctness_acc.npy"), correct)
    np.save(os.path.join(out_dir, "bin", "leaky_acc.npy"), leaky)
    np.save(os.path.join(out_dir, "bin", "leaky_accs_all.npy"), leaky_all)
    labels = get_hookpoint_labels(hookpoints)
    fig, ax = plt.subplots(1, 2, figsize=(20, 10))
    for k, (mat, title) in enumerate(((correct, "Correctness Accuracy"), (leaky, "Leaky Accuracy"))):
        im = ax[k].imshow(mat, cmap="viridis", vmin=0, vmax=1)
        ax[k].set_title(title)
        ax[k].set_xlabel("HL Node")
        ax[k].set_ylabel("Hookpoint")
        ax[k].set_xticks(np.arange(len(hl_nodes)))
        ax[k].set_xticklabels(hl_nodes, rotation=45, ha="right", rotation_mode="anchor")
        ax[k].set_yticks(np.arange(len(hookpoints)))
        ax[k].set_yticklabels(labels)
    fig.colorbar(im, ax=ax.ravel().tolist())
    p1 = os.path.join(out_dir, f"{prefix}_probe_stats.png")
    fig.savefig(p1)
    plt.close(fig)
    fig = plt.figure()
    im = plt.imshow(leaky_all, cmap="viridis")
    plt.colorbar(im)
    plt.xlabel("HL Node")
    plt.ylabel("Hookpoint")
    plt.title("Leaky Accuracy")
    plt.xticks(np.arange(len(leaky_nodes)), get_leaky_hlnode_labels(leaky_nodes), rotation=90)
    plt.yticks(np.arange(len(hookpoints)), labels)
    plt.tight_layout()
    p2 = os.path.join(out_dir, f"{prefix}_leaky_accs_all.png")
    fig.savefig(p2)
    plt.close(fig)
    if use_wandb:
        _wandb_image("probe stats", p1)
        _wandb_image("leaky_accs_all", p2)
    print(f"Plotted probe stats. Find them in {out_dir} folder.")
    return correct, leaky, leaky_all


def plot_ablation_stats(stats_per_layer, prefix: str = "", use_wandb: bool = False, out_dir: str = "plots"):
    plt = _plt()
    hookpoints = list(stats_per_layer)
    hl_nodes = list(stats_per_layer[hookpoints[0]].keys())
    acc = np.zeros((len(hookpoints), len(hl_nodes)))
    for i, h in enumerate(hookpoints):
        for j, n in enumerate(hl_nodes):
            acc[i, j] = stats_per_layer[h][n]
            assert 0 <= acc[i, j] <= 1, f"acc[{i}, {j}] = {acc[i, j]}"
    fig, ax = plt.subplots(1, 1, figsize=(10, 10))
    im = ax.imshow(acc, cmap="viridis", vmin=0, vmax=1)
    ax.set_title("Ablation Accuracy")
    ax.set_xlabel("HL Node")
    ax.set_xticks(np.arange(len(hl_nodes)))
    ax.set_xticklabels(get_leaky_hlnode_labels(hl_nodes), rotation=90)
    ax.set_yticks(np.arange(len(hookpoints)))
    ax.set_yticklabels(get_hookpoint_labels(hookpoints))
    fig.colorbar(im)
    os.makedirs(os.path.join(out_dir, "bin"), exist_ok=True)
    path = os.path.join(out_dir, f"{prefix}_ablation_stats.png")
    fig.savefig(path)
    plt.close(fig)
    if use_wandb:
        _wandb_image("ablation stats", path)
    np.save(os.path.join(out_dir, "bin", f"{prefix}_ablation_acc.npy"), acc)
    print(f"Plotted ablation stats. Find them in {out_dir} folder.")
    return acc
