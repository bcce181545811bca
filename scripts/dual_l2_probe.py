"""The headline step's dual dX + dW launches (csrc/gemm_dual.hip) in context vs in isolation, and what the preceding
kernel's cache state does to them ("first test the untested hypothesis" -- that the 10-25 %
in-context penalty of the pairs is the dirty-L2 writeback of the ~19 MB the previous kernel wrote).

The real step's operands are recorded (one eager training step, ``gemm_pair`` wrapped), then every M = 4096 pair on
its shipped dual configuration is timed on scratch outputs:

* ``in-step``: HIP events around the pair inside eager training steps issued behind a device sleep (the GPU then
  runs the step back to back, as a graph replay does; ``scripts/tune_gemm_in_situ.py``'s method), median of rounds;
* ``hot``: back-to-back launches (graph of 10), operands L2-hot -- the autotuner's view;
* ``<prefix>``: graph of 10 x [prefix, pair] minus graph of 10 x [prefix], prefixes:
  - ``dirty_dy``: rewrite the pair's dY operand (what the producing kernel does in the step: dY dirty in L2),
  - ``dirty_19mb``: write 19 MB to an unrelated buffer (dirty L2 lines that must be written back, operands hot),
  - ``dirty_dy_wb``: rewrite dY, then stream 64 MB of unrelated reads (dY written back, still in the 256 MB MALL),
  - ``evict``: stream 512 MB of reads (clean L2 and MALL, every operand cold),
  - ``dirty_19mb_evict``: both;
  - ``evict_read``: evict, then read the pair's cold operands (X, W) once (a reduction over each): the lines the
    pair needs are back in the caches -- what a perfect prefetch would achieve.

``--pmc`` runs the same conditions eagerly (``--reps`` each) after 3 eager steps, for rocprofv3 --pmc
(``scripts/gpu_r6_dual.sh``), and writes the dispatch sequence to ``--seq``; ``--summarize <counter csv>`` then maps
the trailing dual dispatches to (condition, pair) and the last step's to (in-step, pair).
"""
import argparse
import collections
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

CONDS = ("hot", "dirty_dy", "dirty_19mb", "dirty_dy_wb", "evict", "dirty_19mb_evict", "evict_read")


def label(key):
    _, xm, xn, xk, xepi, _, wm, wn, wk, wepi, fresh, _ = key
    site = {(3072, 768): "W_out", (768, 3072): "W_in", (768, 2304): "W_QKV", (768, 768): "W_O"}.get((xn, xk), "?")
    return f"{site} {'acc' if wepi == 7 else 'store'}"


def record_pairs(pair, loss_fn, opt, it, gd, K):
    """One eager training step with gemm_pair wrapped: {key: (x, w)} for every M = 4096 pair that launches a dual."""
    seen = collections.OrderedDict()
    order = []
    orig = gd.gemm_pair

    def wrap(x, w, prefetch=None):
        res = orig(x, w, prefetch=prefetch)
        if gd._dual_eligible(x, w):
            fresh = bool(w.get("fresh")) and w["epi"] == K.EPI_F32_STORE
            key = ("dual", x["M"], x["N"], x["K"], x["epi"], x.get("colsum") is not None,
                   w["M"], w["N"], w["K"], w["epi"], fresh, gd.deterministic())
            ch = gd.DUAL_DECISIONS.get(key)
            if ch is not None and gd._parse_dual(ch[0]) is not None:
                order.append(key)
                if x["M"] == 4096 and key not in seen:
                    seen[key] = (dict(x), dict(w))
        return res

    from iit_amd.ops import hip_ops  # the callers' binding (``from .gemm_dispatch import gemm_pair``)
    hip_ops.gemm_pair = wrap
    try:
        base, abl = next(it)
        pair.run_train_step(base, abl, loss_fn, opt)
        torch.cuda.synchronize()
    finally:
        hip_ops.gemm_pair = orig
    return seen, order


def specs(gd, x, w):
    """The pair's dual specs on scratch outputs (the dispatcher's timing setup)."""
    xc = gd._scratch(x["C"], x["M"], max(x["ldc"], x["N"]))
    wc = gd._scratch(w["C"], w["M"], max(w["ldc"], w["N"]))
    cs = torch.zeros_like(x["colsum"]) if x.get("colsum") is not None else None
    bs = torch.zeros_like(w["bsum"]) if w.get("bsum") is not None else None
    sq = torch.zeros_like(w["gsq"]) if w.get("gsq") is not None else None
    ws, xs = gd._dual_specs(x, w, xc, wc, cs, bs, sq)
    return ws, xs


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=8)
    ap.add_argument("--pmc", action="store_true")
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--seq", default=os.path.join(ROOT, "gpurun_out", "dual_l2_seq.json"))
    ap.add_argument("--summarize", default=None)
    a = ap.parse_args()
    if a.summarize:
        return summarize(a.summarize, a.seq)

    import bench
    from iit_amd.ops import gemm_dispatch as gd
    from iit_amd.ops import hip_kernels as K

    args = argparse.Namespace(gpus=1, steps=1, warmup=1, batch=256, model="gpt2-small", engine="native", dtype="bf16",
                              graphs=0, profile_dir=None)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    pair, opt, loss_fn, it, step_fn, _, _ = bench.setup(args, dev)
    for _ in range(3):
        base, abl = next(it)
        pair.run_train_step(base, abl, loss_fn, opt)
    torch.cuda.synchronize()
    pairs, order = record_pairs(pair, loss_fn, opt, it, gd, K)
    keys = list(pairs)
    cfgs = {k: gd._parse_dual(gd.DUAL_DECISIONS[k][0]) for k in keys}
    print(f"{len(keys)} M=4096 dual pairs: " + ", ".join(f"{label(k)} -> {gd.DUAL_DECISIONS[k][0]}" for k in keys),
          flush=True)

    # prefixes
    big = torch.empty(512 * 2 ** 20 // 4, dtype=torch.float32, device=dev).uniform_()
    mid = big[: 64 * 2 ** 20 // 4]
    sink = torch.empty(19 * 2 ** 20 // 4, dtype=torch.float32, device=dev)
    out1 = torch.empty(1, dtype=torch.float32, device=dev)
    dys = {k: (pairs[k][0]["A"], pairs[k][0]["A"].clone()) for k in keys}  # dX = dY W^T: A is dY

    def prefix(cond, k):
        dy, src = dys[k]
        if cond in ("dirty_dy", "dirty_dy_wb"):
            dy.copy_(src)
        if cond in ("dirty_19mb", "dirty_19mb_evict"):
            sink.fill_(1.0)
        if cond == "dirty_dy_wb":
            torch.sum(mid, dim=0, keepdim=True, out=out1)
        if cond in ("evict", "dirty_19mb_evict", "evict_read"):
            torch.sum(big, dim=0, keepdim=True, out=out1)
        if cond == "evict_read":
            x, w = pairs[k]
            for t in (w["A"], x["B"]):  # dW = X^T dY: A = X; dX = dY W^T: B = W
                torch.sum(t)  # one read of every line

    launch = {}
    for k in keys:
        ws, xs = specs(gd, *pairs[k])
        launch[k] = (lambda ws=ws, xs=xs, c=cfgs[k]: K.gemm_dual(ws, xs, *c))

    if a.pmc:
        seq = {"step": [label(k) for k in order if k[1] == 4096], "probe": []}
        for cond in CONDS:
            for k in keys:
                for _ in range(a.reps):
                    if cond != "hot":
                        prefix(cond, k)
                    launch[k]()
                    seq["probe"].append([cond, label(k)])
        torch.cuda.synchronize()
        with open(a.seq, "w") as f:
            json.dump(seq, f)
        print(f"pmc probe: {len(seq['probe'])} dual dispatches after the step's {len(seq['step'])}", flush=True)
        return

    # in-step: events around each pair inside eager steps issued behind a device sleep
    samples = collections.defaultdict(list)
    for r in range(a.rounds):
        gd.TIMING = []
        base, abl = next(it)
        torch.cuda.synchronize()
        torch.cuda._sleep(int(1.5e9))
        pair.run_train_step(base, abl, loss_fn, opt)
        torch.cuda.synchronize()
        for key, name, s_ev, e_ev in gd.TIMING:
            if key in launch:
                samples[key].append(s_ev.elapsed_time(e_ev) * 1e3)
        gd.TIMING = None
    res = {}
    for k in keys:
        v = sorted(samples[k])
        row = {"in-step": v[len(v) // 2] if v else float("nan")}
        row["hot"] = min(gd._time(launch[k], reps=10) for _ in range(3))
        for cond in CONDS[1:]:
            both = min(gd._time(lambda: (prefix(cond, k), launch[k]()), reps=10) for _ in range(3))
            alone = min(gd._time(lambda: prefix(cond, k), reps=10) for _ in range(3))
            row[cond] = both - alone
            row[cond + "_prefix"] = alone
        res[k] = row
    hdr = f"{'pair':14s} {'config':10s} " + " ".join(f"{c:>17s}" for c in ("in-step",) + CONDS)
    print(hdr)
    for k in keys:
        r = res[k]
        print(f"{label(k):14s} {gd.DUAL_DECISIONS[k][0]:10s} " + " ".join(f"{r[c]:17.1f}" for c in ("in-step",) + CONDS))
    print("prefix kernels alone (us): " + "; ".join(
        f"{label(k)}: " + " ".join(f"{c} {res[k][c + '_prefix']:.1f}" for c in CONDS[1:]) for k in keys[:1]))
    tot = {c: sum(res[k][c] * order.count(k) for k in keys) for c in ("in-step",) + CONDS}
    print("per step (x dispatches per step): " + "  ".join(f"{c} {tot[c] / 1e3:.3f} ms" for c in tot))


def summarize(csv, seq_path):
    import pandas as pd
    with open(seq_path) as f:
        seq = json.load(f)
    df = pd.read_csv(csv)
    piv = df.pivot_table(index=["Dispatch_Id", "Kernel_Name"], columns="Counter_Name", values="Counter_Value",
                         aggfunc="sum").reset_index().sort_values("Dispatch_Id")
    d = piv[piv["Kernel_Name"].str.contains("gemm_dual_kernel")].reset_index(drop=True)
    n_probe, n_step = len(seq["probe"]), len(seq["step"])
    if len(d) < n_probe + n_step:
        print(f"only {len(d)} dual dispatches in the trace (expected >= {n_probe + n_step})")
        return
    probe = d.iloc[len(d) - n_probe:]
    step = d.iloc[len(d) - n_probe - n_step:len(d) - n_probe]
    labels = [("in-step", s) for s in seq["step"]] + [tuple(p) for p in seq["probe"]]
    rows = collections.defaultdict(lambda: collections.defaultdict(float))
    for (cond, pr), (_, r) in zip(labels, pd.concat([step, probe]).iterrows()):
        g = rows[(pr, cond)]
        g["n"] += 1
        for c in r.index:
            if c not in ("Dispatch_Id", "Kernel_Name"):
                g[c] += float(r[c])
    cols = [c for c in piv.columns if c not in ("Dispatch_Id", "Kernel_Name")]
    print(f"{'pair':14s} {'condition':17s} {'n':>3s} " + " ".join(f"{c:>24s}" for c in cols) + "  (per dispatch)")
    for (pr, cond), g in sorted(rows.items()):
        print(f"{pr:14s} {cond:17s} {int(g['n']):3d} " + " ".join(f"{g[c] / g['n']:24.0f}" for c in cols))


if __name__ == "__main__":
    main()
