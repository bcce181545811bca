"""In-step vs isolated time of every GEMM launch of the headline step (single GEMMs and dX + dW pairs): HIP events
around each dispatch inside eager steps issued behind a device sleep (graph-like back-to-back execution, as
scripts/tune_gemm_in_situ.py), against the dispatcher's isolated back-to-back timing of the same choice (timed here
when the shipped table skipped it).  Where the two differ, the launch pays for cold operands or the previous kernel.

    python scripts/gemm_context_penalty.py [--rounds 8]
"""
import argparse
import collections
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=8)
    a = ap.parse_args()
    import bench
    from iit_amd.ops import gemm_dispatch as gd
    args = argparse.Namespace(gpus=1, steps=1, warmup=1, batch=256, model="gpt2-small", engine="native", dtype="bf16",
                              graphs=0, profile_dir=None)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    pair, opt, loss_fn, it, step_fn, _, _ = bench.setup(args, dev)
    for _ in range(3):
        base, abl = next(it)
        pair.run_train_step(base, abl, loss_fn, opt)
    torch.cuda.synchronize()
    samples = collections.defaultdict(list)
    counts = collections.Counter()
    for r in range(a.rounds):
        gd.TIMING = []
        base, abl = next(it)
        torch.cuda.synchronize()
        torch.cuda._sleep(int(1.5e9))
        pair.run_train_step(base, abl, loss_fn, opt)
        torch.cuda.synchronize()
        for key, name, s_ev, e_ev in gd.TIMING:
            samples[(key, name)].append(s_ev.elapsed_time(e_ev) * 1e3)
            if r == 0:
                counts[(key, name)] += 1
        gd.TIMING = None
    rows = []
    for (key, name), v in samples.items():
        v = sorted(v)
        med = v[len(v) // 2]
        store = gd.DUAL_DECISIONS if key[0] == "dual" else gd.DECISIONS
        iso = store.get(key, (None, {}))[1].get(name, float("nan"))
        rows.append((key, name, counts[(key, name)], med, iso))
    tot_in = tot_iso = 0.0
    print(f"{'problem':64s} {'choice':12s} {'n/step':>6s} {'in-step':>8s} {'isolated':>8s} {'penalty us/step':>15s}")
    for key, name, n, med, iso in sorted(rows, key=lambda r: -(r[3] - (r[4] if r[4] == r[4] else r[3])) * r[2]):
        pen = (med - iso) * n if iso == iso else float("nan")
        if iso == iso:
            tot_in += med * n
            tot_iso += iso * n
        print(f"{str(key)[:64]:64s} {name:12s} {n:6d} {med:8.1f} {iso:8.1f} {pen:15.1f}")
    print(f"total over problems with an isolated time: in-step {tot_in / 1e3:.3f} ms, isolated {tot_iso / 1e3:.3f} ms")


if __name__ == "__main__":
    main()
