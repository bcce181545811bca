"""Per-step kernel time breakdown over the steady-state steps of a rocprofv3 kernel trace of bench.py.

Steps are delimited by the optimizer kernel (3 Adam launches per IOI_ModelPair step); the window is the last
``--steps`` complete steps before the trailing eval.  Prints ms/step per kernel (top N), the GPU busy fraction
and grouped totals (GEMM / attention / norm / elementwise / optimizer)."""
import argparse
import collections
import csv


def group_of(k: str) -> str:
    """Kernel family of a lower-cased kernel name."""
    if "conv" in k or k.startswith("igemm_") or "im2d2col" in k or "col2im" in k:
        return "conv"
    if "gemm" in k or "cijk" in k:
        return "gemm"
    if "attn" in k or "flash" in k or "fa_" in k:
        return "attention"
    if "ln_" in k or "rms_" in k or "batchnorm" in k or "bn_stats" in k or "bn_apply" in k or "bn_bwd" in k:
        return "norm"
    if "adam" in k or "sumsq" in k:
        return "optimizer"
    if "nccl" in k or "rccl" in k:
        return "collective"
    return "elementwise"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--per-step-adam", type=int, default=3)
    ap.add_argument("--top", type=int, default=30)
    ap.add_argument("--gaps", type=int, default=0, help="also list the N largest idle gaps (with neighbours)")
    ap.add_argument("--dump-step", default=None, help="write the last steady step's kernel sequence to this file")
    a = ap.parse_args()
    rows = []
    with open(a.trace) as f:
        for x in csv.DictReader(f):
            rows.append((int(x["Start_Timestamp"]), int(x["End_Timestamp"]), x["Kernel_Name"]))
    rows.sort()
    adam = [i for i, x in enumerate(rows) if "adam" in x[2]]
    ends = [rows[adam[i]][1] for i in range(a.per_step_adam - 1, len(adam), a.per_step_adam)]
    spans = list(zip(ends[:-1], ends[1:]))
    med = sorted(b - s for s, b in spans)[len(spans) // 2]
    spans = [sp for sp in spans if sp[1] - sp[0] < 1.5 * med][-a.steps:]  # drop eval / priming outliers
    t0, t1 = spans[0][0], spans[-1][1]
    n = len(spans)
    per = collections.Counter()
    calls = collections.Counter()
    busy = 0
    cur = None
    for s, e, name in rows:
        if e <= t0 or s >= t1:
            continue
        s, e = max(s, t0), min(e, t1)
        per[name] += e - s
        calls[name] += 1
        if cur is None or s > cur[1]:
            if cur:
                busy += cur[1] - cur[0]
            cur = [s, e]
        else:
            cur[1] = max(cur[1], e)
    if cur:
        busy += cur[1] - cur[0]
    wall = (t1 - t0) / n / 1e6
    print(f"{n} steady-state steps: {wall:.3f} ms/step wall, GPU busy {busy / (t1 - t0):.3f}, "
          f"kernel sum {sum(per.values()) / n / 1e6:.3f} ms/step")
    groups = collections.Counter()
    for name, t in per.items():
        k = name.lower()
        g = group_of(k)
        groups[g] += t
    print("groups (ms/step): " + ", ".join(f"{g} {t / n / 1e6:.2f}" for g, t in groups.most_common()))
    if a.gaps:
        win = [r for r in rows if t0 <= r[0] < t1]
        gaps = []
        end = win[0][1]
        for i in range(1, len(win)):
            if win[i][0] > end:
                gaps.append((win[i][0] - end, win[i - 1][2][:60], win[i][2][:60]))
            end = max(end, win[i][1])
        gaps.sort(reverse=True)
        tot = collections.Counter()
        for gp, before, after in gaps:
            tot[(before, after)] += gp
        print(f"idle gaps: {len(gaps)} totalling {sum(g for g, _, _ in gaps) / n / 1e6:.3f} ms/step; by neighbours:")
        for (before, after), gp in tot.most_common(a.gaps):
            print(f"  {gp / n / 1e3:8.1f} us/step  after {before}  |  before {after}")
    if a.dump_step:
        s0, s1 = spans[-1]
        with open(a.dump_step, "w") as f:
            f.write("# start_us  dur_us  kernel (one steady-state step)\n")
            for s, e, name in rows:
                if s0 <= s < s1:
                    f.write(f"{(s - s0) / 1e3:9.1f} {(e - s) / 1e3:8.1f}  {name[:110]}\n")
    print(f"{'ms/step':>8s} {'calls':>6s} {'avg us':>8s}  kernel")
    for name, t in per.most_common(a.top):
        print(f"{t / n / 1e6:8.3f} {calls[name] / n:6.1f} {t / calls[name] / 1e3:8.1f}  {name[:100]}")


if __name__ == "__main__":
    main()
