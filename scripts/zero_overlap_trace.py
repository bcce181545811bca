"""Overlap of the ZeRO-1 all-gather with compute in a rank's rocprofv3 trace (--kernel-trace --memory-copy-trace):
the time of host-to-device copies (gloo's gathered pieces landing in the arena, in the one-GPU rehearsal) that runs
while a kernel of the same process executes, over the total copy time.

    python scripts/zero_overlap_trace.py <dir with *kernel_trace.csv and *memory_copy_trace.csv>
"""
import glob
import sys

import pandas as pd


def intervals(df):
    s = df.sort_values("Start_Timestamp")
    out = []
    for a, b in zip(s["Start_Timestamp"], s["End_Timestamp"]):
        if out and a <= out[-1][1]:
            out[-1][1] = max(out[-1][1], b)
        else:
            out.append([a, b])
    return out


def overlap(copies, kernels):
    """(total copy ns, ns of it inside a kernel interval)"""
    tot = ov = 0
    j = 0
    for a, b in sorted(copies):
        tot += b - a
        while j < len(kernels) and kernels[j][1] < a:
            j += 1
        k = j
        while k < len(kernels) and kernels[k][0] < b:
            ov += max(0, min(b, kernels[k][1]) - max(a, kernels[k][0]))
            k += 1
    return tot, ov


def main(d):
    kt = pd.read_csv(glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True)[0])
    mc = pd.read_csv(glob.glob(f"{d}/**/*memory_copy_trace.csv", recursive=True)[0])
    kern = intervals(kt)
    col = "Direction" if "Direction" in mc.columns else None
    h2d = mc[mc[col].astype(str).str.contains("HOST_TO_DEVICE|H2D", regex=True)] if col else mc
    copies = list(zip(h2d["Start_Timestamp"], h2d["End_Timestamp"]))
    tot, ov = overlap(copies, kern)
    print(f"{d}: {len(copies)} host-to-device copies, {tot / 1e6:.2f} ms total, {ov / 1e6:.2f} ms under a kernel "
          f"({100.0 * ov / max(tot, 1):.1f} %); {len(kt)} kernels")


if __name__ == "__main__":
    for d in sys.argv[1:]:
        main(d)
