"""Per-kernel hardware counters over whole training steps (rocprofv3 --pmc ... -- python bench.py --graphs 0): for
every GEMM kernel (the repo's LDS-DMA, dual dX + dW and plain MFMA kernels, and hipBLASLt), dispatches, mean MFMA busy (SQ_VALU_MFMA_BUSY_CYCLES /
(GRBM_GUI_ACTIVE * 4 SIMDs * 32 CUs), as scripts/pmc_summary.py), LDS bank-conflict rate and the time-weighted
average over all GEMM dispatches (weights: GRBM_GUI_ACTIVE)."""
import sys
from collections import defaultdict

import pandas as pd


def short(name):
    i = name.find("gemm_glds_kernel<")
    if i >= 0:
        return "glds" + name[i + len("gemm_glds_kernel"):name.find(">", i) + 1]
    i = name.find("gemm_dual_kernel<")
    if i >= 0:  # the dual dX + dW launches (csrc/gemm_dual.hip): both tiles' configurations
        j = name.find("Cfg<", i)
        return "dual" + name[j + 3:name.find(">", j) + 1] if j >= 0 else "dual"
    i = name.find("gemm_kernel<")
    if i >= 0 and "glds" not in name:
        return "hipgemm" + name[i + len("gemm_kernel"):name.find(">", i) + 1]
    if name.startswith("Cijk") or name.startswith("Custom_Cijk"):
        j = name.find("_MT")
        return "hipBLASLt" + name[j:j + 16] if j >= 0 else name[:40]
    return None


def main(path, steps=0, adams_per_step=3):
    df = pd.read_csv(path)
    piv = df.pivot_table(index=["Dispatch_Id", "Kernel_Name"], columns="Counter_Name", values="Counter_Value",
                         aggfunc="sum").reset_index().sort_values("Dispatch_Id")
    if steps:  # only the last ``steps`` training steps (ends: every ``adams_per_step``-th Adam launch)
        adam = piv[piv["Kernel_Name"].str.contains("adam")]["Dispatch_Id"].tolist()
        lo, hi = adam[-(steps * adams_per_step) - 1], adam[-1]
        piv = piv[(piv["Dispatch_Id"] > lo) & (piv["Dispatch_Id"] <= hi)]
        print(f"# the last {steps} steps: dispatches {lo + 1}..{hi}")
    rows = defaultdict(lambda: defaultdict(float))
    for _, r in piv.iterrows():
        k = short(r["Kernel_Name"])
        if k is None:
            continue
        d = rows[k]
        d["n"] += 1
        for c in ("SQ_VALU_MFMA_BUSY_CYCLES", "GRBM_GUI_ACTIVE", "SQ_LDS_BANK_CONFLICT", "SQ_LDS_IDX_ACTIVE"):
            if c in r:
                d[c] += float(r[c])
    tot_m = tot_g = 0.0
    print(f"{'kernel':44s} {'dispatches':>10s} {'MFMA busy':>9s} {'LDS confl/active':>16s} {'GUI cycles/disp':>15s}")
    for k, d in sorted(rows.items(), key=lambda kv: -kv[1]["GRBM_GUI_ACTIVE"]):
        g = d["GRBM_GUI_ACTIVE"]
        m = d["SQ_VALU_MFMA_BUSY_CYCLES"] / max(g * 4 * 32, 1)
        lds = d["SQ_LDS_BANK_CONFLICT"] / max(d["SQ_LDS_IDX_ACTIVE"], 1)
        tot_m += d["SQ_VALU_MFMA_BUSY_CYCLES"]
        tot_g += g
        print(f"{k:44s} {int(d['n']):10d} {100 * m:8.1f}% {100 * lds:15.1f}% {g / d['n']:15.0f}")
    print(f"all GEMM dispatches, GUI-time-weighted MFMA busy: {100 * tot_m / max(tot_g * 4 * 32, 1):.1f}%")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 0)
