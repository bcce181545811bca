"""Summarise rocprofv3 counter CSVs (scripts/gpu_pmc.sh) per GEMM kernel: mean counters per dispatch and derived
ratios.  MFMA busy is normalised as SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE * 4 SIMDs * 32 CUs / XCD), i.e.
assuming GRBM_GUI_ACTIVE sums the 8 XCDs' busy cycles; the LDS conflict rate is SQ_LDS_BANK_CONFLICT per
SQ_LDS_IDX_ACTIVE cycle; the L2 hit rate is TCC_HIT / (TCC_HIT + TCC_MISS)."""
import sys
from collections import defaultdict

import pandas as pd


def load(path):
    df = pd.read_csv(path)
    df = df[df["Kernel_Name"].str.contains("gemm_glds_kernel")]
    piv = df.pivot_table(index=["Dispatch_Id", "Kernel_Name"], columns="Counter_Name", values="Counter_Value",
                         aggfunc="sum").reset_index()
    return piv


def short(name):
    i = name.find("gemm_glds_kernel<")
    return name[i + len("gemm_glds_kernel"):name.find(">", i) + 1] if i >= 0 else name[:60]


def main():
    p1, p2 = load(sys.argv[1]), load(sys.argv[2])
    rows = defaultdict(dict)
    for piv in (p1, p2):
        for name, g in piv.groupby("Kernel_Name"):
            for col in g.columns:
                if col not in ("Dispatch_Id", "Kernel_Name"):
                    rows[short(name)][col] = g[col].mean()
    print(f"{'kernel <BM,BN,NS,AKM,BKM,EPI,NW>':36s} {'MFMA busy':>9s} {'LDS confl/active':>16s} {'L2 hit':>7s} "
          f"{'EA rd req':>10s} {'EA wr req':>10s}")
    for k, r in rows.items():
        gui = r.get("GRBM_GUI_ACTIVE", float("nan"))
        mfma = r.get("SQ_VALU_MFMA_BUSY_CYCLES", float("nan")) / (gui * 4 * 32)
        lds = r.get("SQ_LDS_BANK_CONFLICT", float("nan")) / max(r.get("SQ_LDS_IDX_ACTIVE", float("nan")), 1)
        hit = r.get("TCC_HIT", float("nan")) / max(r.get("TCC_HIT", 0) + r.get("TCC_MISS", 0), 1)
        print(f"{k:36s} {100 * mfma:8.1f}% {100 * lds:15.1f}% {100 * hit:6.1f}% {r.get('TCC_EA0_RDREQ', 0):10.0f} "
              f"{r.get('TCC_EA0_WRREQ', 0):10.0f}")


if __name__ == "__main__":
    main()
