"""Mean of every collected counter per GEMM kernel over one or more rocprofv3 counter CSVs (scripts/gpu_r3_pmc_deep.sh)
plus derived ratios: per-wave fractions of SQ_WAVE_CYCLES spent waiting (SQ_WAIT_ANY: on counters / dependencies,
SQ_WAIT_INST_ANY: for instruction issue), VMEM / LDS instructions active, LDS array busy, TA / TD busy, L2 hit rate."""
import sys
from collections import defaultdict

import pandas as pd


def short(name):
    i = name.find("gemm_glds_kernel<")
    return name[i + len("gemm_glds_kernel"):name.find(">", i) + 1] if i >= 0 else name[:50]


def main(paths):
    rows = defaultdict(dict)
    for p in paths:
        df = pd.read_csv(p)
        df = df[df["Kernel_Name"].str.contains("gemm_glds_kernel")]
        piv = df.pivot_table(index=["Dispatch_Id", "Kernel_Name"], columns="Counter_Name", values="Counter_Value",
                             aggfunc="sum").reset_index()
        for name, g in piv.groupby("Kernel_Name"):
            for col in g.columns:
                if col not in ("Dispatch_Id", "Kernel_Name"):
                    rows[short(name)][col] = float(g[col].mean())
    for k, r in rows.items():
        print(f"== {k}")
        for c in sorted(r):
            print(f"   {c:36s} {r[c]:16.1f}")
        wc = r.get("SQ_WAVE_CYCLES")
        gui = r.get("GRBM_GUI_ACTIVE")
        der = {}
        if wc:
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_VMEM", "SQ_ACTIVE_INST_LDS",
                      "SQ_ACTIVE_INST_ANY"):
                if c in r:
                    der[c + " / SQ_WAVE_CYCLES"] = r[c] / wc
        if gui:
            for c, units in (("SQ_LDS_IDX_ACTIVE", 256), ("TA_TA_BUSY", 256), ("TD_TD_BUSY", 256),
                             ("SQ_VALU_MFMA_BUSY_CYCLES", 4 * 32), ("SQ_BUSY_CU_CYCLES", 256)):
                if c in r:
                    der[f"{c} / (GUI x {units})"] = r[c] / (gui * units)
        if "TCC_HIT" in r and "TCC_MISS" in r:
            der["L2 hit rate"] = r["TCC_HIT"] / max(r["TCC_HIT"] + r["TCC_MISS"], 1)
        for c, v in der.items():
            print(f"   -> {c:52s} {v:8.3f}")


if __name__ == "__main__":
    main(sys.argv[1:])
