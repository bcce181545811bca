"""Hardware counters of the 8-phase GEMM (tile 40, both K-loop schedules) against hipBLASLt on 8192^3:
``rocprofv3 --pmc ... -- python3 scripts/pmc_8ph.py`` runs each kernel 3 times; ``python3 scripts/pmc_8ph.py
--summary CSV...`` prints per-kernel MFMA busy (SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE x 4 SIMDs x 32 CUs per
XCD)), LDS bank conflicts per active LDS cycle, and the wait / busy ratios."""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run():
    from iit_amd.ops import hip_kernels as K
    lib = K.lib()
    lib.iit_gemm_8ph_set_diag.argtypes = [ctypes.c_int]
    dev = "cuda"
    n = 8192
    for mode in (2, 0):
        A = (torch.rand(n, n, device=dev) * 2 - 1).bfloat16()
        B = (torch.rand(n, n, device=dev) * 2 - 1).bfloat16()
        C = torch.zeros(n, n, device=dev, dtype=torch.bfloat16)
        kw = dict(M=n, N=n, K=n, lda=n, ldb=n, ldc=n, mode=mode, epi=K.EPI_BF16, tile=40)
        for diag in (0, 8):
            lib.iit_gemm_8ph_set_diag(diag)
            for _ in range(3):
                K.gemm_glds(A, B, C, **kw)
        lib.iit_gemm_8ph_set_diag(0)
        for t in (41, 42):
            for _ in range(3):
                K.gemm_glds(A, B, C, **{**kw, "tile": t})
        b = B if mode == 2 else B.t()
        for _ in range(3):
            torch.mm(A, b, out=C)
        torch.cuda.synchronize()


def summary(paths):
    import pandas as pd
    df = pd.concat([pd.read_csv(p) for p in paths])
    piv = df.pivot_table(index=["Dispatch_Id", "Kernel_Name"], columns="Counter_Name", values="Counter_Value",
                         aggfunc="sum").reset_index()
    piv["short"] = piv["Kernel_Name"].str.slice(0, 70)
    print(f"{'kernel':70s} {'n':>3s} {'MFMA busy':>9s} {'LDS cf/act':>10s} {'wait/busy':>9s} {'LDS insts':>10s}")
    for name, g in piv.groupby("short"):
        r = g.mean(numeric_only=True)
        gui = r.get("GRBM_GUI_ACTIVE", float("nan"))
        mfma = r.get("SQ_VALU_MFMA_BUSY_CYCLES", float("nan")) / (gui * 4 * 32)
        lds = r.get("SQ_LDS_BANK_CONFLICT", float("nan")) / max(r.get("SQ_LDS_IDX_ACTIVE", float("nan")), 1)
        wait = r.get("SQ_WAIT_ANY", float("nan")) / max(r.get("SQ_WAVE_CYCLES", float("nan")), 1)
        print(f"{name:70s} {len(g):3d} {100 * mfma:8.1f}% {100 * lds:9.1f}% {100 * wait:8.1f}% "
              f"{r.get('SQ_INSTS_LDS', float('nan')):10.0f}")


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "--summary":
        summary(sys.argv[2:])
    else:
        run()
