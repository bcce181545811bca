"""Diagnose wrong tiles of the 8-phase GEMM (tile 40): exact small-integer operands, then explain each wrong 16 x 16
block of the 256 x 256 tile as one K-tile's A or B operand replaced by another K-tile's (a stale / early LDS image).

    python scripts/diag_8ph.py [kd ...]
"""
import os
import sys
from collections import Counter

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run(mode, kd, M=512, N=512):
    from iit_amd.ops import hip_kernels as K
    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(kd + mode)
    a = torch.randint(-3, 4, (M, kd), device=dev, generator=g).float()
    b = torch.randint(-2, 3, (kd, N), device=dev, generator=g).float()
    A = (a.t().contiguous() if mode == 3 else a).bfloat16()
    B = (b if mode in (2, 3) else b.t().contiguous()).bfloat16()
    lda = M if mode == 3 else kd
    ldb = N if mode in (2, 3) else kd
    ref = a @ b
    C = torch.full((M, N), float("nan"), device=dev)
    K.gemm_glds(A, B, C, M=M, N=N, K=kd, lda=lda, ldb=ldb, ldc=N, mode=mode, epi=K.EPI_F32_STORE, tile=40)
    torch.cuda.synchronize()
    bad = C != ref
    nb = int(bad.sum())
    print(f"mode {mode} kd {kd}: {nb} wrong of {M * N}", flush=True)
    if nb == 0:
        return
    nt = kd // 64
    P = [[a[:, 64 * i:64 * i + 64] @ b[64 * j:64 * j + 64, :] for j in range(nt)] for i in range(nt)]
    expl = Counter()
    pos = Counter()
    for r0 in range(0, M, 16):
        for c0 in range(0, N, 16):
            blk = bad[r0:r0 + 16, c0:c0 + 16]
            if not bool(blk.any()):
                continue
            rr, cc = (r0 % 256) // 16, (c0 % 256) // 16
            pos[(rr, cc)] += 1
            got = C[r0:r0 + 16, c0:c0 + 16]
            base = ref[r0:r0 + 16, c0:c0 + 16]
            found = None
            for j in range(nt):
                for i in range(nt):
                    if i == j:
                        continue
                    # A of K-tile j replaced by A of K-tile i (B of j kept) / B replaced / both / missing
                    for kind, sub in (("A", P[i][j]), ("B", P[j][i]), ("AB", P[i][i])):
                        v = base - P[j][j][r0:r0 + 16, c0:c0 + 16] + sub[r0:r0 + 16, c0:c0 + 16]
                        if torch.equal(v, got):
                            found = f"{kind} of kt{j} <- kt{i}"
                            break
                    if found:
                        break
                if found:
                    break
                v = base - P[j][j][r0:r0 + 16, c0:c0 + 16]
                if found is None and torch.equal(v, got):
                    found = f"kt{j} missing"
                    break
            expl[found or "unexplained"] += 1
    print("  explanations:", dict(expl.most_common(12)))
    print("  wrong blocks by (row block, col block) in the 256 tile:", sorted(pos.items())[:40])


def main():
    from iit_amd.ops import hip_kernels
    hip_kernels.lib()
    import ctypes
    lib = hip_kernels.lib()
    lib.iit_gemm_8ph_set_diag.argtypes = [ctypes.c_int]
    kds = [int(x) for x in sys.argv[1:]] or [192, 256, 640]
    for diag in (0, 1, 2, 8):
        lib.iit_gemm_8ph_set_diag(diag)
        print(f"== diag {diag}", flush=True)
        for kd in kds:
            for mode in (0, 2, 3):
                run(mode, kd)
    lib.iit_gemm_8ph_set_diag(0)


if __name__ == "__main__":
    main()
