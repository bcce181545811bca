"""LDS ring depth vs operand intake: the step's intake-bound GEMM shapes on the standard tiles and on their deep-ring
twins (tiles 12-14: 6 / 5 / 8 K-tiles in flight instead of 4), graph-timed (device time), best of 3."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from iit_amd.ops import gemm_dispatch as gd  # noqa: E402
from iit_amd.ops import hip_kernels as K  # noqa: E402

T = 4096
CASES_R3 = [  # round 3: two co-resident workgroups per CU (tiles 23-28) against the shipped choices
    ("fwd QKV [4096][2304] bf16", T, 2304, 768, 2, K.EPI_BF16, [(5, 1, False), (23, 1, False), (25, 1, False),
                                                                 (27, 1, False), (24, 1, False)]),
    ("fwd W_in [4096][3072] gelu", T, 3072, 768, 2, K.EPI_GELU, [(5, 1, False), (23, 1, False), (25, 1, False),
                                                                  (27, 1, False), (28, 1, False)]),
    ("fwd W_O [4096][768] resid", T, 768, 768, 2, K.EPI_F32_RESID, [(9, 1, False), (24, 1, False), (29, 1, False),
                                                                     (30, 1, False), (31, 1, False)]),
    ("fwd W_out [4096][768] resid", T, 768, 3072, 2, K.EPI_F32_RESID, [(9, 1, False), (24, 1, False),
                                                                        (29, 1, False), (30, 1, False), (31, 1, False)]),
    ("dX W_in [4096][768] bf16", T, 768, 3072, 0, K.EPI_BF16, [(9, 1, False), (24, 1, False), (29, 1, False),
                                                                (30, 1, False), (31, 1, False)]),
    ("dX QKV [4096][768] bf16", T, 768, 2304, 0, K.EPI_BF16, [(9, 1, False), (24, 1, False), (29, 1, False),
                                                               (30, 1, False), (31, 1, False)]),
    ("dX W_O [4096][768] bf16", T, 768, 768, 0, K.EPI_BF16, [(9, 1, False), (24, 1, False), (29, 1, False),
                                                              (30, 1, False), (31, 1, False)]),
    ("dX W_out [4096][3072] dgelu", T, 3072, 768, 0, K.EPI_DGELU, [(5, 1, False), (23, 1, False), (25, 1, False),
                                                                    (27, 1, False)]),
    ("dW W_in [768][3072] store", 768, 3072, T, 3, K.EPI_F32_STORE,
     [(11, 2, True), (10, 2, True), (26, 2, True), (23, 2, True), (25, 4, True), (26, 1, False), (24, 1, False)]),
    ("dW W_out [3072][768] store", 3072, 768, T, 3, K.EPI_F32_STORE,
     [(10, 2, True), (11, 2, True), (26, 2, True), (23, 2, True), (25, 4, True), (24, 1, False)]),
    ("dW QKV [768][2304] store", 768, 2304, T, 3, K.EPI_F32_STORE, [(3, 1, False), (26, 2, True), (23, 2, True),
                                                                     (24, 2, True), (25, 4, True)]),
    ("dW W_O [768][768] store", 768, 768, T, 3, K.EPI_F32_STORE, [(3, 2, True), (8, 4, True), (26, 4, True),
                                                                   (24, 4, True), (23, 4, True)]),
]
CASES_R3B = [  # round 3: in-flight depth on the big 8-wave tiles (tiles 32-34 vs 5 / 7)
    ("fwd QKV [4096][2304] bf16", T, 2304, 768, 2, K.EPI_BF16, [(5, 1, False), (7, 1, False), (32, 1, False),
                                                                 (34, 1, False)]),
    ("fwd W_in [4096][3072] gelu", T, 3072, 768, 2, K.EPI_GELU, [(5, 1, False), (7, 1, False), (32, 1, False),
                                                                  (33, 1, False), (34, 1, False)]),
    ("fwd QKV [8192][2304] bf16", 2 * T, 2304, 768, 2, K.EPI_BF16, [(5, 1, False), (7, 1, False), (32, 1, False),
                                                                     (34, 1, False)]),
    ("fwd W_in [8192][3072] gelu", 2 * T, 3072, 768, 2, K.EPI_GELU, [(5, 1, False), (7, 1, False), (32, 1, False),
                                                                      (33, 1, False), (34, 1, False)]),
    ("fwd W_out [8192][768] resid", 2 * T, 768, 3072, 2, K.EPI_F32_RESID, [(7, 1, False), (32, 1, False),
                                                                            (9, 1, False)]),
    ("dX W_out [4096][3072] dgelu", T, 3072, 768, 0, K.EPI_DGELU, [(5, 1, False), (7, 1, False), (32, 1, False),
                                                                    (33, 1, False), (34, 1, False)]),
    ("dW W_in [768][3072] store", 768, 3072, T, 3, K.EPI_F32_STORE, [(10, 2, True), (7, 1, False), (32, 1, False),
                                                                      (33, 1, False), (33, 2, True)]),
]
CASES_GM = [  # round 3: XCD-local tile-order group height (IIT_GM_SWEEP), shipped tiles
    ("fwd QKV [4096][2304] bf16", T, 2304, 768, 2, K.EPI_BF16, [(5, 1, False)]),
    ("fwd W_in [4096][3072] gelu", T, 3072, 768, 2, K.EPI_GELU, [(5, 1, False)]),
    ("fwd W_out [4096][768] resid", T, 768, 3072, 2, K.EPI_F32_RESID, [(9, 1, False), (24, 1, False)]),
    ("dX W_in [4096][768] bf16", T, 768, 3072, 0, K.EPI_BF16, [(9, 1, False)]),
    ("fwd QKV [8192][2304] bf16", 2 * T, 2304, 768, 2, K.EPI_BF16, [(5, 1, False)]),
    ("dW W_in [768][3072] store", 768, 3072, T, 3, K.EPI_F32_STORE, [(8, 1, False), (10, 2, True)]),
]
CASES = [  # name, M, N, K, mode, epi, [(tile, splits, reduce), ...]
    ("dW W_in [768][3072] store", 768, 3072, T, 3, K.EPI_F32_STORE, [(8, 1, False), (12, 1, False), (16, 1, False), (10, 2, True)]),
    ("dW W_O [768][768] store", 768, 768, T, 3, K.EPI_F32_STORE, [(3, 2, True), (14, 2, True), (17, 2, True), (3, 1, False),
                                                                    (17, 1, False), (8, 4, True), (16, 4, True)]),
    ("dW QKV [768][2304] store", 768, 2304, T, 3, K.EPI_F32_STORE, [(3, 1, False), (17, 1, False)]),
    ("fwd W_out [4096][768] resid", T, 768, 3072, 2, K.EPI_F32_RESID, [(9, 1, False), (15, 1, False)]),
    ("fwd W_in [4096][3072] bf16", T, 3072, 768, 2, K.EPI_BF16, [(5, 1, False), (0, 1, False), (18, 1, False)]),
    ("dX W_in [4096][768] bf16", T, 768, 3072, 0, K.EPI_BF16, [(9, 1, False), (15, 1, False)]),
    ("fwd W_O [4096][768] resid", T, 768, 768, 2, K.EPI_F32_RESID, [(9, 1, False), (15, 1, False)]),
]


def main():
    dev = "cuda"
    which = os.environ.get("R3", "1")
    cases = CASES_R3B if which == "b" else CASES_GM if which == "gm" else CASES_R3 if which == "1" else CASES
    for name, M, N, Kd, mode, epi, variants in cases:
        torch.manual_seed(0)
        A = (torch.randn(Kd, M) if mode & 1 else torch.randn(M, Kd)).to(dev).bfloat16()
        B = (torch.randn(Kd, N) if mode & 2 else torch.randn(N, Kd)).to(dev).bfloat16() / 16
        lda = M if mode & 1 else Kd
        ldb = N if mode & 2 else Kd
        f32 = epi in (K.EPI_F32_STORE, K.EPI_F32_ACC, K.EPI_F32_RESID)
        C = torch.zeros(M, N, device=dev, dtype=torch.float32 if f32 else torch.bfloat16)
        R = torch.randn(M, N, device=dev) if epi == K.EPI_F32_RESID else None
        kw = dict(M=M, N=N, K=Kd, lda=lda, ldb=ldb, ldc=N, mode=mode, epi=epi)
        ex = dict(resid=R, ldr=N) if R is not None else {}
        if epi in (K.EPI_GELU, K.EPI_DGELU):  # pre-activation: written (GELU) or read (DGELU)
            ex = dict(C2=torch.randn(M, N, device=dev).bfloat16(), ldc2=N)
        ref = None
        out = []
        gms = [int(g) for g in os.environ.get("IIT_GM_SWEEP", "0").split(",")]
        variants = [(t, sp, red, gm) for t, sp, red in variants for gm in gms]
        for tile, sp, red, gm in variants:
            K.gemm_glds_set_group_m(gm)
            if not K.gemm_glds_ok(A, B, C, tile=tile, splits=sp, reduce=red, **kw, **ex):
                out.append(f"t{tile}{'r' if red else 'k'}{sp}g{gm}: n/a")
                continue
            f = lambda: K.gemm_glds(A, B, C, tile=tile, splits=sp, reduce=red, **kw, **ex)  # noqa: E731
            f()
            torch.cuda.synchronize()
            ref = C.clone() if ref is None else ref
            err = float(((C.float() - ref.float()).norm() / ref.float().norm()))
            us = min(gd._time(f, reps=20) for _ in range(3))
            tf = 2 * M * N * Kd / (us * 1e-6) / 1e12
            out.append(f"t{tile}{'r' if red else 'k'}{sp}{f'g{gm}' if gm else ''}: {us:6.1f} us {tf:5.0f} TF/s "
                       f"(rel diff {err:.1e})")
        print(f"{name:28s} " + " | ".join(out), flush=True)


if __name__ == "__main__":
    main()
