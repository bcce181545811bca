"""ctypes bindings to ``libiit_hip.so`` (the hand-written gfx950 kernels in ``csrc/``).

Every launcher takes raw device pointers and the *current torch stream*, so the
kernels interleave with torch ops and are captured by ``torch.cuda.graph``.
Loading is strict: on a GPU, a missing / unbuildable library raises instead of
silently falling back to PyTorch ops.
"""
from __future__ import annotations

import ctypes
import math
import os
from typing import Optional, Sequence

import numpy as np
import torch

from . import build as _build

c_void_p, c_long, c_int, c_float, c_ull = ctypes.c_void_p, ctypes.c_long, ctypes.c_int, ctypes.c_float, ctypes.c_ulonglong

EPI_BF16, EPI_BF16_BIAS3, EPI_F32_RESID, EPI_GELU, EPI_DGELU, EPI_F32_ACC, EPI_F32_ACC_QKV, EPI_F32_STORE = range(8)
EPI_GELU_ERF = 8  # EPI_GELU with the exact (erf) GELU
EPI_DGELU_ERF = 9  # EPI_DGELU with the exact (erf) GELU's derivative
MODE_NN, MODE_AKM, MODE_BKM, MODE_AF32, MODE_BF32 = 0, 1, 2, 4, 8

_LIB = None

_SIGS = {
    "iit_gemm": [c_void_p] * 10 + [c_long] * 5 + [c_int] * 12 + [c_void_p],
    "iit_gemm_glds": [c_void_p] * 8 + [c_long] * 5 + [c_int] * 8 + [c_void_p] * 4,
    "iit_gemm_glds_ok": [c_void_p] * 5 + [c_long] * 5 + [c_int] * 9,
    "iit_gemm_glds_sm": [c_void_p] * 8 + [c_long] * 5 + [c_int] * 8 + [c_void_p] * 3 + [c_int] + [c_void_p] * 3,
    "iit_embed_pos_fwd": [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_void_p],
    "iit_embed_pos_bwd": [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_void_p],
    "iit_ln_fwd": [c_void_p] * 6 + [c_int, c_int, c_float, c_void_p],
    "iit_ln_bwd": [c_void_p, c_int] + [c_void_p] * 9 + [c_int, c_int, c_int, c_void_p],
    "iit_ln_fwd_sel": [c_void_p] * 6 + [c_int, c_int, c_float, c_ull, c_int, c_int, c_void_p],
    "iit_ln_bwd_xh16": [c_void_p, c_int] + [c_void_p] * 5 + [c_int, c_int, c_int, c_void_p],
    "iit_ln_bwd_sel": [c_void_p, c_int] + [c_void_p] * 9 + [c_int, c_int, c_int, c_ull, c_int, c_void_p],
    "iit_ln_bwd_part": [c_void_p, c_int] + [c_void_p] * 10 + [c_int, c_int, c_int, c_ull, c_int, c_void_p, c_void_p],
    "iit_ln_fwd_twin": [c_void_p] * 7 + [c_int, c_int, c_float, c_void_p],
    "iit_ln_bwd_part_rows": [],
    "iit_attn_small_fwd": [c_void_p] * 4 + [c_ull, c_int, c_int, c_int, c_int, c_long, c_long, c_long, c_float, c_int,
                                            c_void_p],
    "iit_attn_small_bwd": [c_void_p] * 4 + [c_ull, c_int, c_int, c_int, c_int, c_long, c_long, c_float, c_int, c_void_p],
    "iit_attn_mfma_fwd": [c_void_p] * 4 + [c_ull, c_int, c_int, c_int, c_int, c_long, c_long, c_long, c_float, c_int,
                                           c_void_p],
    "iit_attn_mfma_fwd_pair": [c_void_p] * 4 + [c_ull, c_int, c_int, c_int, c_int, c_long, c_long, c_long, c_float,
                                                c_int, c_void_p, c_int, c_ull, c_void_p],
    "iit_attn_mfma_bwd": [c_void_p] * 4 + [c_ull, c_int, c_int, c_int, c_int, c_long, c_long, c_float, c_int, c_void_p],
    "iit_attn_mfma_fwd_spec": [c_void_p] * 3 + [c_int] * 4 + [c_long, c_long, c_float, c_int, c_int, c_void_p,
                                                               c_void_p],
    "iit_attn_mfma_bwd_spec": [c_void_p] * 4 + [c_int] * 4 + [c_long, c_long, c_float, c_int, c_void_p, c_void_p],
    "iit_ce_fwd": [c_void_p, c_long, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_void_p],
    "iit_ce_bwd": [c_void_p, c_long, c_void_p, c_void_p, c_void_p, c_float, c_void_p, c_long, c_int, c_int, c_int,
                   c_void_p, c_void_p],
    "iit_adam_flat": [c_void_p] * 6 + [c_int, c_void_p, c_int] + [c_float] * 6 + [c_void_p] * 3
                     + [c_void_p, c_int, c_void_p, c_void_p],
    "iit_sumsq_2d": [c_void_p, c_long, c_int, c_int, c_void_p, c_void_p],
    "iit_kl_rows": [c_void_p, c_long, c_void_p, c_long, c_int, c_int, c_void_p, c_void_p],
    "iit_adam_span_size": [],
    "iit_sumsq_spans": [c_void_p, c_void_p, c_int, c_void_p, c_int, c_int, c_void_p, c_void_p],
    "iit_adam_spans": [c_void_p] * 6 + [c_int, c_void_p] + [c_float] * 6 + [c_void_p] * 4,
    "iit_gelu_fwd": [c_void_p, c_long, c_void_p, c_long, c_int, c_int, c_int, c_void_p],
    "iit_shadow_refresh": [c_void_p, c_int, c_void_p],
    "iit_shadow_desc_size": [],
    "iit_colsum_accum": [c_void_p, c_int, c_long, c_void_p, c_int, c_int, c_void_p],
    "iit_dgelu": [c_void_p, c_void_p, c_void_p, c_long, c_int, c_void_p],
    "iit_add_bf16": [c_void_p, c_long, c_void_p, c_long, c_void_p, c_long, c_void_p, c_int, c_int, c_void_p],
    "iit_device_sync": [],
    "iit_zero_chunks": [c_void_p, c_void_p, c_int, c_void_p],
    "iit_zero_ranges": [c_void_p, c_void_p, c_void_p, c_int, c_void_p],
    "iit_colsum_multi": [c_void_p] * 6 + [c_int, c_void_p],
    "iit_rms_fwd": [c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_int, c_int, c_float, c_void_p],
    "iit_rms_bwd": [c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_void_p],
    "iit_rms_bwd_res": [c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int,
                        c_void_p],
    "iit_rotary": [c_void_p, c_long, c_long, c_long, c_void_p, c_void_p, c_void_p] + [c_int] * 8 + [c_void_p],
    "iit_swiglu_fwd": [c_void_p, c_void_p, c_void_p, c_long, c_void_p],
    "iit_swiglu_bwd": [c_void_p] * 5 + [c_long, c_void_p],
    "iit_swiglu_splice_fwd": [c_void_p] * 4 + [c_long, c_void_p, c_void_p],
    "iit_sparse_pair": [c_void_p, c_long, c_long, c_void_p, c_int, c_void_p],
    "iit_gemm_dual_set_group_m": [c_int],
    "iit_swiglu_splice_bwd": [c_void_p] * 5 + [c_long, c_void_p, c_void_p],
    "iit_embed_splice_fwd": [c_void_p, c_void_p, c_long, c_void_p, c_void_p, c_long, c_int, c_void_p, c_void_p],
    "iit_embed_splice_bwd": [c_void_p, c_void_p, c_int, c_void_p, c_long, c_long, c_int, c_void_p, c_void_p],
    "iit_flash_fwd": [c_void_p] * 3 + [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_ull] + [c_int] * 5
                     + [c_float, c_int, c_void_p, c_void_p],
    "iit_flash_bwd": [c_void_p] * 3 + [c_void_p] * 11 + [c_ull] + [c_int] * 5 + [c_float, c_int, c_void_p, c_void_p],
    "iit_splice": [c_void_p, c_void_p, c_void_p, c_long, c_void_p, c_int, c_int, c_float, c_void_p],
    "iit_splice_spec_size": [],
    "iit_bn_fwd": [c_void_p] * 8 + [c_long, c_int, c_float, c_int, c_int, c_void_p, c_float, c_void_p, c_void_p,
                                    c_void_p, c_int, c_int, c_int, c_int, c_void_p],
    "iit_bn_bwd": [c_void_p] * 7 + [c_long, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                    c_int, c_int, c_int, c_int, c_void_p],
    "iit_gemm_glds_set_prof": [c_void_p],
    "iit_maxpool3s2_fwd": [c_void_p] * 3 + [c_int] * 5 + [c_void_p],
    "iit_bn_ws_floats": [c_int],
    "iit_maxpool3s2_bwd": [c_void_p] * 3 + [c_int] * 5 + [c_void_p],
    "iit_gemm_dual_ok": [c_void_p] * 3 + [c_long] * 3 + [c_int] * 7 + [c_void_p] * 4 + [c_long] * 4 + [c_int] * 5,
    "iit_gemm_dual": [c_void_p] * 3 + [c_long] * 3 + [c_int] * 6 + [c_void_p] * 2 + [c_void_p] * 4 + [c_long] * 4
                     + [c_int] * 5 + [c_void_p] * 3 + [c_void_p, c_long, c_void_p, c_long, c_int, c_void_p],
    "iit_gemm_glds_set_group_m": [c_int],
    "iit_ioi_hl_label": [c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_void_p, c_void_p],
    "iit_conv3x3_tiles": [],
    "iit_conv3x3_ok": [c_long, c_int, c_int, c_int, c_int, c_int, c_int],
    "iit_conv3x3": [c_void_p] * 4 + [c_long, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_void_p, c_void_p,
                                     c_void_p, c_void_p],
    "iit_conv3x3_rows": [c_int],
    "iit_conv2d_ok": [c_long] + [c_int] * 12,
    "iit_conv2d": [c_void_p] * 4 + [c_long] + [c_int] * 12 + [c_void_p] * 4,
    "iit_conv2d_wgrad_ok": [c_long] + [c_int] * 11,
    "iit_conv2d_wgrad": [c_void_p] * 4 + [c_long] + [c_int] * 12 + [c_void_p] * 3,
    "iit_bn_fwd_tiles": [c_void_p] * 4 + [c_int, c_int] + [c_void_p] * 4 + [c_long, c_int, c_float, c_int, c_void_p,
                                                                           c_float, c_void_p, c_void_p],
    "iit_conv3x3_wgrad_tiles": [],
    "iit_conv3x3_wgrad_ok": [c_long, c_int, c_int, c_int, c_int, c_int, c_int],
    "iit_conv3x3_wgrad": [c_void_p] * 4 + [c_long, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_void_p, c_void_p,
                                           c_void_p],
}


def lib():
    """Load (building first if stale) the kernel library."""
    global _LIB
    if _LIB is None:
        if not _build.is_up_to_date():
            _build.build()
        L = ctypes.CDLL(_build.LIB)
        for name, argtypes in _SIGS.items():
            fn = getattr(L, name)
            fn.argtypes = argtypes
            fn.restype = c_int
        _LIB = L
        # XCD-local tile-order group height of the single-problem LDS-DMA launches: 4 M-tiles per column group
        # measured 0.2-0.3 % faster than 8 on the headline step over two alternating rounds on one box (16 slower;
        # profiles/launch_knobs_r4s2.txt); IIT_GEMM_GROUP_M overrides
        gm = os.environ.get("IIT_GEMM_GROUP_M", "4")
        if gm:
            L.iit_gemm_glds_set_group_m(int(gm))
        # the same for the dual dX + dW launches: 2 measured 0.2-0.4 % faster than the body's 8 over two alternating
        # rounds (4 in between, 16 slower; profiles/launch_knobs_r4s2.txt); IIT_GEMM_DUAL_GROUP_M overrides
        dgm = os.environ.get("IIT_GEMM_DUAL_GROUP_M", "2")
        if dgm:
            L.iit_gemm_dual_set_group_m(int(dgm))
    return _LIB


def available() -> bool:
    try:
        lib()
        return True
    except Exception:
        return False


def _p(t: Optional[torch.Tensor]):
    return None if t is None else t.data_ptr()


def _stream():
    return torch.cuda.current_stream().cuda_stream


CHECK_BOUNDS = os.environ.get("IIT_CHECK_BOUNDS", "0") == "1"


def _avail(t: torch.Tensor) -> int:
    """Elements of ``t``'s storage from its first element to the end."""
    st = t.untyped_storage()
    return (st.nbytes() - (t.data_ptr() - st.data_ptr())) // t.element_size()


def _bounds(what: str, *spans):
    """Host-side extent check (``IIT_CHECK_BOUNDS=1``) of raw-pointer kernel operands before a launch: each span
    ``(name, t, rows, cols, ld)`` must fit inside ``t``'s storage -- a debugging aid that turns an out-of-bounds
    launch into a Python error instead of a GPU fault."""
    for name, t, rows, cols, ld in spans:
        if t is None or rows <= 0 or cols <= 0:
            continue
        need = (rows - 1) * ld + cols
        have = _avail(t)
        if need > have or ld < cols and rows > 1:
            raise RuntimeError(f"{what}: operand {name} needs {rows}x{cols} (ld {ld}) = {need} elements, "
                               f"storage holds {have} (shape {tuple(t.shape)}, stride {t.stride()})")


def _check(rc: int, what: str):
    if rc != 0:
        raise RuntimeError(f"{what} failed with hip error {rc}")


# ------------------------------------------------------------------------------ GEMM
N_CU = 256


def _tiling(M: int, N: int, K: int, allow_split: bool):
    t128 = math.ceil(M / 128) * math.ceil(N / 128)
    if t128 >= 240:
        return 1, 1
    t64 = math.ceil(M / 64) * math.ceil(N / 64)
    splits = 1
    if allow_split and t64 < 240 and K >= 1024:
        splits = max(1, min(math.ceil(480 / t64), K // 512))
    return 0, splits


def gemm(A, B, C, *, M: int, N: int, K: int, lda: int, ldb: int, ldc: int, mode: int = MODE_NN, epi: int = EPI_BF16,
         C2=None, C3=None, bias0=None, bias1=None, bias2=None, resid=None, ldr: int = 0, aux=None, ldc2: int = 0,
         bias_cols: int = 0, qkv=(0, 0, 0), atomic: bool = False, splits: Optional[int] = None):
    """C = A @ B (+ epilogue). Operand layouts: see ``csrc/gemm.hip``; strides in elements."""
    can_split = epi in (EPI_F32_ACC, EPI_F32_ACC_QKV)
    big, auto_splits = _tiling(M, N, K, can_split)
    if splits is None:
        splits = auto_splits
    if CHECK_BOUNDS:
        _gemm_bounds("iit_gemm", A, B, C, C2, resid, M, N, K, lda, ldb, ldc, ldc2, ldr, mode, qkv)
    rc = lib().iit_gemm(_p(A), _p(B), _p(C), _p(C2), _p(C3), _p(bias0), _p(bias1), _p(bias2), _p(resid), _p(aux),
                        lda, ldb, ldc, ldc2, ldr, M, N, K, mode, epi, splits, big, bias_cols, qkv[0], qkv[1], qkv[2],
                        int(atomic), _stream())
    _check(rc, "iit_gemm")


GLDS_TILES = {0: (128, 128), 1: (128, 64), 2: (64, 128), 3: (64, 64), 4: (128, 128),  # tile 4: 4 LDS stages
              5: (256, 192),  # tiles 5-7: 8 waves (two per SIMD); 5: 4 x 6 MFMA tiles per wave, 2 stages
              6: (128, 128), 7: (256, 128),
              8: (96, 96),  # 96 x 96: 256 tiles for the [768][3072] weight gradients
              9: (128, 96),  # 128 x 96: 256 tiles for the [4096][768] outputs
              10: (96, 192), 11: (192, 96),  # 2-way reduction split: 256 workgroups for the [768][3072] gradients
              12: (96, 96), 13: (128, 96), 14: (64, 64),  # deep LDS rings (6 / 5 / 8 K-tiles)
              15: (128, 96), 16: (96, 96), 17: (64, 64), 18: (128, 128),  # 128-deep K-tiles (K % 128 == 0)
              20: (192, 192),  # weight gradients with a 4-way reduction split (2-deep ring)
              21: (192, 128), 22: (128, 192),
              # two co-resident workgroups per CU (<= 80 KiB LDS each): prologue / epilogue overlap
              23: (128, 96), 24: (64, 96), 25: (128, 128), 26: (96, 96), 27: (128, 192), 28: (64, 192),
              29: (64, 96), 30: (64, 64), 31: (64, 128),  # three / four workgroups per CU
              32: (256, 128), 33: (128, 256), 34: (256, 256),  # 8 waves: 3-deep rings (32, 33), 256 x 256 (34)
              # csrc/gemm_8ph.hip: 256 x 256, 8 waves in two ping-pong groups, 8-phase K-loop (no K split)
              40: (256, 256),
              # csrc/gemm_4w.hip: 256 x 256, 4 waves of 128 x 128 on 32x32x16 MFMA, AGPR accumulators (no K split),
              # 64-deep K-tiles in a 2-slot ring (41) / 32-deep in a 4-slot ring (42)
              41: (256, 256), 42: (256, 256)}
# tiles 12-14 measured slower than their 4-deep twins on every step shape (profiles/gemm_ring_depth_r2.txt: the tiles
# are intake-bandwidth-bound, not latency-bound), so the dispatcher does not offer them; kept for the experiment.
# Tiles 15-18 (128-deep K-tiles) are within a few % of the 64-deep tiles and compete per shape.
# Tile 42 (the four-wave kernel with 32-deep K-tiles) measured slower than tile 41 on every large shape
# (profiles/gemm_big_tiles_r5.txt): not offered either.
GLDS_DISPATCH_TILES = tuple(t for t in GLDS_TILES if t not in (12, 13, 14, 32, 33, 34, 42))


def _gemm_bounds(what, A, B, C, C2, resid, M, N, K, lda, ldb, ldc, ldc2, ldr, mode, qkv=(0, 0, 0)):
    a = ("A", A, K, M, lda) if mode & MODE_AKM else ("A", A, M, K, lda)
    b = ("B", B, K, N, ldb) if mode & MODE_BKM else ("B", B, N, K, ldb)
    if qkv[0]:
        # head-blocked QKV scatter (EPI_F32_ACC_QKV): C / C2 / C3 each hold [H][qkv_d][dh] (rows of the model dim)
        dh, H, d = qkv
        per = ("C", C, 1, H * d * dh, H * d * dh)
        _bounds(what, a, b, per, ("C2",) + per[1:] if C2 is None else ("C2", C2, 1, H * d * dh, H * d * dh))
        return
    _bounds(what, a, b, ("C", C, M, N, ldc), ("C2", C2, M, N, ldc2 or ldc), ("resid", resid, M, N, ldr or ldc))


def gemm_glds_ok(A, B, C, *, M, N, K, lda, ldb, ldc, mode, epi, C2=None, resid=None, ldc2=0, ldr=0, bias_cols=0,
                 tile=0, splits=1, reduce=False) -> bool:
    """Whether the LDS-DMA kernel (``csrc/gemm_glds.hip``) covers this problem with tile ``tile`` and split-K
    factor ``splits`` (atomic split-K: fp32-accumulate epilogue only; ``reduce``: the deterministic reduction
    split, fp32 accumulate or store)."""
    if any(t is not None and (not t.is_cuda or t.dtype not in (torch.bfloat16,)) for t in (A, B)):
        return False
    return bool(lib().iit_gemm_glds_ok(_p(A), _p(B), _p(C), _p(C2), _p(resid), lda, ldb, ldc, ldc2, ldr, M, N, K,
                                       mode, epi, bias_cols, tile, splits, int(reduce)))


_SPLIT_WS = {}  # (device, stream) -> [fp32 partial-tile workspace, int32 tickets, retired buffers]


def split_workspace(M: int, N: int, tile, splits: int, device) -> tuple:
    """Workspace of the reduction split-K: ``splits * M * N`` fp32 partials and one ticket per output tile.

    One buffer pair per (device, stream), shared by every problem launched on that stream (launches on one
    stream are serial, and every launch leaves its tickets at zero), grown on demand.  A grown-out buffer is
    retired, never freed: a captured graph keeps using the address it was captured with.  Launches on different
    streams never share partial tiles.  The dispatcher measures the candidates -- and so sizes the buffers --
    outside graph capture."""
    stream = torch.cuda.current_stream(device).cuda_stream
    key = (str(device), stream)
    ent = _SPLIT_WS.get(key)
    bm, bn = GLDS_TILES[tile] if isinstance(tile, int) else tile  # a tile id or its (BM, BN)
    need_ws, need_cnt = splits * M * N, (M // bm) * (N // bn)
    if ent is None:
        ent = _SPLIT_WS[key] = [None, None, []]
    if ent[0] is None or ent[0].numel() < need_ws:
        if ent[0] is not None:
            ent[2].append(ent[0])
        ent[0] = torch.empty(need_ws, dtype=torch.float32, device=device)
    if ent[1] is None or ent[1].numel() < need_cnt:
        if ent[1] is not None:
            ent[2].append(ent[1])
        ent[1] = torch.zeros(max(need_cnt, 1024), dtype=torch.int32, device=device)
    return ent[0], ent[1]


GLDS_STORE_MODE = int(os.environ.get("IIT_GEMM_STORE", "0"))  # epilogue stores: 0 plain, 1 non-temporal, 2 write-through


def gemm_glds(A, B, C, *, M, N, K, lda, ldb, ldc, mode, epi, C2=None, bias0=None, bias1=None, bias2=None, resid=None,
              ldc2=0, ldr=0, bias_cols=0, tile=0, splits=1, csum=None, reduce=False, store_mode=None, bsum=None,
              gsq=None):
    """C = A @ B (+ epilogue) on the LDS-DMA MFMA kernel; bf16 operands, M/N/K multiples of the tile.
    ``EPI_DGELU`` (mode 0): ``C2`` is the saved bf16 pre-activation (row stride ``ldc2``); ``csum`` (fp32 [N],
    optional) accumulates the column sums of the stored bf16 output.
    ``splits > 1``: split-K.  By default the partial tiles are added into C with fp32 atomics (accumulate
    epilogue); with ``reduce`` they go to a workspace and the last-arriving split sums them in a fixed order
    (run-to-run deterministic, no atomics, and valid for fp32 stores too).
    ``bsum`` (mode 3 only, fp32 [N], optional): += the column sums of B over K (a weight gradient's bias gradient
    ``colsum(dY)``), fused into the main loop, added with fp32 atomics.
    ``gsq`` (``EPI_F32_STORE`` only, fp32 [64], optional): += the sum of squares of the stored values (spread over the
    64 slots) -- a weight gradient's share of the clip's global norm (:meth:`FlatParams.norm_cover`)."""
    ws = cnt = None
    if reduce:
        ws, cnt = split_workspace(M, N, tile, splits, A.device)
    if CHECK_BOUNDS:
        _gemm_bounds("iit_gemm_glds", A, B, C, C2, resid, M, N, K, lda, ldb, ldc, ldc2, ldr, mode)
        _bounds("iit_gemm_glds", ("csum", csum, 1, N, N))
    sm = GLDS_STORE_MODE if store_mode is None else store_mode
    _check(lib().iit_gemm_glds_sm(_p(A), _p(B), _p(C), _p(C2), _p(bias0), _p(bias1), _p(bias2), _p(resid), lda, ldb,
                                  ldc, ldc2, ldr, M, N, K, mode, epi, bias_cols, tile, splits, _p(csum), _p(ws),
                                  _p(cnt), int(sm), _p(bsum) if mode == 3 else None,
                                  _p(gsq) if epi == EPI_F32_STORE else None, _stream()),
           "iit_gemm_glds")


# ------------------------------------------------------------------------------ dual GEMM (csrc/gemm_dual.hip)
# one launch runs a layer's weight gradient dW = X^T dY (mode 3; fp32 store / accumulate, optional K-split) and its
# input gradient dX = dY W^T (mode 0; bf16 or the fused dgelu epilogue), two workgroups per CU
# three families (a launch takes both tiles from one): 4-wave tiles, two workgroups per CU (W 0-4, X 0-3); 8-wave
# tiles, one per CU (W 5-6, X 4-6); 4-wave tiles, one per CU with 3-4 deep rings (W 7-8, X 7-8)
DUAL_W_TILES = {0: (128, 96), 1: (128, 128), 2: (96, 96), 3: (64, 96), 4: (64, 64),
                5: (256, 128), 6: (128, 128), 7: (128, 128), 8: (128, 96)}
DUAL_X_TILES = {0: (128, 96), 1: (64, 96), 2: (128, 192), 3: (128, 128),
                4: (256, 192), 5: (256, 128), 6: (128, 128), 7: (128, 128), 8: (128, 192)}


def _dual_family(t: int, first_big: int) -> int:
    return 2 if t >= 7 else (1 if t >= first_big else 0)


def dual_family_ok(wtile: int, xtile: int) -> bool:
    return _dual_family(wtile, 5) == _dual_family(xtile, 4)


def _bf16_cuda(*ts) -> bool:
    return all(t is not None and t.is_cuda and t.dtype == torch.bfloat16 for t in ts)


def gemm_dual_ok(w: dict, x: dict, wtile: int, xtile: int, splits: int = 1, reduce: bool = False) -> bool:
    """Whether :func:`gemm_dual` covers the pair.  ``w``: A (X [T][K_in]), B (dY [T][N]), C (fp32), M, N, K, lda, ldb,
    ldc, epi (EPI_F32_STORE / EPI_F32_ACC); ``x``: A (dY), B (W [K_in][N] as [N][K]), C (bf16), C2 (the saved
    pre-activation for EPI_DGELU), M, N, K, lda, ldb, ldc, ldc2, epi (EPI_BF16 / EPI_DGELU)."""
    if not _bf16_cuda(w["A"], w["B"], x["A"], x["B"]):
        return False
    return bool(lib().iit_gemm_dual_ok(
        _p(w["A"]), _p(w["B"]), _p(w["C"]), w["lda"], w["ldb"], w["ldc"], w["M"], w["N"], w["K"], w["epi"], wtile,
        splits, int(reduce), _p(x["A"]), _p(x["B"]), _p(x["C"]), _p(x.get("C2")), x["lda"], x["ldb"], x["ldc"],
        x.get("ldc2", 0), x["M"], x["N"], x["K"], x["epi"], xtile))


def gemm_dual(w: dict, x: dict, wtile: int, xtile: int, splits: int = 1, reduce: bool = False,
              prefetch=None) -> None:
    """Both problems of :func:`gemm_dual_ok` in one launch (``x["csum"]``: the DGELU column sums, ``w["bsum"]``: the
    column sums of dY over the tokens, i.e. the bias gradient; both optional, += atomically).  ``prefetch``: up to two
    tensors (the next pair's cold operands) that extra workgroups of the launch read into the caches."""
    ws = cnt = None
    if reduce:
        ws, cnt = split_workspace(w["M"], w["N"], DUAL_W_TILES[wtile], splits, w["A"].device)
    if CHECK_BOUNDS:
        _gemm_bounds("iit_gemm_dual(dW)", w["A"], w["B"], w["C"], None, None, w["M"], w["N"], w["K"], w["lda"],
                     w["ldb"], w["ldc"], 0, 0, MODE_AKM | MODE_BKM)
        _gemm_bounds("iit_gemm_dual(dX)", x["A"], x["B"], x["C"], x.get("C2"), None, x["M"], x["N"], x["K"],
                     x["lda"], x["ldb"], x["ldc"], x.get("ldc2", 0), 0, MODE_NN)
        _bounds("iit_gemm_dual", ("csum", x.get("csum"), 1, x["N"], x["N"]))
    _check(lib().iit_gemm_dual(
        _p(w["A"]), _p(w["B"]), _p(w["C"]), w["lda"], w["ldb"], w["ldc"], w["M"], w["N"], w["K"], w["epi"], wtile,
        splits, _p(ws), _p(cnt), _p(x["A"]), _p(x["B"]), _p(x["C"]), _p(x.get("C2")), x["lda"], x["ldb"], x["ldc"],
        x.get("ldc2", 0), x["M"], x["N"], x["K"], x["epi"], xtile, _p(x.get("csum")), _p(w.get("bsum")),
        _p(w.get("gsq")) if w["epi"] == EPI_F32_STORE else None, *_prefetch_args(prefetch), _stream()),
        "iit_gemm_dual")


# workgroups of a dual launch that prefetch the next pair's cold operands, per MiB of them (IIT_DUAL_PREFETCH_WGS_PER_MB;
# 0 disables the prefetch).  Headline step, same box: off 15.58-15.65, 4/MiB 15.46-15.49, 8/MiB 15.44-15.47, 16/MiB
# 15.43, 32/MiB 15.48-15.51 ms (profiles/dual_l2_hypothesis_r6.txt)
_PF_PER_MB = float(os.environ.get("IIT_DUAL_PREFETCH_WGS_PER_MB", "16"))


def _prefetch_args(prefetch):
    ts = [t for t in (prefetch or ()) if t is not None and t.is_cuda and t.is_contiguous()][:2]
    if not ts or _PF_PER_MB <= 0:
        return (None, 0, None, 0, 0)
    ts += [None] * (2 - len(ts))
    nb = [t.numel() * t.element_size() if t is not None else 0 for t in ts]
    wgs = max(8, min(1024, int(sum(nb) / 2 ** 20 * _PF_PER_MB)))
    return (_p(ts[0]), nb[0], _p(ts[1]), nb[1], wgs)


def kl_rows(a, b):
    """Per-row statistics of an LL output ``a`` [R, V] against an HL pmf ``b`` [R, V] (fp32, unit column stride):
    [R, 4] = (sum a, logsumexp a, sum b a, sum_{b > 0} b log a), one pass over both (csrc/kernels.hip)."""
    R, V = a.shape
    out = torch.empty(R, 4, dtype=torch.float32, device=a.device)
    if CHECK_BOUNDS:
        _bounds("kl_rows", ("a", a, R, V, a.stride(0)), ("b", b, R, V, b.stride(0)))
    _check(lib().iit_kl_rows(_p(a), a.stride(0), _p(b), b.stride(0), R, V, _p(out), _stream()), "kl_rows")
    return out


# Adam span length (float4 groups per span record): the kernel runs one workgroup per span (IIT_ADAM_MAX_BLOCKS
# default, csrc/kernels.hip), so this is also its per-workgroup work unit; IIT_ADAM_SPAN4 overrides
_ADAM_SPAN4 = int(os.environ.get("IIT_ADAM_SPAN4", "1024"))


def sumsq_2d(c, ldc: int, M: int, N: int, gsq) -> None:
    """gsq[slot] += sum of squares of the fp32 [M][N] matrix ``c`` (row stride ``ldc``)."""
    if CHECK_BOUNDS:
        _bounds("sumsq_2d", ("c", c, M, N, ldc))
    _check(lib().iit_sumsq_2d(_p(c), ldc, M, N, _p(gsq), _stream()), "sumsq_2d")


def sumsq_spans(g, spans, nspans, part, step_dev, do_norm: bool):
    """Sharded optimizer stage 1: per-block partial sums of g^2 over ``spans`` into ``part`` (1024 floats) and the
    device step-counter bump."""
    _check(lib().iit_sumsq_spans(_p(g), _p(spans), nspans, _p(part), part.numel(), int(do_norm), _p(step_dev),
                                 _stream()), "sumsq_spans")


def adam_spans(flat, g, m, v, spans, nspans, total, step_dev, *, lr, b1, b2, eps, wd, clip_norm, skipped=None,
               hyper=None):
    """Sharded optimizer stage 2: fused clip + Adam over ``spans`` (arena offsets for weights / mirror, shard offsets
    for gradient / moments) with the global g^2 sum in ``total`` (fp32[1])."""
    _check(lib().iit_adam_spans(_p(flat.data), _p(g), _p(m), _p(v), _p(flat.shadow), _p(spans), nspans, _p(total),
                                float(clip_norm or 0.0), lr, b1, b2, eps, wd, _p(hyper), _p(step_dev), _p(skipped),
                                _stream()), "adam_spans")


# ------------------------------------------------------------------------------ others
def splice(act, src, out, n, spec_ptr, f32, mode, scale=1.0):
    """``csrc/splice.hip``: out = splice / zero-mask / scale of ``act`` over the packed range table at host address
    ``spec_ptr`` (see :mod:`iit_amd.ops.splice`); act / out contiguous with ``n`` elements."""
    if CHECK_BOUNDS:
        _bounds("iit_splice", ("act", act, 1, n, n), ("out", out, 1, n, n))
    _check(lib().iit_splice(_p(act), _p(src), _p(out), n, spec_ptr, int(f32), int(mode), float(scale), _stream()),
           "iit_splice")


def embed_pos_fwd(tokens, W_E, W_pos, out, B, S, d):
    _check(lib().iit_embed_pos_fwd(_p(tokens), _p(W_E), _p(W_pos), _p(out), B * S, S, d, _stream()), "embed_pos_fwd")


def embed_pos_bwd(tokens, g, dWE, dWpos, B, S, d):
    _check(lib().iit_embed_pos_bwd(_p(tokens), _p(g), _p(dWE), _p(dWpos), B, S, d, _stream()), "embed_pos_bwd")


def ln_fwd(x, w, b, y, mean, rstd, T, d, eps):
    if CHECK_BOUNDS:
        _bounds("ln_fwd", ("x", x, T, d, d), ("y", y, T, d, d), ("mean", mean, 1, T, T), ("rstd", rstd, 1, T, T))
    _check(lib().iit_ln_fwd(_p(x), _p(w), _p(b), _p(y), _p(mean), _p(rstd), T, d, eps, _stream()), "ln_fwd")


def ln_fwd_twin(x, w, b, y, y32, mean, rstd, T, d, eps) -> bool:
    """``ln_fwd`` that also writes ``y32`` = fp32(y) in the same pass; False when the vector layout does not apply
    (nothing launched: the caller casts)."""
    if CHECK_BOUNDS:
        _bounds("ln_fwd_twin", ("x", x, T, d, d), ("y", y, T, d, d), ("y32", y32, T, d, d))
    return lib().iit_ln_fwd_twin(_p(x), _p(w), _p(b), _p(y), _p(y32), _p(mean), _p(rstd), T, d, eps, _stream()) == 0


def _ln_part(dw, T: int, d: int):
    """Scratch of the fused affine-gradient LN backward (``iit_ln_bwd_part``): one (dw, db) partial row pair per
    block of ``iit_ln_bwd_part_rows()`` rows; None without affine gradients or with ``IIT_LN_FUSED_DWDB=0``."""
    if dw is None or os.environ.get("IIT_LN_FUSED_DWDB", "1") == "0":
        return None
    rows = _LN_PART_ROWS[0] or lib().iit_ln_bwd_part_rows()
    _LN_PART_ROWS[0] = rows
    return torch.empty(((T + rows - 1) // rows) * 2 * d, dtype=torch.float32, device=dw.device)


_LN_PART_ROWS = [0]


def ln_bwd(dy, x, mean, rstd, w, dx, dw, db, T, d, accumulate=False, dres=None, dx16=None, dy2=None):
    """dx = LN'(dy) (+ dres, the skip-connection gradient, fp32 [T, d]); ``dx16`` (optional) gets a bf16 copy; with
    ``dw`` / ``db`` the affine gradients are added in the same pass (``iit_ln_bwd_part``); ``dy2`` (fp32 [T, d],
    optional) is a second gradient of the output, added to ``dy`` inside the kernel where it can be."""
    if CHECK_BOUNDS:
        _bounds("ln_bwd", ("dy", dy, T, d, d), ("x", x, T, d, d), ("dx", dx, T, d, d), ("dres", dres, T, d, d),
                ("dx16", dx16, T, d, d), ("mean", mean, 1, T, T), ("dy2", dy2, T, d, d))
    part = _ln_part(dw, T, d)
    if part is not None:
        rc = lib().iit_ln_bwd_part(_p(dy), int(dy.dtype == torch.float32), _p(x), _p(mean), _p(rstd), _p(w),
                                   _p(dx), _p(dres), _p(dx16), _p(dw), _p(db), _p(part), T, d, int(accumulate), 0,
                                   1, _p(dy2), _stream())
        if rc == 0 or dy2 is None:
            _check(rc, "ln_bwd_part")
            return
    if dy2 is not None:  # (no fused path: sum the two gradients first)
        dy = dy.float() + dy2
    _check(lib().iit_ln_bwd(_p(dy), int(dy.dtype == torch.float32), _p(x), _p(mean), _p(rstd), _p(w), _p(dx),
                            _p(dres), _p(dx16), _p(dw), _p(db), T, d, int(accumulate), _stream()), "ln_bwd")


def ln_bwd_xh16(dy, xh, rstd, dx, T, d, dres=None, dx16=None):
    """LNPre backward from the forward's bf16 output ``xh`` (= xhat; 2 B per element instead of the fp32 input)."""
    if CHECK_BOUNDS:
        _bounds("ln_bwd_xh16", ("dy", dy, T, d, d), ("xh", xh, T, d, d), ("dx", dx, T, d, d), ("dres", dres, T, d, d),
                ("dx16", dx16, T, d, d), ("rstd", rstd, 1, T, T))
    assert xh.dtype == torch.bfloat16
    _check(lib().iit_ln_bwd_xh16(_p(dy), int(dy.dtype == torch.float32), _p(xh), _p(rstd), _p(dx), _p(dres),
                                 _p(dx16), T, d, 0, _stream()), "ln_bwd_xh16")


def ln_fwd_sel(x, w, b, y, mean, rstd, T, d, eps, pos_mask: int, S: int, Tb: int):
    """``ln_fwd`` over paired rows with the whole-position splice inside the kernel: base rows [0, Tb) at positions
    whose bit is set in ``pos_mask`` normalise the source row ``row + Tb`` (csrc/kernels.hip RowSel)."""
    if CHECK_BOUNDS:
        _bounds("ln_fwd_sel", ("x", x, T, d, d), ("y", y, T, d, d), ("mean", mean, 1, T, T), ("rstd", rstd, 1, T, T))
    _check(lib().iit_ln_fwd_sel(_p(x), _p(w), _p(b), _p(y), _p(mean), _p(rstd), T, d, eps, pos_mask, S, Tb, _stream()), "ln_fwd_sel")


def ln_bwd_sel(dy, x, mean, rstd, w, dx, dw, db, T, d, pos_mask: int, S: int, dres=None, dx16=None):
    """Backward of :func:`ln_fwd_sel` over the base rows: spliced rows pass only ``dres`` and add nothing to dw/db."""
    if CHECK_BOUNDS:
        _bounds("ln_bwd_sel", ("dy", dy, T, d, d), ("x", x, T, d, d), ("dx", dx, T, d, d), ("mean", mean, 1, T, T))
    part = _ln_part(dw, T, d)
    if part is not None:
        _check(lib().iit_ln_bwd_part(_p(dy), int(dy.dtype == torch.float32), _p(x), _p(mean), _p(rstd), _p(w),
                                     _p(dx), _p(dres), _p(dx16), _p(dw), _p(db), _p(part), T, d, 0, pos_mask, S,
                                     None, _stream()), "ln_bwd_sel_part")
        return
    _check(lib().iit_ln_bwd_sel(_p(dy), int(dy.dtype == torch.float32), _p(x), _p(mean), _p(rstd), _p(w), _p(dx),
                                _p(dres), _p(dx16), _p(dw), _p(db), T, d, 0, pos_mask, S,
                                _stream()), "ln_bwd_sel")


def heads_to_mask(heads: Optional[Sequence[int]]) -> int:
    m = 0
    for h in heads or ():
        m |= 1 << int(h)
    return m


def _mfma_attn(S, dh):
    return S <= 16 and dh in (32, 64, 96, 128) and os.environ.get("IIT_ATTN", "mfma") == "mfma"


def attn_small_fwd(qkv, z, lse, zsrc, head_mask, B, S, H, dh, ld_qkv, ld_z, ld_src, scale, causal):
    """Causal attention for S <= 64 (MFMA one-wave-per-head kernel when S <= 16, csrc/attn_mfma.hip)."""
    if CHECK_BOUNDS:
        _bounds("attn_fwd", ("qkv", qkv, B * S, 3 * H * dh, ld_qkv), ("z", z, B * S, H * dh, ld_z),
                ("zsrc", zsrc, B * S, H * dh, ld_src), ("lse", lse, 1, B * H * S, B * H * S))
    if _mfma_attn(S, dh):
        _check(lib().iit_attn_mfma_fwd(_p(qkv), _p(z), _p(lse), _p(zsrc), head_mask, B, S, H, dh, ld_qkv, ld_z, ld_src,
                                       scale, int(causal), _stream()), "attn_mfma_fwd")
        return
    _check(lib().iit_attn_small_fwd(_p(qkv), _p(z), _p(lse), _p(zsrc), head_mask, B, S, H, dh, ld_qkv, ld_z, ld_src,
                                    scale, int(causal), _stream()), "attn_small_fwd")


def attn_pair_ok(S, dh) -> bool:
    """Whether the paired-row options (dual store, mirrored heads) of the MFMA attention kernel apply."""
    return _mfma_attn(S, dh)


def attn_pair_fwd(qkv, z, lse, B, S, H, dh, ld_qkv, ld_z, scale, causal, z2=None, pair_seqs=0, pair_mask=0):
    """MFMA short-sequence attention with ``z2`` (a second copy of z) and / or paired rows: the first ``pair_seqs``
    of the ``B`` sequences are base rows whose heads in ``pair_mask`` take the z of the sequence ``pair_seqs`` later
    (computed once, stored twice; see csrc/attn_mfma.hip)."""
    if not _mfma_attn(S, dh):
        raise RuntimeError("attn_pair_fwd needs the MFMA short-sequence kernel (S <= 16, dh in 32/64/96/128)")
    if CHECK_BOUNDS:
        _bounds("attn_pair_fwd", ("qkv", qkv, B * S, 3 * H * dh, ld_qkv), ("z", z, B * S, H * dh, ld_z),
                ("z2", z2, B * S, H * dh, ld_z), ("lse", lse, 1, B * H * S, B * H * S))
    _check(lib().iit_attn_mfma_fwd_pair(_p(qkv), _p(z), _p(lse), None, 0, B, S, H, dh, ld_qkv, ld_z, 0, scale,
                                        int(causal), _p(z2), pair_seqs, pair_mask, _stream()), "attn_mfma_fwd_pair")


def attn_pair_fwd_spec(qkv, z, lse, B, S, H, dh, ld_qkv, ld_z, scale, causal, pair_seqs, spec_ptr):
    """Paired-row MFMA attention with a general ``hook_z`` splice (patch spec over the base rows' [B/2, S, H, dh] z at
    host address ``spec_ptr``) applied in the kernel's store: the source rows' selected elements go to the base rows
    (csrc/attn_mfma.hip)."""
    if not _mfma_attn(S, dh):
        raise RuntimeError("attn_pair_fwd_spec needs the MFMA short-sequence kernel (S <= 16, dh in 32/64/96/128)")
    if CHECK_BOUNDS:
        _bounds("attn_pair_fwd_spec", ("qkv", qkv, B * S, 3 * H * dh, ld_qkv), ("z", z, B * S, H * dh, ld_z),
                ("lse", lse, 1, B * H * S, B * H * S))
    _check(lib().iit_attn_mfma_fwd_spec(_p(qkv), _p(z), _p(lse), B, S, H, dh, ld_qkv, ld_z, scale, int(causal),
                                        pair_seqs, spec_ptr, _stream()), "attn_mfma_fwd_spec")


def attn_bwd_spec(qkv, dz, lse, dqkv, B, S, H, dh, ld_qkv, ld_dz, scale, causal, spec_ptr):
    """The base rows' attention backward with the spliced elements of ``dz`` zeroed in the kernel."""
    if CHECK_BOUNDS:
        _bounds("attn_bwd_spec", ("qkv", qkv, B * S, 3 * H * dh, ld_qkv), ("dz", dz, B * S, H * dh, ld_dz),
                ("dqkv", dqkv, B * S, 3 * H * dh, ld_qkv))
    _check(lib().iit_attn_mfma_bwd_spec(_p(qkv), _p(dz), _p(lse), _p(dqkv), B, S, H, dh, ld_qkv, ld_dz, scale,
                                        int(causal), spec_ptr, _stream()), "attn_mfma_bwd_spec")


def attn_small_bwd(qkv, dz, lse, dqkv, head_mask, B, S, H, dh, ld_qkv, ld_dz, scale, causal):
    if CHECK_BOUNDS:
        _bounds("attn_bwd", ("qkv", qkv, B * S, 3 * H * dh, ld_qkv), ("dz", dz, B * S, H * dh, ld_dz),
                ("dqkv", dqkv, B * S, 3 * H * dh, ld_qkv))
    if _mfma_attn(S, dh):
        _check(lib().iit_attn_mfma_bwd(_p(qkv), _p(dz), _p(lse), _p(dqkv), head_mask, B, S, H, dh, ld_qkv, ld_dz, scale,
                                       int(causal), _stream()), "attn_mfma_bwd")
        return
    _check(lib().iit_attn_small_bwd(_p(qkv), _p(dz), _p(lse), _p(dqkv), head_mask, B, S, H, dh, ld_qkv, ld_dz, scale,
                                    int(causal), _stream()), "attn_small_bwd")


def _bsh(t: torch.Tensor):
    """(batch, position, head) element strides of a [B, S, H, dh] view with unit stride on dh."""
    assert t.stride(-1) == 1 and t.dtype == torch.bfloat16, "flash attention takes bf16 [B,S,H,dh] with unit d stride"
    return [t.stride(0), t.stride(1), t.stride(2)]


def _longs(vals):
    return (c_long * len(vals))(*vals)


def flash_fwd(q, k, v, z, lse, src, head_mask: int, scale: float, causal: bool, spec=None):
    """Tiled attention forward (csrc/flash_attn.hip): q/z [B,S,Hq,dh], k/v [B,S,Hkv,dh], lse [B,Hq,S] fp32.
    ``spec`` (a :class:`iit_amd.ops.splice.PatchSpec` over z's [B,S,Hq,dh] with ``src``'s strides): general splice of
    the output, applied by the output store (replaces ``head_mask``)."""
    B, S, Hq, dh = q.shape
    Hkv = k.shape[2]
    st = _longs(_bsh(q) + _bsh(k) + _bsh(v))
    zs = _longs(_bsh(z))
    ss = _longs(_bsh(src)) if (src is not None and spec is None) else None
    _check(lib().iit_flash_fwd(_p(q), _p(k), _p(v), ctypes.cast(st, c_void_p), _p(z), ctypes.cast(zs, c_void_p),
                               _p(lse), _p(src), None if ss is None else ctypes.cast(ss, c_void_p),
                               head_mask if src is not None else 0, B, S, Hq, Hkv, dh, scale, int(causal),
                               None if spec is None else spec.ptr, _stream()),
           "flash_fwd")


def flash_bwd(q, k, v, z, dz, lse, dd, dq, dk, dv, head_mask: int, scale: float, causal: bool, spec=None):
    B, S, Hq, dh = q.shape
    Hkv = k.shape[2]
    st = _longs(_bsh(q) + _bsh(k) + _bsh(v))
    gs = _longs(_bsh(dq) + _bsh(dk) + _bsh(dv))
    zs, ds = _longs(_bsh(z)), _longs(_bsh(dz))
    _check(lib().iit_flash_bwd(_p(q), _p(k), _p(v), ctypes.cast(st, c_void_p), _p(z), ctypes.cast(zs, c_void_p),
                               _p(dz), ctypes.cast(ds, c_void_p), _p(lse), _p(dd), _p(dq), _p(dk), _p(dv),
                               ctypes.cast(gs, c_void_p), head_mask, B, S, Hq, Hkv, dh, scale, int(causal),
                               None if spec is None else spec.ptr, _stream()),
           "flash_bwd")


def bn_ws_floats(C: int) -> int:
    """Length of the fused BatchNorm's self-re-arming accumulator for C channels (csrc/bn_nhwc.hip)."""
    return int(lib().iit_bn_ws_floats(C))


def maxpool3s2_fwd(x, y, idx, N: int, H: int, W: int, C: int):
    """3x3 / stride 2 / padding 1 max pool of channels-last bf16 ``x`` [N, C, H, W] into ``y``; ``idx``: uint8 argmax
    tap per output element (csrc/bn_nhwc.hip)."""
    if CHECK_BOUNDS:
        OH, OW = (H - 1) // 2 + 1, (W - 1) // 2 + 1
        assert y.numel() == N * OH * OW * C and idx.numel() == y.numel() and x.numel() == N * H * W * C
    _check(lib().iit_maxpool3s2_fwd(_p(x), _p(y), _p(idx), N, H, W, C, int(x.dtype == torch.float32), _stream()),
           "maxpool3s2_fwd")


# ------------------------------------------------------------------------------ implicit-GEMM conv (csrc/conv_nhwc.hip)
_ZERO_PAGE = {}


def zero_page(device) -> torch.Tensor:
    """>= 128 zero bytes on ``device`` (16-B aligned): the LDS-DMA source of the convolution's padding rows."""
    key = str(device)
    z = _ZERO_PAGE.get(key)
    if z is None:
        z = _ZERO_PAGE[key] = torch.zeros(256, dtype=torch.bfloat16, device=device)
    return z


def conv3x3_tiles() -> int:
    return int(lib().iit_conv3x3_tiles())


def conv3x3_ok(N: int, H: int, W: int, Cin: int, Cout: int, tile: int, splits: int = 1) -> bool:
    return bool(lib().iit_conv3x3_ok(N, H, W, Cin, Cout, tile, splits))


CONV_TILES = {0: (128, 64), 1: (128, 128), 2: (64, 64), 3: (128, 128), 4: (64, 128), 5: (128, 64)}


def conv3x3_rows(tile: int) -> int:
    """Output rows per tile (BM) of forward tile ``tile``: the row-tile size of the ``cstat`` records."""
    return CONV_TILES[tile][0]


def conv3x3(x, w, y, N: int, H: int, W: int, Cin: int, Cout: int, flip: bool = False, tile: int = 0,
            splits: int = 1, cstat=None):
    """``y`` [N,H,W,Cout] = 3x3 / stride-1 / pad-1 convolution of the NHWC bf16 ``x`` [N,H,W,Cin] with ``w``
    [Cout,3,3,Cin] (``flip``: the input gradient -- ``x`` = dy [N,H,W,Cout'], ``w`` the forward weight [Cout',3,3,Cin'],
    output channels ``Cout`` = Cin');
    ``splits`` > 1: deterministic reduction split over the 9 Cin reduction.  ``cstat`` (fp32, >= 3 Cout T floats,
    T = N H W / :func:`conv3x3_rows`): per-tile column statistics of ``y`` for :func:`bn_fwd_tiles`."""
    ws = cnt = None
    if splits > 1:
        ws, cnt = split_workspace(N * H * W, Cout, CONV_TILES[tile], splits, x.device)
    if CHECK_BOUNDS:
        assert x.numel() >= N * H * W * Cin and y.numel() >= N * H * W * Cout and w.numel() >= 9 * Cin * Cout
        assert x.dtype == w.dtype == y.dtype == torch.bfloat16
        if cstat is not None:
            assert cstat.dtype == torch.float32 and cstat.numel() >= 3 * Cout * (N * H * W // conv3x3_rows(tile))
    _check(lib().iit_conv3x3(_p(x), _p(w), _p(y), _p(zero_page(x.device)), N, H, W, Cin, Cout, int(flip), tile,
                             splits, _p(ws), _p(cnt), _p(cstat), _stream()), "conv3x3")


def conv2d_ok(N: int, SH: int, SW: int, Cs: int, OH: int, OW: int, Co: int, k: int, s: int, pad: int,
              transposed: bool, tile: int, splits: int = 1) -> bool:
    return bool(lib().iit_conv2d_ok(N, SH, SW, Cs, OH, OW, Co, k, s, pad, int(transposed), tile, splits))


def conv2d(x, w, y, N: int, SH: int, SW: int, Cs: int, OH: int, OW: int, Co: int, k: int, s: int, pad: int,
           transposed: bool, tile: int = 0, splits: int = 1, cstat=None):
    """Implicit-GEMM convolution (csrc/conv_nhwc.hip): forward ``y`` [N,OH,OW,Co] = conv(``x`` [N,SH,SW,Cs], ``w``
    [Co,k,k,Cs], stride ``s``, padding ``pad``), or (``transposed``) the input gradient of a forward conv from
    [OH,OW,Co] to [SH,SW,Cs]: ``x`` = dy, ``w`` the FORWARD weight [Cs = Cout][k][k][Co = Cin] (``transposed`` = 1 or
    True; read k-major in place) or its re-laid copy [Co = Cin][k][k][Cs = Cout] (``transposed`` = 2), ``y`` = dx."""
    ws = cnt = None
    if splits > 1:
        ws, cnt = split_workspace(N * OH * OW, Co, CONV_TILES[tile], splits, x.device)
    if CHECK_BOUNDS:
        assert x.numel() >= N * SH * SW * Cs and y.numel() >= N * OH * OW * Co and w.numel() >= k * k * Cs * Co
        assert x.dtype == w.dtype == y.dtype == torch.bfloat16
        if cstat is not None:
            assert cstat.dtype == torch.float32 and cstat.numel() >= 3 * Co * (N * OH * OW // conv3x3_rows(tile))
    _check(lib().iit_conv2d(_p(x), _p(w), _p(y), _p(zero_page(x.device)), N, SH, SW, Cs, OH, OW, Co, k, s, pad,
                            int(transposed), tile, splits, _p(ws), _p(cnt), _p(cstat), _stream()), "conv2d")


def conv2d_wgrad_ok(N: int, SH: int, SW: int, Cin: int, OH: int, OW: int, Cout: int, k: int, s: int, pad: int,
                    tile: int, splits: int) -> bool:
    return bool(lib().iit_conv2d_wgrad_ok(N, SH, SW, Cin, OH, OW, Cout, k, s, pad, tile, splits))


def conv2d_wgrad(dy, x, dw, N: int, SH: int, SW: int, Cin: int, OH: int, OW: int, Cout: int, k: int, s: int,
                 pad: int, acc: bool, tile: int, splits: int = 1):
    """``dw`` [Cout,k,k,Cin] fp32 (+)= the weight gradient of the conv ``x`` [N,SH,SW,Cin] -> ``dy`` [N,OH,OW,Cout];
    ``splits`` > 1: deterministic reduction split over the output pixels."""
    ws = cnt = None
    if splits > 1:
        ws, cnt = split_workspace(Cout, k * k * Cin, CONV_WG_TILES[tile], splits, dy.device)
    if CHECK_BOUNDS:
        assert dw.dtype == torch.float32 and dw.numel() >= k * k * Cin * Cout
        assert dy.numel() >= N * OH * OW * Cout and x.numel() >= N * SH * SW * Cin
    _check(lib().iit_conv2d_wgrad(_p(dy), _p(x), _p(dw), _p(zero_page(x.device)), N, SH, SW, Cin, OH, OW, Cout, k, s,
                                  pad, int(acc), tile, splits, _p(ws), _p(cnt), _stream()), "conv2d_wgrad")


CONV_WG_TILES = {0: (64, 64), 1: (128, 64), 2: (128, 128), 3: (64, 128)}


def conv3x3_wgrad_splits(pixels: int) -> list:
    """K-split candidates of a weight gradient over ``pixels`` (a multiple of 64): for each target 1, 2, 4, ..., 64
    the largest divisor of the K-tile count not above it (the reduction split needs equal K ranges)."""
    nkt = pixels // 64
    out = []
    for target in (1, 2, 4, 8, 16, 32, 64):
        d = max(x for x in range(1, target + 1) if nkt % x == 0)
        if d not in out:
            out.append(d)
    return out


def conv3x3_wgrad_ok(N: int, H: int, W: int, Cin: int, Cout: int, tile: int, splits: int) -> bool:
    return bool(lib().iit_conv3x3_wgrad_ok(N, H, W, Cin, Cout, tile, splits))


def conv3x3_wgrad(dy, x, dw, N: int, H: int, W: int, Cin: int, Cout: int, acc: bool, tile: int, splits: int = 1):
    """``dw`` [Cout,3,3,Cin] fp32 (+)= the weight gradient of the 3x3 / stride-1 / pad-1 convolution (NHWC bf16 ``dy``
    [N,H,W,Cout], ``x`` [N,H,W,Cin]); ``splits`` > 1: deterministic reduction split over the pixels."""
    ws = cnt = None
    if splits > 1:
        ws, cnt = split_workspace(Cout, 9 * Cin, CONV_WG_TILES[tile], splits, dy.device)
    if CHECK_BOUNDS:
        assert dw.dtype == torch.float32 and dw.numel() >= 9 * Cin * Cout
        assert dy.numel() >= N * H * W * Cout and x.numel() >= N * H * W * Cin
    _check(lib().iit_conv3x3_wgrad(_p(dy), _p(x), _p(dw), _p(zero_page(x.device)), N, H, W, Cin, Cout, int(acc), tile,
                                   splits, _p(ws), _p(cnt), _stream()), "conv3x3_wgrad")


def maxpool3s2_bwd(dy, idx, dx, N: int, H: int, W: int, C: int):
    _check(lib().iit_maxpool3s2_bwd(_p(dy), _p(idx), _p(dx), N, H, W, C, int(dy.dtype == torch.float32), _stream()),
           "maxpool3s2_bwd")


def bn_two_level() -> bool:
    """The BatchNorm statistics' fixed-order two-level reduction (bit-identical run to run) instead of the faster
    fp32-atomic one: in deterministic mode (``IIT_DETERMINISTIC=1`` / ``torch.use_deterministic_algorithms``) or with
    ``IIT_BN_REDUCE=two``."""
    if os.environ.get("IIT_BN_REDUCE", "") == "two":
        return True
    return os.environ.get("IIT_DETERMINISTIC", "0") == "1" or torch.are_deterministic_algorithms_enabled()


def bn_fwd(x, res, y, ws, rmean, rvar, w, b, M: int, C: int, eps: float, relu: bool, training: bool, save,
           momentum: float, nbt, src=None, spec=None, H: int = 0, W: int = 0):
    """Fused BatchNorm (+ residual) (+ ReLU) forward over NHWC bf16 or fp32 rows (csrc/bn_nhwc.hip; every activation
    of one call has ``x``'s dtype); ``ws`` = the module's self-re-arming accumulator (:func:`bn_ws_floats`)."""
    if CHECK_BOUNDS:
        for t in (x, y) + ((res,) if res is not None else ()):
            assert _avail(t) >= M * C and t.dtype == x.dtype, "bn_fwd: activation smaller than M x C / dtype"
        assert ws.numel() >= bn_ws_floats(C) and save.numel() >= 2 * C
    _check(lib().iit_bn_fwd(_p(x), _p(res), _p(y), _p(ws), _p(rmean), _p(rvar), _p(w), _p(b), M, C, eps, int(relu),
                            int(training), _p(save), momentum, _p(nbt), _p(src), None if spec is None else spec.ptr,
                            H, W, int(x.dtype == torch.float32), int(bn_two_level()), _stream()), "bn_fwd")


def bn_fwd_tiles(x, res, y, cstat, T: int, R: int, rmean, rvar, w, b, M: int, C: int, eps: float, relu: bool, save,
                 momentum: float, nbt):
    """Training forward of :func:`bn_fwd` on a bf16 ``x`` whose statistics its producing convolution's epilogue wrote
    (``cstat``: T row tiles of R rows, :func:`conv3x3`): a per-channel combine of the tile records, then the apply
    pass -- no statistics pass over ``x``."""
    if CHECK_BOUNDS:
        for t in (x, y) + ((res,) if res is not None else ()):
            assert _avail(t) >= M * C and t.dtype == torch.bfloat16, "bn_fwd_tiles: activation smaller than M x C"
        assert T * R == M and cstat.numel() >= 3 * C * T and save.numel() >= 2 * C
    _check(lib().iit_bn_fwd_tiles(_p(x), _p(res), _p(y), _p(cstat), T, R, _p(rmean), _p(rvar), _p(w), _p(b), M, C,
                                  eps, int(relu), _p(save), momentum, _p(nbt), _stream()), "bn_fwd_tiles")


def bn_bwd(dy, y, x, save, w, ws, coef, M: int, C: int, training: bool, dx, dres, dw, db, src=None, spec=None,
           H: int = 0, W: int = 0):
    """Backward of :func:`bn_fwd`; ``dw`` / ``db`` (fp32 [C], nullable) are accumulated into."""
    if CHECK_BOUNDS:
        for t in (dy, x, dx):
            assert _avail(t) >= M * C, "bn_bwd: activation smaller than M x C"
    _check(lib().iit_bn_bwd(_p(dy), _p(y), _p(x), _p(save), _p(w), _p(ws), _p(coef), M, C, int(training), _p(dx),
                            _p(dres), _p(dw), _p(db), _p(src), None if spec is None else spec.ptr, H, W,
                            int(x.dtype == torch.float32), int(bn_two_level()), _stream()), "bn_bwd")


def zero_ranges(base, starts, lens):
    """Zero the element ranges ``[starts[i], starts[i] + lens[i])`` of fp32 ``base``; ``starts`` / ``lens`` are
    host int64 numpy arrays, passed to the kernel by value (capturable: no device table, no host->device copy)."""
    import numpy as np
    starts = np.ascontiguousarray(starts, dtype=np.int64)
    lens = np.ascontiguousarray(lens, dtype=np.int64)
    if CHECK_BOUNDS and len(lens):
        assert int((starts + lens).max()) <= _avail(base) and int(starts.min()) >= 0, "zero_ranges out of bounds"
    _check(lib().iit_zero_ranges(_p(base), starts.ctypes.data, lens.ctypes.data, len(lens), _stream()),
           "zero_ranges")


def zero_chunks(base, chunks, n: int):
    """Zero the (start, len) element ranges listed in the int64 device tensor ``chunks`` of fp32 ``base``."""
    _check(lib().iit_zero_chunks(_p(base), _p(chunks), n, _stream()), "zero_chunks")


def rms_fwd(x, w, y, rstd, T: int, d: int, eps: float):
    _check(lib().iit_rms_fwd(_p(x), int(x.dtype == torch.float32), _p(w), _p(y), _p(rstd), T, d, eps, _stream()),
           "rms_fwd")


def rms_bwd(dy, x, rstd, w, dx, dw, T: int, d: int, dres=None):
    """RMSNorm backward; ``dres`` (optional, x's dtype [T, d]): the skip-connection gradient added into dx."""
    _check(lib().iit_rms_bwd_res(_p(dy), _p(x), int(x.dtype == torch.float32), _p(rstd), _p(w), _p(dx), _p(dres),
                                 _p(dw), T, d, _stream()), "rms_bwd")


def rotary(x, out, cos, sin, rd: int, offset: int, adjacent: bool, inverse: bool):
    """out [B,S,H,D] contiguous = rotary(x) (x any batch/position/head strides, unit d stride), bf16."""
    B, S, H, D = x.shape
    _check(lib().iit_rotary(_p(x), x.stride(0), x.stride(1), x.stride(2), _p(out), _p(cos), _p(sin), int(inverse),
                            B, S, H, D, rd, offset, int(adjacent), _stream()), "rotary")


def swiglu_fwd(gate, up, post):
    _check(lib().iit_swiglu_fwd(_p(gate), _p(up), _p(post), gate.numel(), _stream()), "swiglu_fwd")


def sparse_pair(act, T: int, ld: int, spec_ptr, mode: int) -> None:
    """Sparse paired splice over a [2T][ld] bf16 activation (csrc/splice.hip): mode 0 copies the selected elements of
    the source half into the base half in place, mode 1 zeroes them (one thread per selected element)."""
    if CHECK_BOUNDS:
        _bounds("sparse_pair", ("act", act, 2 * T if mode == 0 else T, ld, ld))
    _check(lib().iit_sparse_pair(_p(act), T, ld, spec_ptr, int(mode), _stream()), "sparse_pair")


def swiglu_splice_fwd(gate, up, post, src, spec_ptr):
    """``post = silu(gate) * up`` with the patch spec at host address ``spec_ptr`` spliced from ``src`` (same
    element order as the spec; see :mod:`iit_amd.ops.splice`)."""
    _check(lib().iit_swiglu_splice_fwd(_p(gate), _p(up), _p(post), _p(src), gate.numel(), spec_ptr, _stream()),
           "swiglu_splice_fwd")


def embed_splice_fwd(tokens, W16, out, src, spec_ptr):
    """``out[t] = W16[tokens[t]]`` (bf16 rows, row stride ``W16.stride(0)``) with the patch spec at host address
    ``spec_ptr`` spliced from ``src`` (csrc/llama_ops.hip)."""
    T, d = tokens.numel(), out.shape[-1]
    if CHECK_BOUNDS:
        _bounds("embed_splice_fwd", ("out", out, T, d, d))
    _check(lib().iit_embed_splice_fwd(_p(tokens), _p(W16), W16.stride(0), _p(out), _p(src), T, d, spec_ptr,
                                      _stream()), "embed_splice_fwd")


def embed_splice_bwd(tokens, dout, grad, spec_ptr):
    """``grad[tokens[t]] += dout[t]`` (fp32 rows) except the spliced elements."""
    T, d = tokens.numel(), dout.shape[-1]
    _check(lib().iit_embed_splice_bwd(_p(tokens), _p(dout), int(dout.dtype == torch.float32), _p(grad),
                                      grad.stride(0), T, d, spec_ptr, _stream()), "embed_splice_bwd")


def swiglu_splice_bwd(dpost, gate, up, dgate, dup, spec_ptr):
    """SwiGLU backward with the spliced elements' gradient zeroed."""
    _check(lib().iit_swiglu_splice_bwd(_p(dpost), _p(gate), _p(up), _p(dgate), _p(dup), gate.numel(), spec_ptr,
                                       _stream()), "swiglu_splice_bwd")


def swiglu_bwd(dpost, gate, up, dgate, dup):
    _check(lib().iit_swiglu_bwd(_p(dpost), _p(gate), _p(up), _p(dgate), _p(dup), gate.numel(), _stream()),
           "swiglu_bwd")


def ce_fwd(logits, ld, labels, loss, lse, amax, R, V):
    if CHECK_BOUNDS:
        _bounds("ce_fwd", ("logits", logits, R, V, ld))
    _check(lib().iit_ce_fwd(_p(logits), ld, _p(labels), _p(loss), _p(lse), _p(amax), R, V, _stream()), "ce_fwd")


def ce_bwd(logits, ld, labels, lse, gscale, inv_rows, out, ld_out, R, V, out16=None):
    """dlogits into ``out`` (fp32 or bf16, row stride ``ld_out``; pad columns zeroed)."""
    if CHECK_BOUNDS:
        _bounds("ce_bwd", ("logits", logits, R, V, ld), ("out", out, R, V, ld_out))
    _check(lib().iit_ce_bwd(_p(logits), ld, _p(labels), _p(lse), _p(gscale), inv_rows, _p(out), ld_out, R, V,
                            int(out.dtype == torch.bfloat16), _p(out16), _stream()), "ce_bwd")


def colsum_accum(x, ld, out, T, N):
    if CHECK_BOUNDS:
        _bounds("colsum", ("x", x, T, N, ld), ("out", out, 1, N, N))
    _check(lib().iit_colsum_accum(_p(x), int(x.dtype == torch.float32), ld, _p(out), T, N, _stream()), "colsum")


def colsum_vec_ok(x, ld, out, N) -> bool:
    """Whether ``colsum_multi`` can take this sum (vector-aligned rows of a bf16 / fp32 operand)."""
    cpt = 4 if x.dtype == torch.float32 else 8
    return (x.dtype in (torch.float32, torch.bfloat16) and out.dtype == torch.float32 and N % cpt == 0
            and ld % cpt == 0 and x.data_ptr() % 16 == 0)


def colsum_multi(items):
    """``out_i[n] += sum_t x_i[t][n]`` for every ``(x, ld, out, T, N)`` in ``items`` -- one launch per 32 sums,
    descriptors passed by value (capturable).  Every item must satisfy :func:`colsum_vec_ok`."""
    import numpy as np
    if not items:
        return
    xs = np.array([it[0].data_ptr() for it in items], dtype=np.int64)
    outs = np.array([it[2].data_ptr() for it in items], dtype=np.int64)
    lds = np.array([it[1] for it in items], dtype=np.int64)
    Ts = np.array([it[3] for it in items], dtype=np.int32)
    Ns = np.array([it[4] for it in items], dtype=np.int32)
    f32s = np.array([int(it[0].dtype == torch.float32) for it in items], dtype=np.int32)
    if CHECK_BOUNDS:
        for x, ld, out, T, N in items:
            _bounds("colsum_multi", ("x", x, T, N, ld), ("out", out, 1, N, N))
    _check(lib().iit_colsum_multi(xs.ctypes.data, outs.ctypes.data, lds.ctypes.data, Ts.ctypes.data, Ns.ctypes.data,
                                  f32s.ctypes.data, len(items), _stream()), "colsum_multi")


def colsum3_accum(x, ld, outs, T, N):
    """outs[i][n] += sum_t x[t][i*N + n] for the packed QKV bias gradients."""
    for i, o in enumerate(outs):
        colsum_accum(x[:, i * N:], ld, o, T, N)


def gelu_fwd(pre, out, M, N, erf=False):
    """out = gelu(pre) (gelu_new, or the exact erf form), bf16 [M, N] views with unit column stride."""
    _check(lib().iit_gelu_fwd(_p(pre), pre.stride(0), _p(out), out.stride(0), M, N, int(erf), _stream()), "gelu_fwd")


def dgelu(dpost, pre, out, erf=False):
    _check(lib().iit_dgelu(_p(dpost), _p(pre), _p(out), dpost.numel(), int(erf), _stream()), "dgelu")


def add_bf16(out, ldo, base, ldb, y, ldy, bias, M, N):
    """out = base + y + bias (fp32 out/base, bf16 y, fp32 bias or None); base may alias out."""
    if CHECK_BOUNDS:
        _bounds("add_bf16", ("out", out, M, N, ldo), ("base", base, M, N, ldb), ("y", y, M, N, ldy))
    _check(lib().iit_add_bf16(_p(out), ldo, _p(base), ldb, _p(y), ldy, _p(bias), M, N, _stream()), "add_bf16")


def shadow_refresh(descs: torch.Tensor, n: int):
    _check(lib().iit_shadow_refresh(_p(descs), n, _stream()), "shadow_refresh")


_SHADOW_DTYPE = np.dtype([("src", np.uint64), ("dst", np.uint64), ("rows", np.int32), ("cols", np.int32),
                          ("ld", np.int64), ("heads", np.int32), ("transpose", np.int32), ("src_hs", np.int64),
                          ("dst_hs", np.int64)])


def make_shadow_descs(entries, device) -> torch.Tensor:
    """entries: (src_ptr, dst_ptr, rows, cols, ld, transpose[, heads, src_head_stride, dst_head_stride])."""
    assert _SHADOW_DTYPE.itemsize == lib().iit_shadow_desc_size()
    arr = np.zeros(len(entries), dtype=_SHADOW_DTYPE)
    for i, e in enumerate(entries):
        src_ptr, dst_ptr, rows, cols, ld, tr = e[:6]
        heads, shs, dhs = (e[6], e[7], e[8]) if len(e) > 6 else (1, 0, 0)
        arr[i] = (src_ptr, dst_ptr, rows, cols, ld, heads, int(tr), shs, dhs)
    return torch.from_numpy(arr.view(np.uint8).copy()).to(device)


def adam_step(flat, exp_avg, exp_avg_sq, step_dev, *, lr, b1, b2, eps, wd, clip_norm, skipped=None, hyper=None):
    """Fused clip + Adam over the arena's active spans (``flat.active_spans``); bumps the device step counter
    ``step_dev`` (int32[1]) and writes the bf16 mirror (``flat.shadow``) when present.  No host scalars depend
    on the step: graph-capturable.  ``hyper`` (fp32[5] on the device: lr, beta1, beta2, eps, weight decay)
    overrides the scalar arguments, so a captured replay follows later learning-rate changes."""
    nparts = 1024
    part = getattr(flat, "_norm_parts", None)
    if part is None or part.numel() < nparts:
        part = flat._norm_parts = torch.zeros(nparts, dtype=torch.float32, device=flat.data.device)
    spans, nspans = flat.span_table(lib().iit_adam_span_size(), max_len4=_ADAM_SPAN4)
    # fused norm: the weight gradients a GEMM stored this step already added their sums of squares into gsq
    sq_spans, n_sq, gsq = flat.norm_spans(lib().iit_adam_span_size())
    _check(lib().iit_adam_flat(_p(flat.data), _p(flat.grad), _p(exp_avg), _p(exp_avg_sq), _p(flat.shadow),
                               _p(spans), nspans, _p(part), nparts, float(clip_norm or 0.0), lr, b1, b2, eps, wd,
                               _p(hyper), _p(step_dev), _p(skipped), _p(sq_spans), n_sq, _p(gsq), _stream()),
           "adam_flat")
    flat.after_step(mirror_written=flat.shadow is not None)


IOI_HL_NODES = {"all_nodes_hook": 0, "hook_duplicate": 1, "hook_s_inhibition": 2, "hook_name_mover": 3}


def ioi_hl_label(base, src, name_table, V: int, node: int, out):
    """Intervened IOI HL label per sequence (csrc/ioi_hl.hip): ``base`` / ``src`` int64 [B, S] tokens, ``node`` the
    interchanged HL node (IOI_HL_NODES), ``out`` int64 [B]."""
    B, S = base.shape
    _check(lib().iit_ioi_hl_label(_p(base), _p(src), _p(name_table), name_table.numel(), B, S, V, node, _p(out),
                                  _stream()), "ioi_hl_label")


def gemm_glds_set_prof(buf) -> None:
    """Arm the LDS-DMA GEMM's timeline probe for the next ``gemm_glds`` launch on this thread: ``buf`` int64
    [workgroups * 64] on the device (scripts/gemm_timeline.py)."""
    lib().iit_gemm_glds_set_prof(_p(buf))


def gemm_glds_set_group_m(gm: int) -> None:
    """M-tiles per group of the LDS-DMA GEMM's XCD-local tile order for later launches (0 = default 8)."""
    lib().iit_gemm_glds_set_group_m(int(gm))
