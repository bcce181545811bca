// LDS-DMA (global_load_lds) MFMA GEMM for gfx950: the engine's mid-size GEMMs (M, N, K multiples of the tile).
//
// C[M,N] = A[M,K] * B[K,N] for the three operand layouts the transformer uses:
//   mode 0  A [M][K], B [N][K]          dX = dY W^T
//   mode 2  A [M][K], B [K][N]          forward, TL-layout weights (bf16 arena mirror)
//   mode 3  A [K][M], B [K][N]          weight gradients X^T dY (reduction over tokens)
// with the epilogue fused (bias / packed-QKV bias / fp32 residual add / bias+gelu_new with the pre-activation /
// fp32 accumulate into the gradient arena / fp32 store).
//
// Structure (cdna_hip_programming.md §5, "step-3" + T1/T2/T10):
// * 256 threads = 4 wave64 as 2x2; tile BM x BN x 64; each wave a (BM/2) x (BN/2) block of 16x16 fp32
//   accumulators fed by v_mfma_f32_16x16x32_bf16.
// * Operands are staged global -> LDS with 16-byte global_load_lds (no VGPR round trip, no ds_write pass) into
//   an NS-deep ring of LDS buffers: NS-1 K-tiles are in flight while the MFMAs consume one; each K-step waits
//   with a counted s_waitcnt vmcnt (never 0 in steady state) and one raw s_barrier, so the DMA spans barriers
//   (a __syncthreads() would drain it: "Pipelining across barriers").
// * LDS images are lane-linear per wave (what LDS-DMA requires) and XOR-swizzled through the *source* address:
//     k-contiguous [rows][64]:   16-B chunk c of row r lives at slot c ^ ((r >> 1) & 7)  -> ds_read_b128 fragment
//                                 reads of 16 rows hit 16 distinct bank groups (conflict-free);
//     k-major [64][cols]:         32-B block b of k-row r lives at b ^ f(r)  -> the 16 k-rows one
//                                 ds_read_b64_tr_b16 instruction touches spread over all 64 banks (2 passes, the minimum).
// * k-major operands (X^T dY, [K][N] weights) are transposed by the gfx950 LDS transpose read, so no operand is
//   ever re-laid-out in memory.
// * Bijective XCD-aware tile remap: the tiles of one XCD share A row panels in its L2.
// * Split-K (fp32 accumulate epilogue only): blockIdx.y takes a K range and adds its partial tile with fp32
//   atomics -- for the weight gradients, whose [d][N] outputs are too few tiles to fill 256 CUs.
// * Epilogue: accumulators -> LDS (fp32 tile) -> each thread owns 8 consecutive columns of a row: 16-B / 32-B
//   vector loads of bias / residual / accumulator and vector stores (the MFMA C layout would otherwise give
//   2-byte column-strided stores).
// * E_DGELU (mode 0, the MLP backward dpre = (dY W_out^T) * gelu_new'(pre)): reads the saved pre-activation in the
//   epilogue and, with ``csum``, also reduces the stored dpre tile over its rows in LDS into the b_in gradient
//   (one atomic per column per tile) -- the separate dgelu pass and the bias column-sum pass disappear.
#include "gemm_glds_body.h"

namespace {

template <int BM, int BN, int NS, bool AKM, bool BKM, int EPI, int NW, int BK = 64, int OCC = 1>
__global__ __launch_bounds__(NW * 64, OCC) void gemm_glds_kernel(G2Args p) {
  __shared__ __attribute__((aligned(16))) char smem[GldsSmem<BM, BN, NS, NW, BK, OCC>::BYTES];  // ONE LDS object
  gemm_glds_body<BM, BN, NS, AKM, BKM, EPI, NW, BK, OCC>(p, blockIdx.x, gridDim.x, blockIdx.y, gridDim.y, smem);
}

template <int BM, int BN, int NS, bool AKM, bool BKM, int EPI, int NW = 4, int BK = 64, int OCC = 1>
hipError_t launch(const G2Args& a, hipStream_t s) {
  const int tiles = (a.M / BM) * (a.N / BN);
  hipLaunchKernelGGL((gemm_glds_kernel<BM, BN, NS, AKM, BKM, EPI, NW, BK, OCC>), dim3(tiles, a.K / a.k_per_split),
                     dim3(NW * 64), 0, s, a);
  return hipGetLastError();
}

// tile configurations: (BM, BN, LDS stages)
template <bool AKM, bool BKM, int EPI>
hipError_t launch_tile(const G2Args& a, int tile, hipStream_t s) {
  switch (tile) {
    case 0: return launch<128, 128, 3, AKM, BKM, EPI>(a, s);
    case 1: return launch<128, 64, 4, AKM, BKM, EPI>(a, s);
    case 2: return launch<64, 128, 4, AKM, BKM, EPI>(a, s);
    case 3: return launch<64, 64, 4, AKM, BKM, EPI>(a, s);
    // 8 waves (two per SIMD, 64 x 96 each): one 256-CU round for 4096 x {2304, 3072}
    case 5: return launch<256, 192, 2, AKM, BKM, EPI, 8>(a, s);
    case 6: return launch<128, 128, 4, AKM, BKM, EPI, 8>(a, s);  // two waves per SIMD (32 x 64 each)
    case 7: return launch<256, 128, 2, AKM, BKM, EPI, 8>(a, s);
    // 96 x 96: the [768][3072] / [3072][768] weight gradients are exactly 256 tiles (one per CU) where 128 x 128
    // leaves 112 CUs idle; 2 x 2 waves of 48 x 48 (3 x 3 MFMA blocks)
    case 8: return launch<96, 96, 4, AKM, BKM, EPI>(a, s);
    // 128 x 96: the 4096 x 768 outputs (W_O / W_out forward, dX of QKV / W_O / W_in) are exactly 256 tiles
    case 9: return launch<128, 96, 4, AKM, BKM, EPI>(a, s);
    // 96 x 192 / 192 x 96 (2 x 2 waves of 48 x 96 / 96 x 48): the weight gradients with a 2-way reduction split
    // -- 256 workgroups for [768][3072] / [3072][768], a third fewer operand bytes per CU than 96 x 96
    case 10: return launch<96, 192, 4, AKM, BKM, EPI>(a, s);
    case 11: return launch<192, 96, 4, AKM, BKM, EPI>(a, s);
    // deep LDS rings (5-8 K-tiles, up to 144 KiB): more operand bytes in flight per CU for the intake-bound tiles
    case 12: return launch<96, 96, 6, AKM, BKM, EPI>(a, s);
    case 13: return launch<128, 96, 5, AKM, BKM, EPI>(a, s);
    case 14: return launch<64, 64, 8, AKM, BKM, EPI>(a, s);
    // 128-deep K-tiles (256-B row segments per DMA, half the K-tiles / barriers per K): the intake experiment
    case 15: return launch<128, 96, 2, AKM, BKM, EPI, 4, 128>(a, s);
    case 16: return launch<96, 96, 3, AKM, BKM, EPI, 4, 128>(a, s);
    case 17: return launch<64, 64, 4, AKM, BKM, EPI, 4, 128>(a, s);
    case 18: return launch<128, 128, 2, AKM, BKM, EPI, 4, 128>(a, s);
    // 192 x 192 (2 x 2 waves of 96 x 96, 6 x 6 MFMA blocks): the weight gradients with a 4-way reduction split --
    // 192 workgroups for [768][3072] / [3072][768] / 144 for [768][2304] at half the operand bytes per flop of
    // 96 x 96 (the intake-bound regime); 3- and 2-deep rings
    // (tile 19 was 192 x 192 with a 3-deep ring: wrong results under the reduction split; not offered)
    case 20: return launch<192, 192, 2, AKM, BKM, EPI>(a, s);
    // 192 x 128 / 128 x 192 (2 x 2 waves of 96 x 64 / 64 x 96), 4-deep rings (exactly 160 KiB)
    case 21: return launch<192, 128, 4, AKM, BKM, EPI>(a, s);
    case 22: return launch<128, 192, 4, AKM, BKM, EPI>(a, s);
    // two co-resident workgroups per CU (OCC = 2: <= 80 KiB LDS, <= 256 registers per lane), so one tile's
    // prologue / epilogue overlaps the other's main loop; shapes with >= 512 tiles
    case 23: return launch<128, 96, 2, AKM, BKM, EPI, 4, 64, 2>(a, s);
    case 24: return launch<64, 96, 3, AKM, BKM, EPI, 4, 64, 2>(a, s);
    case 25: return launch<128, 128, 2, AKM, BKM, EPI, 4, 64, 2>(a, s);
    case 26: return launch<96, 96, 3, AKM, BKM, EPI, 4, 64, 2>(a, s);
    case 27: return launch<128, 192, 2, AKM, BKM, EPI, 4, 64, 2>(a, s);
    case 28: return launch<64, 192, 2, AKM, BKM, EPI, 4, 64, 2>(a, s);
    // three / four co-resident workgroups per CU: the HBM-bound residual-epilogue shapes ([4096][768] outputs)
    case 29: return launch<64, 96, 2, AKM, BKM, EPI, 4, 64, 3>(a, s);
    case 30: return launch<64, 64, 2, AKM, BKM, EPI, 4, 64, 4>(a, s);
    case 31: return launch<64, 128, 2, AKM, BKM, EPI, 4, 64, 3>(a, s);
    // the in-flight-depth test on the big 8-wave tiles: 3-deep rings (2 K-tiles in flight while one is consumed,
    // tile 5 / 7 keep one) within 160 KiB, and the 256 x 256 two-stage tile
    case 32: return launch<256, 128, 3, AKM, BKM, EPI, 8>(a, s);
    case 33: return launch<128, 256, 3, AKM, BKM, EPI, 8>(a, s);
    case 34: return launch<256, 256, 2, AKM, BKM, EPI, 8>(a, s);
    // (tiles 35-37, 128 / 256 x 288 for the packed-QKV forward -- 8 N-tiles of [*][2304], whole 256-CU rounds --
    // measured 52.9-53.9 us at M = 8192 vs 39.6 us for tile 27 and 39.0 us hipBLASLt, and the 2-deep 128 x 288
    // returned NaNs (profiles/qkv_fwd_tiles_r4.txt): removed; not offered)
    default: return launch<128, 128, 4, AKM, BKM, EPI>(a, s);
  }
}

}  // namespace

#define IIT_GLDS_TILES 38
static const int kTileBM[IIT_GLDS_TILES] = {128, 128, 64, 64, 128, 256, 128, 256, 96, 128, 96, 192, 96, 128, 64,
                                            128, 96, 64, 128, 192, 192, 192, 128, 128, 64, 128, 96, 128, 64,
                                            64, 64, 64, 256, 128, 256, 128, 256, 128};
static const int kTileBN[IIT_GLDS_TILES] = {128, 64, 128, 64, 128, 192, 128, 128, 96, 96, 192, 96, 96, 96, 64,
                                            96, 96, 64, 128, 192, 192, 128, 192, 96, 96, 128, 96, 192, 192,
                                            96, 64, 128, 128, 256, 256, 288, 288, 288};
static const int kTileBK[IIT_GLDS_TILES] = {64, 64, 64, 64, 64, 64, 64, 64, 64, 64, 64, 64, 64, 64, 64,
                                            128, 128, 128, 128, 64, 64, 64, 64, 64, 64, 64, 64, 64, 64,
                                            64, 64, 64, 64, 64, 64, 64, 64, 64};

// 1 when (shape, layout, epilogue, tile) is covered by the LDS-DMA kernel (caller falls back otherwise)
// tile 40: the 256 x 256 8-phase kernel of gemm_8ph.hip; tiles 41 / 42: the 256 x 256 four-wave 32x32x16 kernel
// of gemm_4w.hip with 64- / 32-deep K-tiles (2- / 4-slot LDS-DMA rings); no K split for any of them
#define IIT_8PH_TILE 40
#define IIT_4W_TILE 41
#define IIT_4W32_TILE 42
extern "C" int iit_gemm_8ph_ok(int M, int N, int K, int mode, int epi);
extern "C" int iit_gemm_8ph_run(const void* args, int mode, int epi, void* stream);
extern "C" int iit_gemm_4w_run(const void* args, int mode, int epi, int bk, void* stream);

IIT_EXPORT int iit_gemm_glds_ok(const void* A, const void* B, const void* C, const void* C2, const void* resid,
                                long lda, long ldb, long ldc, long ldc2, long ldr, int M, int N, int K, int mode,
                                int epi, int bias_cols, int tile, int splits, int reduce) {
  if (tile == IIT_8PH_TILE || tile == IIT_4W_TILE || tile == IIT_4W32_TILE) {  // 256 x 256 tiles, K % 64 == 0
    if (splits != 1 || reduce || !iit_gemm_8ph_ok(M, N, K, mode, epi)) return 0;
    if ((epi == E_DGELU || epi == E_DGELU_ERF) && !C2) return 0;
    if (lda % 8 || ldb % 8 || ldc % 8 || (C2 && ldc2 % 8) || (resid && ldr % 8)) return 0;
    if (((uintptr_t)A | (uintptr_t)B | (uintptr_t)C | (uintptr_t)C2 | (uintptr_t)resid) & 15) return 0;
    if (epi == E_BF16_BIAS3 && bias_cols % 8) return 0;
    return 1;
  }
  if (tile < 0 || tile >= IIT_GLDS_TILES || tile == 19 || tile >= 35) return 0;
  // atomic split-K: fp32 accumulate only; reduction split-K (``reduce``): fp32 accumulate, store or residual add (the
  // last-arriving split runs the epilogue once on the summed tile)
  const bool split_epi = epi == E_F32_ACC || (reduce && (epi == E_F32_STORE || epi == E_F32_RESID));
  const int bk = kTileBK[tile];
  if (splits < 1 || (splits > 1 && (!split_epi || K % (bk * splits)))) return 0;
  if (reduce && splits < 2) return 0;
  if (!(mode == 0 || mode == 2 || mode == 3)) return 0;
  const bool epi_ok = mode == 3 ? (epi == E_F32_ACC || epi == E_F32_STORE)
                                : (epi == E_BF16 || epi == E_BF16_BIAS3 || epi == E_F32_RESID || epi == E_GELU ||
                                   epi == E_GELU_ERF || epi == E_F32_ACC || epi == E_F32_STORE || epi == E_DGELU ||
                                   epi == E_DGELU_ERF);
  if (!epi_ok) return 0;
  const bool dg = epi == E_DGELU || epi == E_DGELU_ERF;
  if (mode == 0 && !(epi == E_BF16 || epi == E_F32_ACC || epi == E_F32_STORE || dg)) return 0;
  if (dg && (mode != 0 || !C2)) return 0;
  if (M <= 0 || N <= 0 || K <= 0 || M % kTileBM[tile] || N % kTileBN[tile] || K % bk) return 0;
  if (lda % 8 || ldb % 8 || ldc % 8 || (C2 && ldc2 % 8) || (resid && ldr % 8)) return 0;
  const uintptr_t al = (uintptr_t)A | (uintptr_t)B | (uintptr_t)C | (uintptr_t)C2 | (uintptr_t)resid;
  if (al & 15) return 0;
  if (epi == E_BF16_BIAS3 && bias_cols % 8) return 0;
  return 1;
}

IIT_EXPORT int iit_gemm_glds_sm(const void* A, const void* B, void* C, void* C2, const float* bias0,
                                const float* bias1, const float* bias2, const float* resid, long lda, long ldb, long ldc,
                                long ldc2, long ldr, int M, int N, int K, int mode, int epi, int bias_cols, int tile,
                                int splits, float* csum, float* ws, int* counters, int store_mode, float* bsum,
                                float* gsq, void* stream);

// the timeline probe of the NEXT iit_gemm_glds* launch from this host thread (scripts/gemm_timeline.py): a
// [workgroups][64] int64 device buffer, consumed by that launch
static thread_local long long* g_prof_buf = nullptr;
IIT_EXPORT void iit_gemm_glds_set_prof(void* buf) { g_prof_buf = (long long*)buf; }
// M-tiles per group of the XCD-local tile order for every later launch (0 = the default; the group experiment)
static int g_group_m = 0;
IIT_EXPORT void iit_gemm_glds_set_group_m(int gm) { g_group_m = gm; }

IIT_EXPORT int iit_gemm_glds(const void* A, const void* B, void* C, void* C2, const float* bias0, const float* bias1,
                             const float* bias2, const float* resid, long lda, long ldb, long ldc, long ldc2, long ldr,
                             int M, int N, int K, int mode, int epi, int bias_cols, int tile, int splits,
                             float* csum, float* ws, int* counters, void* stream) {
  return iit_gemm_glds_sm(A, B, C, C2, bias0, bias1, bias2, resid, lda, ldb, ldc, ldc2, ldr, M, N, K, mode, epi,
                          bias_cols, tile, splits, csum, ws, counters, 0, nullptr, nullptr, stream);
}

// the same with the epilogue store flavour (G2Args::store_mode) and, for the weight gradients (mode 3), the fused
// column sums of B (``bsum``, += atomically; nullable); ``gsq`` (fp32 store epilogue, nullable): += the sum of squares
// of the stored values, spread over 64 slots
IIT_EXPORT int iit_gemm_glds_sm(const void* A, const void* B, void* C, void* C2, const float* bias0,
                                const float* bias1, const float* bias2, const float* resid, long lda, long ldb, long ldc,
                                long ldc2, long ldr, int M, int N, int K, int mode, int epi, int bias_cols, int tile,
                                int splits, float* csum, float* ws, int* counters, int store_mode, float* bsum,
                                float* gsq, void* stream) {
  const int reduce = ws != nullptr;
  if (!iit_gemm_glds_ok(A, B, C, C2, resid, lda, ldb, ldc, ldc2, ldr, M, N, K, mode, epi, bias_cols, tile, splits,
                        reduce))
    return (int)hipErrorInvalidValue;
  if (reduce && !counters) return (int)hipErrorInvalidValue;
  G2Args a{};
  a.A = (const __bf16*)A; a.B = (const __bf16*)B; a.C = C; a.C2 = C2;
  a.bias0 = bias0; a.bias1 = bias1; a.bias2 = bias2; a.resid = resid;
  a.lda = lda; a.ldb = ldb; a.ldc = ldc; a.ldc2 = ldc2; a.ldr = ldr;
  a.M = M; a.N = N; a.K = K; a.bias_cols = bias_cols; a.k_per_split = K / splits;
  a.csum = (epi == E_DGELU || epi == E_DGELU_ERF) ? csum : nullptr;
  a.ws = reduce ? ws : nullptr;  // workspace >= splits * M * N floats, counters >= tiles ints (zero when idle)
  a.counters = reduce ? counters : nullptr;
  a.store_mode = store_mode;
  a.prof = g_prof_buf;
  g_prof_buf = nullptr;
  a.group_m = g_group_m;
  a.bsum = mode == 3 ? bsum : nullptr;
  a.gsq = epi == E_F32_STORE ? gsq : nullptr;
  hipStream_t s = (hipStream_t)stream;
  if (tile == IIT_8PH_TILE) return iit_gemm_8ph_run(&a, mode, epi, stream);
  if (tile == IIT_4W_TILE) return iit_gemm_4w_run(&a, mode, epi, 64, stream);
  if (tile == IIT_4W32_TILE) return iit_gemm_4w_run(&a, mode, epi, 32, stream);
#define G2(MODE, AK, BK_, EPI) \
  if (mode == (MODE) && epi == (EPI)) return (int)launch_tile<AK, BK_, EPI>(a, tile, s);
  G2(0, false, false, E_BF16)
  G2(0, false, false, E_F32_ACC)
  G2(0, false, false, E_F32_STORE)
  G2(0, false, false, E_DGELU)
  G2(0, false, false, E_DGELU_ERF)
  G2(2, false, true, E_BF16)
  G2(2, false, true, E_BF16_BIAS3)
  G2(2, false, true, E_F32_RESID)
  G2(2, false, true, E_GELU)
  G2(2, false, true, E_GELU_ERF)
  G2(2, false, true, E_F32_ACC)
  G2(2, false, true, E_F32_STORE)
  G2(3, true, true, E_F32_ACC)
  G2(3, true, true, E_F32_STORE)
#undef G2
  return (int)hipErrorInvalidValue;
}
