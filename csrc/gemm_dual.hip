// Two GEMM problems in ONE launch: a layer's weight gradient dW = X^T dY (mode 3, fp32 store / accumulate, optional
// K-split) and its input gradient dX = dY W^T (mode 0, bf16 or the fused dgelu epilogue).  The two are independent,
// and each alone is about one round of tiles on the 256 CUs: run back to back, every launch pays its own ramp,
// pipeline fill, epilogue drain and tail (profiles/gemm_timeline_r3.txt: 5-13 us of a 20-37 us GEMM), and HIP graph
// branches on side streams do not overlap them (profiles/graph_branch_concurrency_r3.txt).  Here the workgroups of
// both problems share one grid -- two workgroups per CU (4 waves, <= 80 KiB LDS each), so one problem's prologue /
// epilogue runs under the other's main loop, or one big 8-wave tile per CU -- and the launch has one tail instead of
// two.
//
// The per-tile code is gemm_glds_body (csrc/gemm_glds_body.h), unchanged: workgroups [0, w_tiles * w_splits) take
// the dW tiles (split-major, so the K-splits of a tile are a launch round apart and its reduction ticket is taken
// late), the rest the dX tiles.  The dW problem comes first because its K (the token count) is the longer loop.
#include "gemm_glds_body.h"

namespace {

// a tile of the dual launch: BM x BN, NS-deep LDS ring, NW waves, OCC workgroups per CU (both problems of one launch
// share NW and OCC)
template <int BM_, int BN_, int NS_, int NW_ = 4, int OCC_ = 2>
struct Cfg {
  static constexpr int BM = BM_, BN = BN_, NS = NS_, NW = NW_, OCC = OCC_;
  static constexpr int SMEM = GldsSmem<BM_, BN_, NS_, NW_, 64, OCC_>::BYTES;
};

// Cold-operand prefetch (profiles/dual_l2_hypothesis_r6.txt: inside the step a pair runs 7-19 % slower than back to
// back because its forward-saved activation and its weight come from HBM, not the Infinity Cache): the first
// ``pf.wgs`` workgroups of the launch read the NEXT pair's cold operands (up to two ranges) once, one 4-B load per
// 64-B granule, so they are cache-resident when that pair starts.  They run beside the tiles, whose operand intake is
// L2 -> LDS bound and leaves HBM bandwidth unused.  Loads only: nothing is written.
struct Prefetch {
  const char* p[2];
  long bytes[2];
  int wgs;
};

__device__ __forceinline__ void prefetch_part(const Prefetch& pf, int part) {
  unsigned acc = 0u;
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    if (!pf.p[r] || pf.bytes[r] <= 0) continue;
    const long gran = (pf.bytes[r] + 63) / 64;
    const long per = (gran + pf.wgs - 1) / pf.wgs;
    const long g0 = (long)part * per;
    const long g1 = g0 + per < gran ? g0 + per : gran;
    const char* base = pf.p[r];
    for (long g = g0 + threadIdx.x; g < g1; g += (long)blockDim.x * 8) {
      unsigned v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const long gg = g + (long)u * blockDim.x;
        v[u] = gg < g1 ? *(const unsigned*)(base + gg * 64) : 0u;
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) acc ^= v[u];
    }
  }
  asm volatile("" ::"v"(acc));  // keep the loads
}

template <class TW, int EW, class TX, int EX>
__global__ __launch_bounds__(TW::NW * 64, TW::OCC) void gemm_dual_kernel(G2Args pw, G2Args px, int w_tiles,
                                                                         int w_splits, int x_tiles, Prefetch pf) {
  static_assert(TW::NW == TX::NW && TW::OCC == TX::OCC, "one launch geometry");
  __shared__ __attribute__((aligned(16))) char smem[TW::SMEM > TX::SMEM ? TW::SMEM : TX::SMEM];  // ONE LDS object
  if ((int)blockIdx.x < pf.wgs) {
    prefetch_part(pf, blockIdx.x);
    return;
  }
  const int b = blockIdx.x - pf.wgs;  // (pf.wgs is a multiple of 8: the tiles keep their XCD placement)
  const int nw = w_tiles * w_splits;
  if (b < nw) {
    gemm_glds_body<TW::BM, TW::BN, TW::NS, true, true, EW, TW::NW, 64, TW::OCC>(pw, b % w_tiles, w_tiles,
                                                                                b / w_tiles, w_splits, smem);
  } else {
    gemm_glds_body<TX::BM, TX::BN, TX::NS, false, false, EX, TX::NW, 64, TX::OCC>(px, b - nw, x_tiles, 0, 1, smem);
  }
}

// Two families of tiles (a launch takes both of its tiles from one family):
// * 4 waves, two workgroups per CU: dW 128x96, 128x128, 96x96, 64x96, 64x64; dX 128x96, 64x96, 128x192, 128x128 --
//   one problem's prologue / epilogue under the other's main loop on the same CU;
// * 8 waves (two per SIMD), one workgroup per CU: dW 256x128, 128x128, dX 256x192, 256x128, 128x128 -- the big
//   tiles that run the
//   paired forward at ~1 PF/s (fewer operand bytes per flop than 128x128), which alone leave most of the CUs idle on a
//   [768][N] weight gradient; here the dX tiles fill them.  (A 256x192 dW tile spills registers: not offered.)
// (index -> the single-launch tile id of the same shape, for the shape checks)
// * 4 waves, one workgroup per CU, deep rings (3-4 K-tiles, up to 128 KiB): dW 128x128, 128x96, dX 128x128,
//   128x192 -- more operand bytes in flight for the operands that come cold from HBM inside the step (the
//   activations saved by the forward), where the two-stage rings of the two-per-CU tiles wait on the fill.
constexpr int kWTiles = 9, kXTiles = 9;
const int kWTileId[kWTiles] = {23, 25, 26, 24, 3, 7, 6, 4, 13};
const int kXTileId[kXTiles] = {23, 24, 27, 25, 5, 7, 6, 4, 22};
const int kWBM[kWTiles] = {128, 128, 96, 64, 64, 256, 128, 128, 128};
const int kWBN[kWTiles] = {96, 128, 96, 96, 64, 128, 128, 128, 96};
const int kXBM[kXTiles] = {128, 64, 128, 128, 256, 256, 128, 128, 128};
const int kXBN[kXTiles] = {96, 96, 192, 128, 192, 128, 128, 128, 192};
// tile family: 0 = 4 waves x 2 per CU, 1 = 8 waves x 1 per CU, 2 = 4 waves x 1 per CU with deep rings
__host__ __device__ constexpr int w_family(int t) { return t >= 7 ? 2 : (t >= 5 ? 1 : 0); }
__host__ __device__ constexpr int x_family(int t) { return t >= 7 ? 2 : (t >= 4 ? 1 : 0); }

template <class TW, int EW, class TX, int EX>
hipError_t launch2(const G2Args& w, const G2Args& x, int w_splits, const Prefetch& pf, hipStream_t s) {
  const int wt = (w.M / TW::BM) * (w.N / TW::BN), xt = (x.M / TX::BM) * (x.N / TX::BN);
  hipLaunchKernelGGL((gemm_dual_kernel<TW, EW, TX, EX>), dim3(pf.wgs + wt * w_splits + xt), dim3(TW::NW * 64), 0, s,
                     w, x, wt, w_splits, xt, pf);
  return hipGetLastError();
}

template <class TW, int EW, int EX>
hipError_t pick_x(const G2Args& w, const G2Args& x, int w_splits, int xtile, const Prefetch& pf, hipStream_t s) {
  if constexpr (TW::NW == 4 && TW::OCC == 1) {
    switch (xtile) {
      case 7: return launch2<TW, EW, Cfg<128, 128, 4, 4, 1>, EX>(w, x, w_splits, pf, s);
      case 8: return launch2<TW, EW, Cfg<128, 192, 3, 4, 1>, EX>(w, x, w_splits, pf, s);
      default: return hipErrorInvalidValue;
    }
  } else if constexpr (TW::NW == 4) {
    switch (xtile) {
      case 0: return launch2<TW, EW, Cfg<128, 96, 2>, EX>(w, x, w_splits, pf, s);
      case 1: return launch2<TW, EW, Cfg<64, 96, 3>, EX>(w, x, w_splits, pf, s);
      case 2: return launch2<TW, EW, Cfg<128, 192, 2>, EX>(w, x, w_splits, pf, s);
      case 3: return launch2<TW, EW, Cfg<128, 128, 2>, EX>(w, x, w_splits, pf, s);
      default: return hipErrorInvalidValue;
    }
  } else {
    switch (xtile) {
      case 4: return launch2<TW, EW, Cfg<256, 192, 2, 8, 1>, EX>(w, x, w_splits, pf, s);
      case 5: return launch2<TW, EW, Cfg<256, 128, 2, 8, 1>, EX>(w, x, w_splits, pf, s);
      case 6: return launch2<TW, EW, Cfg<128, 128, 4, 8, 1>, EX>(w, x, w_splits, pf, s);
      default: return hipErrorInvalidValue;
    }
  }
}

template <int EW, int EX>
hipError_t pick_w(const G2Args& w, const G2Args& x, int w_splits, int wtile, int xtile, const Prefetch& pf,
                  hipStream_t s) {
  switch (wtile) {
    case 0: return pick_x<Cfg<128, 96, 2>, EW, EX>(w, x, w_splits, xtile, pf, s);
    case 1: return pick_x<Cfg<128, 128, 2>, EW, EX>(w, x, w_splits, xtile, pf, s);
    case 2: return pick_x<Cfg<96, 96, 3>, EW, EX>(w, x, w_splits, xtile, pf, s);
    case 3: return pick_x<Cfg<64, 96, 3>, EW, EX>(w, x, w_splits, xtile, pf, s);
    case 4: return pick_x<Cfg<64, 64, 4>, EW, EX>(w, x, w_splits, xtile, pf, s);
    case 5: return pick_x<Cfg<256, 128, 2, 8, 1>, EW, EX>(w, x, w_splits, xtile, pf, s);
    case 6: return pick_x<Cfg<128, 128, 4, 8, 1>, EW, EX>(w, x, w_splits, xtile, pf, s);
    case 7: return pick_x<Cfg<128, 128, 4, 4, 1>, EW, EX>(w, x, w_splits, xtile, pf, s);
    case 8: return pick_x<Cfg<128, 96, 4, 4, 1>, EW, EX>(w, x, w_splits, xtile, pf, s);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace

extern "C" int iit_gemm_glds_ok(const void* A, const void* B, const void* C, const void* C2, const void* resid,
                                long lda, long ldb, long ldc, long ldc2, long ldr, int M, int N, int K, int mode,
                                int epi, int bias_cols, int tile, int splits, int reduce);

IIT_EXPORT int iit_gemm_dual_tiles(int* w_tiles, int* x_tiles) {
  *w_tiles = kWTiles;
  *x_tiles = kXTiles;
  return 0;
}

// 1 when the pair (dW problem on dual tile ``wtile`` with ``wsplits`` K-splits -- reduction split when ``reduce`` --,
// dX problem on dual tile ``xtile``) is covered by the dual kernel
IIT_EXPORT int iit_gemm_dual_ok(const void* wA, const void* wB, const void* wC, long wlda, long wldb, long wldc, int wM,
                                int wN, int wK, int wepi, int wtile, int wsplits, int reduce, const void* xA,
                                const void* xB, const void* xC, const void* xC2, long xlda, long xldb, long xldc,
                                long xldc2, int xM, int xN, int xK, int xepi, int xtile) {
  if (wtile < 0 || wtile >= kWTiles || xtile < 0 || xtile >= kXTiles || w_family(wtile) != x_family(xtile)) return 0;
  if (!(wepi == E_F32_STORE || wepi == E_F32_ACC) || !(xepi == E_BF16 || xepi == E_DGELU)) return 0;
  if (!iit_gemm_glds_ok(wA, wB, wC, nullptr, nullptr, wlda, wldb, wldc, 0, 0, wM, wN, wK, 3, wepi, 0,
                        kWTileId[wtile], wsplits, reduce))
    return 0;
  if (!iit_gemm_glds_ok(xA, xB, xC, xepi == E_DGELU ? xC2 : nullptr, nullptr, xlda, xldb, xldc, xldc2, 0, xM, xN, xK,
                        0, xepi, 0, kXTileId[xtile], 1, 0))
    return 0;
  // the dW tiles' XCD-local order needs their count to be a multiple of the 8 XCDs only for locality, not for
  // correctness; the grid must stay within one dimension
  const long wg = (long)(wM / kWBM[wtile]) * (wN / kWBN[wtile]) * wsplits + (long)(xM / kXBM[xtile]) * (xN / kXBN[xtile]);
  return wg > 0 && wg < (1L << 31) ? 1 : 0;
}

// M-tiles per group of the XCD-local tile order for both problems of every later dual launch (0 = the body's default
// of 8; IIT_GEMM_DUAL_GROUP_M, the tile-order experiment of the dual kernels)
static int g_dual_group_m = 0;
IIT_EXPORT void iit_gemm_dual_set_group_m(int gm) { g_dual_group_m = gm; }

IIT_EXPORT int iit_gemm_dual(const void* wA, const void* wB, void* wC, long wlda, long wldb, long wldc, int wM, int wN,
                             int wK, int wepi, int wtile, int wsplits, float* ws, int* counters, const void* xA,
                             const void* xB, void* xC, void* xC2, long xlda, long xldb, long xldc, long xldc2, int xM,
                             int xN, int xK, int xepi, int xtile, float* csum, float* bsum, float* gsq,
                             const void* pf0, long pf0_bytes, const void* pf1, long pf1_bytes, int pf_wgs,
                             void* stream) {
  const int reduce = ws != nullptr;
  if (!iit_gemm_dual_ok(wA, wB, wC, wlda, wldb, wldc, wM, wN, wK, wepi, wtile, wsplits, reduce, xA, xB, xC, xC2, xlda,
                        xldb, xldc, xldc2, xM, xN, xK, xepi, xtile))
    return (int)hipErrorInvalidValue;
  if (reduce && !counters) return (int)hipErrorInvalidValue;
  G2Args w{};
  w.A = (const __bf16*)wA; w.B = (const __bf16*)wB; w.C = wC;
  w.lda = wlda; w.ldb = wldb; w.ldc = wldc;
  w.M = wM; w.N = wN; w.K = wK; w.k_per_split = wK / wsplits;
  w.ws = reduce ? ws : nullptr;
  w.counters = reduce ? counters : nullptr;
  w.bsum = bsum;  // the dW problem's column sums of dY (its bias gradient), nullable
  w.gsq = wepi == E_F32_STORE ? gsq : nullptr;  // its sum of squares (the clip's global norm), nullable
  G2Args x{};
  x.A = (const __bf16*)xA; x.B = (const __bf16*)xB; x.C = xC; x.C2 = xC2;
  x.lda = xlda; x.ldb = xldb; x.ldc = xldc; x.ldc2 = xldc2;
  x.M = xM; x.N = xN; x.K = xK; x.k_per_split = xK;
  x.csum = xepi == E_DGELU ? csum : nullptr;
  w.group_m = x.group_m = g_dual_group_m;
  // prefetch workgroups: a multiple of 8 (the tiles keep their blockIdx % 8 XCD placement), none without a range
  Prefetch pf{{(const char*)pf0, (const char*)pf1}, {pf0 ? pf0_bytes : 0, pf1 ? pf1_bytes : 0}, 0};
  if ((pf.bytes[0] > 0 || pf.bytes[1] > 0) && pf_wgs > 0) pf.wgs = ((pf_wgs + 7) / 8) * 8;
  if (pf.wgs > 1024) pf.wgs = 1024;
  hipStream_t s = (hipStream_t)stream;
  if (wepi == E_F32_STORE && xepi == E_BF16)
    return (int)pick_w<E_F32_STORE, E_BF16>(w, x, wsplits, wtile, xtile, pf, s);
  if (wepi == E_F32_STORE && xepi == E_DGELU)
    return (int)pick_w<E_F32_STORE, E_DGELU>(w, x, wsplits, wtile, xtile, pf, s);
  if (wepi == E_F32_ACC && xepi == E_BF16) return (int)pick_w<E_F32_ACC, E_BF16>(w, x, wsplits, wtile, xtile, pf, s);
  if (wepi == E_F32_ACC && xepi == E_DGELU) return (int)pick_w<E_F32_ACC, E_DGELU>(w, x, wsplits, wtile, xtile, pf, s);
  return (int)hipErrorInvalidValue;
}
