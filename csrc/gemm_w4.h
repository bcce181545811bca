// Shared device code of the 256 x 256 four-wave GEMM (csrc/gemm_4w.hip documents the design): geometry, the 32x32x16
// fragment reads, the lean LDS-DMA staging, and the main loop over a range of K-tiles of one output tile
// (``w4_tile_loop``) -- used by the one-tile-per-workgroup launches of gemm_4w.hip and the persistent stream-K
// launches of gemm_sk.hip.
#pragma once
#include <type_traits>

#include "gemm_glds_body.h"

namespace {

constexpr int W4_BM = 256, W4_BN = 256, W4_NW = 4, W4_NT = 256;
constexpr int W4_EPS = W4_BN + 4;
constexpr int W4_ECH = 2;  // epilogue row chunks = the two wave rows
constexpr int W4_LDS = 128 * 1024;  // the LDS-DMA ring: 2 slots of 64-deep K-tiles or 4 of 32-deep ones
constexpr int W4_BYTES = W4_LDS > W4_BM / W4_ECH * W4_EPS * 4 ? W4_LDS : W4_BM / W4_ECH * W4_EPS * 4;
static_assert(W4_BYTES <= 160 * 1024, "LDS budget");

// geometry of a K-tile depth: BK = 64 -> 2 ring slots (K-tile t + 2 staged at the boundary of t, waited for one
// K-tile later); BK = 32 -> 4 slots (t + 4 staged at the boundary of t, waited for three K-tiles later: the DMA
// of a K-tile has ~3 x 1024 MFMA cycles to land instead of ~2048, at one barrier per 1024 MFMA cycles)
template <int BK>
struct W4G {
  static constexpr int AB = W4_BM * BK * 2;  // bytes of one operand's K-tile image
  static constexpr int STAGE = 2 * AB;       // A + B
  static constexpr int NSLOT = W4_LDS / STAGE;
  static constexpr int KS = BK / 16;  // 16-deep k-steps per K-tile
};

typedef float f32x16 __attribute__((ext_vector_type(16)));

// compile-time loop: f(std::integral_constant<int, I>) for I = B .. E - 1 (every index a constant expression, so the
// fragment-register and accumulator indices never become run-time indices -- a run-time-indexed register array is
// moved to scratch, and an asm LDS read's destination stored to scratch before the data lands reads garbage)
template <int I, int E>
struct Unroll {
  template <class F>
  __device__ __forceinline__ static void run(F&& f) {
    if constexpr (I < E) {
      f(std::integral_constant<int, I>());
      Unroll<I + 1, E>::run(f);
    }
  }
};

// One 32x32x16 operand fragment (lane l: 8 consecutive k of row / column l & 31, k half l >> 5) of a 32-row block
// of an operand image, issued one LDS instruction (``part``) at a time.  k-contiguous image [256][64]: one
// ds_read_b128; k-major panel image [64][64]: two ds_read_b64_tr_b16 (k rows 0-3 / 4-7 of the lane's k half),
// lane 4q + p of each 16-lane group addressing k row q, columns 4p..4p+3 of the group's 16 columns
// (cdna_hip_programming.md T10).
template <bool KMAJ> constexpr int KMAJ_READS = KMAJ ? 2 : 1;

template <bool KMAJ, int BK>
__device__ __forceinline__ void frag32_part(const char* img, int row0, int kbase, int lane, RawFrag<KMAJ>& f,
                                            int part) {
  if constexpr (!KMAJ) {
    const int row = row0 + (lane & 31);
    const int c = (kbase >> 3) + (lane >> 5);
    const unsigned a = lds_addr(img + row * (BK * 2) + ((c ^ kcont_swz<BK>(row)) << 4));
    asm volatile("ds_read_b128 %0, %1" : "=v"(f.v) : "v"(a));
  } else {
    // panel of 64 columns holding column row0: [BK k][64 cols], 128-B k-rows, 32-B block b of k-row r at
    // b ^ kmaj_swz<64>(r); k rows kr and kr + 4 share the swizzle (kr % 8 < 4): part 1 is part 0 four k-rows on
    const char* pimg = img + (row0 >> 6) * 64 * BK * 2;
    const int grp = lane >> 4, q = (lane >> 2) & 3, pp = lane & 3;
    const int col = (row0 & 63) + 16 * (grp & 1) + 4 * pp;  // lanes 0-15 / 32-47: columns 0-15, 16-31 / 48-63: 16-31
    const int kr = kbase + 8 * (grp >> 1) + q;
    const unsigned a0 =
        lds_addr(pimg + kr * (64 * 2) + ((((col >> 4) ^ kmaj_swz<64>(kr))) << 5) + ((col & 15) << 1));
    if (part == 0) asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(f.lo) : "v"(a0));
    else asm volatile("ds_read_b64_tr_b16 %0, %1 offset:512" : "=v"(f.hi) : "v"(a0));
  }
}

// LDS-DMA instruction g (of OS::N per wave per K-tile) of a lean operand stager
template <int BK, class OS>
__device__ __forceinline__ void stage_one(const OS& os, int kt, char* img, int g) {
  constexpr int NPER = OS::N / OS::NP;
  const int q = g / NPER, i = g % NPER;
  const auto& st = os.st[q];
  glds16(st.ptr[0] + (kt * st.kstep + i * st.istep), img + q * OS::PR * BK * 2 + st.off[0] + i * st.ostep);
}


// acc (+)= A[m0 .. m0 + 256) x B[.., n0 .. n0 + 256) over the K-tiles [kt0, kt0 + nt) of depth BK (the accumulators are
// NOT zeroed here); ``do_cs``: cs[j] += the column sums of this wave's B fragments (the fused bias gradient of a weight
// gradient).  Starts by staging into an idle LDS ring and ends with every wave past its last LDS read of the ring
// (the caller's epilogue may reuse the LDS after a barrier).
template <bool AKM, bool BKM, int EPI, int BK>
__device__ __forceinline__ void w4_tile_loop(const G2Args& p, const int m0, const int n0, const int kt0, const int nt,
                                             char* smem, f32x16 (&acc)[4][4], const bool do_cs, float (&cs)[4]) {
  using G = W4G<BK>;
  constexpr int AB = G::AB, STAGE = G::STAGE, NSLOT = G::NSLOT, KS = G::KS;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  auto slot = [&](int kt) -> char* { return smem + (kt % NSLOT) * STAGE; };
  constexpr bool CS = AKM && BKM && (EPI == E_F32_ACC || EPI == E_F32_STORE);
  using SA = OperandStager<AKM, W4_BM, W4_NW, BK, true>;
  using SB = OperandStager<BKM, W4_BN, W4_NW, BK, true>;
  SA stA;
  SB stB;
  constexpr int NA = SA::N, LOADS = SA::N + SB::N;  // LDS-DMA per wave per K-tile
  stA.init(p.A, p.lda, m0, kt0 * BK, wave, lane);
  stB.init(p.B, p.ldb, n0, kt0 * BK, wave, lane);
  // prologue: K-tiles 0 .. NSLOT - 1 (as many as exist); K-tile 0 waited for
#pragma unroll
  for (int s = 0; s < NSLOT; ++s)
    if (s < nt) {
      stA.stage(s, slot(s));
      stB.stage(s, slot(s) + AB);
    }
  wait_tiles<LOADS>(min(NSLOT, nt) - 1);
  __builtin_amdgcn_s_barrier();

  RawFrag<AKM> fa[2][4];
  RawFrag<BKM> fb[2][4];
  constexpr int RPA = KMAJ_READS<AKM>, RPB = KMAJ_READS<BKM>;
  constexpr int NR = 4 * RPA + 4 * RPB;  // LDS read instructions per k-step: 8 (mode 0), 12 (mode 2), 16 (mode 3)
  // read instruction r of k-step ks into register buffer bufi (A fragments first, then B)
  auto read_one = [&](const char* st, const int ks, const int bufi, const int r) __attribute__((always_inline)) {
    if (r < 4 * RPA) {
      frag32_part<AKM, BK>(st, wm * 128 + (r / RPA) * 32, ks * 16, lane, fa[bufi][r / RPA], r % RPA);
    } else {
      const int rb = r - 4 * RPA;
      frag32_part<BKM, BK>(st + AB, wn * 128 + (rb / RPB) * 32, ks * 16, lane, fb[bufi][rb / RPB], rb % RPB);
    }
  };
  auto glds_one = [&](int kt, char* buf, int gi) __attribute__((always_inline)) {
    if (gi < NA) stage_one<BK>(stA, kt, buf, gi);
    else stage_one<BK>(stB, kt, buf + AB, gi - NA);
  };
#pragma unroll
  for (int r = 0; r < NR; ++r) read_one(smem, 0, 0, r);

  // One k-step = 16 MFMAs; the memory instructions of the next k-step (its NR fragment reads and, at a K-tile
  // boundary, the LOADS LDS-DMA of K-tile kt + NSLOT) are spread between them in program order (sched_barrier pins
  // it), so the single wave of each SIMD keeps the matrix pipe fed while it issues them.  BOUNDARY (the last k-step
  // of a K-tile): after 4 MFMAs the wave waits for K-tile kt + 1's DMA and meets the others at the one barrier of
  // the K-tile -- which also releases slot kt -- and the memory instructions (predicated on kt + 1 < nt /
  // kt + NSLOT < nt) follow it.
  for (int kt = 0; kt < nt; ++kt) {
    const bool has_next = kt + 1 < nt, has_stage = kt + NSLOT < nt;
    // K-tiles in flight after kt + 1 at the boundary wait: kt + 2 .. min(kt + NSLOT - 1, nt - 1)
    const int after = max(0, min(kt + NSLOT - 1, nt - 1) - (kt + 1));
    Unroll<0, KS>::run([&](auto ks_c) __attribute__((always_inline)) {
      constexpr int ks = decltype(ks_c)::value;
      constexpr bool BOUNDARY = ks == KS - 1;
      // placement: the next k-step's memory instructions are spread evenly over the k-step's MFMAs (spreading them
      // over the first half only, so the last read has ~6 MFMAs to land, measured 2-5 % slower); at the boundary
      // the barrier follows MFMA BAR and the reads + the K-tile's LDS-DMA share MFMAs (BAR, 16)
      constexpr int BAR = 3;
      constexpr int LO = BOUNDARY ? BAR + 1 : 0;
      constexpr int NMEM = BOUNDARY ? NR + LOADS : NR;
      constexpr int cur = ks & 1, nxt = cur ^ 1;
      // this k-step's fragments were issued one k-step (16 MFMAs) ago; at the boundary these are the last reads of
      // slot kt, retired before the barrier
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      bf16x8 a[4], b[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) a[i] = frag_use<AKM>(fa[cur][i]);
#pragma unroll
      for (int j = 0; j < 4; ++j) b[j] = frag_use<BKM>(fb[cur][j]);
      const char* rst = !BOUNDARY ? slot(kt) : slot(kt + 1);
      constexpr int rks = !BOUNDARY ? ks + 1 : 0;
      char* gbuf = slot(kt);
      Unroll<0, 16>::run([&](auto m_c) __attribute__((always_inline)) {
        constexpr int m = decltype(m_c)::value;
        acc[m >> 2][m & 3] =
            __builtin_amdgcn_mfma_f32_32x32x16_bf16(b[m & 3], a[m >> 2], acc[m >> 2][m & 3], 0, 0, 0);
        if constexpr (BOUNDARY && m == BAR) {
          // K-tile boundary with BAR + 1 MFMAs queued: wait for K-tile kt + 1's DMA, publish it (and the release of
          // slot kt) with one barrier
          wait_tiles<LOADS>(after);
          __builtin_amdgcn_sched_barrier(0);
          __builtin_amdgcn_s_barrier();
        }
        if constexpr (m >= LO) {
          constexpr int x0 = ((m - LO) * NMEM + (16 - LO) - 1) / (16 - LO);
          constexpr int x1 = ((m - LO + 1) * NMEM + (16 - LO) - 1) / (16 - LO);
          Unroll<x0, x1>::run([&](auto x_c) __attribute__((always_inline)) {
            constexpr int x = decltype(x_c)::value;
            if constexpr (x < NR) {
              if (!BOUNDARY || has_next) read_one(rst, rks, nxt, x);
            } else {
              if (has_stage) glds_one(kt + NSLOT, gbuf, x - NR);
            }
          });
        }
        __builtin_amdgcn_sched_barrier(0);
      });
      if constexpr (CS) {
        if (do_cs) {  // lane l's B fragment: column l & 31 of block j, k rows 8 (l >> 5) + e
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const i32x4 w = __builtin_bit_cast(i32x4, b[j]);
            float u = 0.f;
#pragma unroll
            for (int e = 0; e < 4; ++e)
              u += __builtin_bit_cast(float, (unsigned)w[e] << 16) +
                   __builtin_bit_cast(float, (unsigned)w[e] & 0xffff0000u);
            cs[j] += u;
          }
        }
      }
      __builtin_amdgcn_sched_barrier(0);
    });
  }
}

}  // namespace
