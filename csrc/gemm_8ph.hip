// 256 x 256 x 64 bf16 MFMA GEMM for the large problems (Llama-3-8B projections, 8192-row paired forwards): 8 waves in
// two ping-pong groups and an 8-phase K-loop with one half-tile LDS-DMA prefetch per phase
// (cdna_hip_programming.md §5 "The 256² 8-phase template", T2 / T3 / T4 / T5).  Same operand layouts, epilogues and
// C ABI as the LDS-DMA kernel of gemm_glds.hip (served there as tiles 40+):
//   mode 0  A [M][K], B [N][K];  mode 2  A [M][K], B [K][N];  mode 3  A [K][M], B [K][N]
//
// Geometry.  One workgroup = one 256 x 256 output tile, 512 threads.  Wave w is in group g = w / 4 (the SIMD
// partners are w and w + 4, one per group) at column slot c = w % 4; its output is the four 64 x 32 quadrants
// (qm, qn) at rows qm * 128 + g * 64 + [0, 64) and columns qn * 128 + c * 32 + [0, 32): quadrant (qm, qn) reads
// only the staging half qm of A (tile rows [qm * 128, +128)) and the staging half qn of B.
//
// LDS: two K-tile buffers (parity of the K-tile) of four 16-KiB staging halves {A0, A1, B0, B1} = 128 KiB, filled
// by global_load_lds (lane-linear images, XOR-swizzled through the source address: gemm_glds_body.h Stager).
//
// K-loop: per K-tile t four phases q = 0..3 on the quadrants (0,0) (0,1) (1,1) (1,0).  A phase of a wave is
//   L-segment: stage one half-tile (2 LDS-DMA per wave), read this phase's new operand fragments from LDS
//              (q0: A0 + B0 = 12 reads, q1: B1, q2: A1, q3: B0), s_waitcnt lgkmcnt(0) [, vmcnt at q3], s_barrier
//   M-segment: 16 MFMA 16x16x32 (the quadrant, K = 64) between s_setprio(1) / (0), s_barrier
// and group 1 runs one barrier behind group 0 (one extra s_barrier up front), so on every SIMD one wave's MFMA
// segment overlaps its partner's load segment: the matrix pipe alternates between the two waves.
//
// Hazards (a barrier is passed only when all 8 waves arrive; group 1's segment k coincides with group 0's k + 1):
//  * WAR: a staging half is re-staged one phase after its last read; the reading waves retire their reads
//    (lgkmcnt(0)) before the barrier that ends that L-segment, which every wave passes before its next L-segment.
//    Stage schedule in phase q of K-tile t: q0 B0(t + 1), q1 A0(t + 2), q2 B1(t + 2), q3 A1(t + 2)
//    (last reads of the same-parity halves: B0(t - 1) at q3 of t - 1, A0(t) q0, B1(t) q1, A1(t) q2).
//  * RAW: at q3 of K-tile t every wave waits vmcnt(6) -- three half-tiles (A0 / B1 / A1 of t + 2) stay in
//    flight, everything of K-tile t + 1 has landed -- before the barrier ending that L-segment; K-tile t + 1 is
//    first read in the next L-segment of either group, after that barrier.
#include "gemm_glds_body.h"

namespace {

constexpr int P8_BM = 256, P8_BN = 256, P8_BK = 64, P8_NW = 8, P8_NT = 512;
constexpr int P8_HALF = 128 * P8_BK * 2;  // one staging half-tile, bytes
constexpr int P8_BUF = 4 * P8_HALF;        // one K-tile: A0 A1 B0 B1
constexpr int P8_EPS = P8_BN + 4;          // fp32 epilogue row stride
constexpr int P8_ECH = 2;                  // epilogue row chunks (128 rows each = the quadrant row halves)
constexpr int P8_EPI_BYTES = P8_BM / P8_ECH * P8_EPS * 4;
constexpr int P8_BYTES = 2 * P8_BUF > P8_EPI_BYTES ? 2 * P8_BUF : P8_EPI_BYTES;
static_assert(P8_BYTES <= 160 * 1024, "LDS budget");

// runtime vmcnt(2 n) for n = 0..5 (an immediate is required; 2 LDS-DMA per half-tile)
__device__ __forceinline__ void wait_halves(int n) {
  if (n >= 5) asm volatile("s_waitcnt vmcnt(10)" ::: "memory");
  else if (n == 4) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  else if (n == 3) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  else if (n == 2) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  else if (n == 1) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// S = 0: the schedule of the header comment (one B quadrant in registers, re-staging one phase after the last read,
//        reads retired before the L-segment barrier).
// S = 1: both B quadrants stay in registers (B0 is not re-read at q3), so every staging half is last read at one
//        phase and re-staged two phases later: the reads retire after the barrier (their LDS latency overlaps the
//        partner group's MFMA segment) and each half is issued in the order the phases need it, waited for four
//        half-tiles later (vmcnt(8) every phase) -- ~5 phases between the DMA issue and the first read.
//        Per K-tile t: q0 (0,0) reads A0 + B0, stages B1(t+1); q1 (0,1) reads B1, stages A1(t+1); q2 (1,1) reads
//        A1, stages A0(t+2); q3 (1,0) reads nothing, stages B0(t+2).
template <bool AKM, bool BKM, int EPI, int S>
__global__ __launch_bounds__(P8_NT, 2) void gemm_8ph_kernel(G2Args p, int diag) {
  __shared__ __attribute__((aligned(16))) char smem[P8_BYTES];  // ONE LDS object (see gemm_glds.hip)
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = wave >> 2, c = wave & 3;
  const int tiles_n = p.N / P8_BN;
  const int t = xcd_remap(blockIdx.x, gridDim.x);
  int tm, tn;
  grouped_tile(t, p.M / P8_BM, tiles_n, tm, tn, p.group_m > 0 ? p.group_m : 8);
  const int m0 = tm * P8_BM, n0 = tn * P8_BN;
  const int nt = p.K / P8_BK;

  // accumulators: quadrant (qm, qn), 4 x 2 blocks of 16 x 16, transposed form (lane: row l & 15, 4 columns) for
  // the one-write-per-accumulator LDS epilogue
  f32x4 acc[2][2][4][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[a][b][i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // fused column sums of B (weight gradients, ``bsum``): group-0 waves of the first M-tile row add the B fragments
  // of their first read of each K-tile's B halves (q0: B0, q1: B1) -- every (k, column) once
  constexpr bool CS = AKM && BKM && (EPI == E_F32_ACC || EPI == E_F32_STORE);
  const bool do_cs = CS && p.bsum != nullptr && tm == 0 && g == 0;
  float cs[2][2] = {{0.f, 0.f}, {0.f, 0.f}};

  Stager<AKM, 128, P8_NW, P8_BK> stA0, stA1;
  Stager<BKM, 128, P8_NW, P8_BK> stB0, stB1;
  stA0.init(p.A, p.lda, m0, 0, wave, lane);
  stA1.init(p.A, p.lda, m0 + 128, 0, wave, lane);
  stB0.init(p.B, p.ldb, n0, 0, wave, lane);
  stB1.init(p.B, p.ldb, n0 + 128, 0, wave, lane);
  auto slot = [&](int kt, int h) -> char* { return smem + (kt & 1) * P8_BUF + h * P8_HALF; };  // h: 0 A0 1 A1 2 B0 3 B1

  if constexpr (S == 0) {
    // prologue: K-tile 0 whole, K-tile 1's A0 / B1 / A1 (B0 of K-tile 1 is staged by phase 0)
    stA0.stage(0, slot(0, 0));
    stA1.stage(0, slot(0, 1));
    stB0.stage(0, slot(0, 2));
    stB1.stage(0, slot(0, 3));
    if (nt > 1) {
      stA0.stage(1, slot(1, 0));
      stB1.stage(1, slot(1, 3));
      stA1.stage(1, slot(1, 1));
      asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
  } else {
    // prologue: the half-tiles in need order -- K-tile 0: A0 B0 B1 A1, K-tile 1: A0 B0 (index 4 u + {0..3});
    // phase p (= 4 t + q) then issues half 6 + p
    stA0.stage(0, slot(0, 0));
    stB0.stage(0, slot(0, 2));
    stB1.stage(0, slot(0, 3));
    stA1.stage(0, slot(0, 1));
    if (nt > 1) {
      stA0.stage(1, slot(1, 0));
      stB0.stage(1, slot(1, 2));
    }
    wait_halves((nt > 1 ? 5 : 3) - 1);  // A0 / B0 of K-tile 0 have landed
  }
  __builtin_amdgcn_s_barrier();
  if (g == 1 && !(diag & 2)) __builtin_amdgcn_s_barrier();  // the stagger: group 1 runs one barrier behind

  RawFrag<AKM> fa[4][2];   // A quadrant: 4 row blocks x 2 k-steps of 32
  RawFrag<BKM> fb[2][2];   // B quadrant (S = 0); S = 1: B0
  RawFrag<BKM> fb1[2][2];  // S = 1: B1

  for (int kt = 0; kt < nt; ++kt) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int qm = q >= 2, qn = q == 1 || q == 2;  // q0 (0,0) q1 (0,1) q2 (1,1) q3 (1,0)
      // ---------------- L-segment
      if constexpr (S == 0) {
        if (q == 0) {
          if (kt + 1 < nt) stB0.stage(kt + 1, slot(kt + 1, 2));
        } else if (q == 1) {
          if (kt + 2 < nt) stA0.stage(kt + 2, slot(kt + 2, 0));
        } else if (q == 2) {
          if (kt + 2 < nt) stB1.stage(kt + 2, slot(kt + 2, 3));
        } else {
          if (kt + 2 < nt) stA1.stage(kt + 2, slot(kt + 2, 1));
        }
      } else {
        if (q == 0) {
          if (kt + 1 < nt) stB1.stage(kt + 1, slot(kt + 1, 3));
        } else if (q == 1) {
          if (kt + 1 < nt) stA1.stage(kt + 1, slot(kt + 1, 1));
        } else if (q == 2) {
          if (kt + 2 < nt) stA0.stage(kt + 2, slot(kt + 2, 0));
        } else {
          if (kt + 2 < nt) stB0.stage(kt + 2, slot(kt + 2, 2));
        }
      }
      if (q == 0 || q == 2) {  // new A quadrant rows
        const char* img = slot(kt, qm);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int s = 0; s < 2; ++s) frag_issue<AKM, 128, P8_BK>(img, g * 64 + i * 16, s * 32, lane, fa[i][s]);
      }
      if constexpr (S == 0) {
        if (q != 2) {  // new B quadrant columns (q2 keeps q1's B1 fragments: B1 is re-staged in this very phase)
          const char* img = slot(kt, 2 + qn);
#pragma unroll
          for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int s = 0; s < 2; ++s) frag_issue<BKM, 128, P8_BK>(img, c * 32 + j * 16, s * 32, lane, fb[j][s]);
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (diag & 1) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (q == 3) {
          if (kt + 2 < nt) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
          else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
      } else {
        if (q < 2) {  // B0 at q0, B1 at q1: both stay in registers for the K-tile
          const char* img = slot(kt, 2 + q);
#pragma unroll
          for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int s = 0; s < 2; ++s)
              frag_issue<BKM, 128, P8_BK>(img, c * 32 + j * 16, s * 32, lane, q == 0 ? fb[j][s] : fb1[j][s]);
        }
        // RAW: the halves the NEXT phase reads (index R) must have landed; halves issued so far: 0 .. I
        const int pn = 4 * kt + q + 1;  // next phase
        const int qn1 = pn & 3, tn1 = pn >> 2;
        const int R = 4 * tn1 + (qn1 == 0 ? 1 : (qn1 == 1 ? 2 : 3));
        const int I = min(4 * kt + q + 6, 4 * nt - 1);
        wait_halves((diag & 1) ? 0 : max(0, I - R));
      }
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
      // ---------------- M-segment
      if constexpr (S == 1) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this phase's fragment reads (none at q3)
        __builtin_amdgcn_sched_barrier(0);
      }
      {
        bf16x8 a[4][2], b[2][2];
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int s = 0; s < 2; ++s) a[i][s] = frag_use<AKM>(fa[i][s]);
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int s = 0; s < 2; ++s) b[j][s] = frag_use<BKM>((S == 1 && qn == 1) ? fb1[j][s] : fb[j][s]);
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int s = 0; s < 2; ++s)
#pragma unroll
          for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j) acc[qm][qn][i][j] = mfma_tile<true>(a[i][s], b[j][s], acc[qm][qn][i][j]);
        __builtin_amdgcn_s_setprio(0);
        if constexpr (CS) {
          if (do_cs && q < 2) {
#pragma unroll
            for (int j = 0; j < 2; ++j)
#pragma unroll
              for (int s = 0; s < 2; ++s) {
                const i32x4 w = __builtin_bit_cast(i32x4, b[j][s]);
                float u = 0.f;
#pragma unroll
                for (int e = 0; e < 4; ++e)
                  u += __builtin_bit_cast(float, (unsigned)w[e] << 16) +
                       __builtin_bit_cast(float, (unsigned)w[e] & 0xffff0000u);
                cs[qn][j] += u;
              }
          }
        }
      }
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  if (g == 0 && !(diag & 2)) __builtin_amdgcn_s_barrier();  // balance the stagger barrier
  if constexpr (CS) {
    if (do_cs) {  // lane l's B fragment: column l & 15 of its block, k-rows 8 (l >> 4) + e: combine the 4 k-groups
#pragma unroll
      for (int qn = 0; qn < 2; ++qn)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          float v = cs[qn][j];
          v += __shfl_xor(v, 16);
          v += __shfl_xor(v, 32);
          if (lane < 16) atomicAdd(p.bsum + n0 + qn * 128 + c * 32 + j * 16 + lane, v);
        }
    }
  }
  // epilogue: chunk ch = the 128 rows of quadrant row half qm = ch
  glds_epilogue<P8_BM, P8_BN, EPI, P8_NT, P8_ECH, P8_EPS>(p, smem, m0, n0, blockIdx.x, [&](float* E, int ch) {
#pragma unroll
    for (int qm = 0; qm < 2; ++qm) {
      if (qm != ch) continue;
#pragma unroll
      for (int qn = 0; qn < 2; ++qn)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            const int row = g * 64 + i * 16 + (lane & 15);
            const int col = qn * 128 + c * 32 + j * 16 + 4 * (lane >> 4);
            *(f32x4*)(E + row * P8_EPS + col) = acc[qm][qn][i][j];
          }
    }
  });
}

// diagnostics (scripts/diag_8ph.py, scripts/bench_gemm_8ph.py): 1 vmcnt(0) every phase, 2 no stagger,
// 8 the two-B-register schedule S = 1 instead of the shipped S = 0 (S = 0 measured 0-6 % faster on the square and
// Llama-3-8B shapes, profiles/gemm_big_tiles_r5.txt)
int g_8ph_diag = 0;

template <bool AKM, bool BKM, int EPI>
hipError_t launch_8ph(const G2Args& a, hipStream_t s) {
  const int tiles = (a.M / P8_BM) * (a.N / P8_BN);
  if (g_8ph_diag & 8)
    hipLaunchKernelGGL((gemm_8ph_kernel<AKM, BKM, EPI, 1>), dim3(tiles), dim3(P8_NT), 0, s, a, g_8ph_diag);
  else
    hipLaunchKernelGGL((gemm_8ph_kernel<AKM, BKM, EPI, 0>), dim3(tiles), dim3(P8_NT), 0, s, a, g_8ph_diag);
  return hipGetLastError();
}

}  // namespace

IIT_EXPORT void iit_gemm_8ph_set_diag(int d) { g_8ph_diag = d; }

// 1 when the 8-phase kernel covers (shape, layout, epilogue): M, N multiples of 256, K of 64, no K split
IIT_EXPORT int iit_gemm_8ph_ok(int M, int N, int K, int mode, int epi) {
  if (M <= 0 || N <= 0 || K <= 0 || M % P8_BM || N % P8_BN || K % P8_BK) return 0;
  if (mode == 3) return epi == E_F32_ACC || epi == E_F32_STORE;
  if (mode == 0) return epi == E_BF16 || epi == E_F32_ACC || epi == E_F32_STORE || epi == E_DGELU || epi == E_DGELU_ERF;
  if (mode == 2)
    return epi == E_BF16 || epi == E_BF16_BIAS3 || epi == E_F32_RESID || epi == E_GELU || epi == E_GELU_ERF ||
           epi == E_F32_ACC || epi == E_F32_STORE;
  return 0;
}

// launch on a G2Args filled (and validated: operands, alignment, strides) by iit_gemm_glds_sm of gemm_glds.hip,
// passed as its bytes (the struct is defined once, in gemm_glds_body.h)
IIT_EXPORT int iit_gemm_8ph_run(const void* args, int mode, int epi, void* stream) {
  const G2Args& a = *(const G2Args*)args;
  hipStream_t s = (hipStream_t)stream;
#define P8(MODE, AK, BK_, EPI) \
  if (mode == (MODE) && epi == (EPI)) return (int)launch_8ph<AK, BK_, EPI>(a, s);
  P8(0, false, false, E_BF16)
  P8(0, false, false, E_F32_ACC)
  P8(0, false, false, E_F32_STORE)
  P8(0, false, false, E_DGELU)
  P8(0, false, false, E_DGELU_ERF)
  P8(2, false, true, E_BF16)
  P8(2, false, true, E_BF16_BIAS3)
  P8(2, false, true, E_F32_RESID)
  P8(2, false, true, E_GELU)
  P8(2, false, true, E_GELU_ERF)
  P8(2, false, true, E_F32_ACC)
  P8(2, false, true, E_F32_STORE)
  P8(3, true, true, E_F32_ACC)
  P8(3, true, true, E_F32_STORE)
#undef P8
  return (int)hipErrorInvalidValue;
}
