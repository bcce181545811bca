// Shared device code of the LDS-DMA MFMA GEMM (csrc/gemm_glds.hip documents the design): operand staging,
// fragment reads, tile order and the per-tile body ``gemm_glds_body``, used by the single-problem launches of
// gemm_glds.hip and the two-problem launches of gemm_dual.hip.
#pragma once
#include <type_traits>

#include "common.h"

namespace {

// E_BF16_CS: E_BF16 + per-tile column statistics of the stored (bf16-rounded) output into ``cstat`` -- the
// BatchNorm statistics of a convolution's output from its epilogue (csrc/conv_nhwc.hip, csrc/bn_nhwc.hip)
enum : int { E_BF16 = 0, E_BF16_BIAS3 = 1, E_F32_RESID = 2, E_GELU = 3, E_DGELU = 4, E_F32_ACC = 5,
             E_F32_STORE = 7, E_GELU_ERF = 8, E_DGELU_ERF = 9, E_BF16_CS = 10 };

struct G2Args {
  const __bf16* A;
  const __bf16* B;
  void* C;
  void* C2;
  const float* bias0;
  const float* bias1;
  const float* bias2;
  const float* resid;
  long lda, ldb, ldc, ldc2, ldr;
  int M, N, K, bias_cols;
  int k_per_split;  // split-K: blockIdx.y owns [y * k_per_split, (y + 1) * k_per_split); partials added atomically
  float* csum;      // E_DGELU: optional column sums of the stored output (the MLP input-bias gradient), += atomically
  // reduction split-K (fp32 accumulate / store epilogues, gridDim.y > 1): every split stores its partial tile to
  // ws[(split * tiles + tile) * BM * BN] and takes a ticket on counters[tile]; the last arriver sums the partials
  // in split order (deterministic) and runs the normal epilogue, then resets the ticket for the next launch
  float* ws;
  int* counters;
  // epilogue store flavour of the output tiles: 0 plain, 1 non-temporal (streamed past the caches), 2 write-through
  // (sc1: written to memory and dropped from the XCD's L2, so the kernel boundary has no dirty lines to write back)
  int store_mode;
  // timeline probe (nullable, diagnostic builds of the bench only): wave 0 of every workgroup records the shader
  // clock at the kernel's phases into prof[wg * 64 + e] -- e 0 start, 1 first K-tile landed, 2.. each later K-tile
  // landed, 61 main loop done, 62 epilogue stores drained; the 100 MHz wall clock at 63 (start) and 60 (end)
  long long* prof;
  int group_m;  // M-tiles per column group of the XCD-local tile order (0 = 8)
  // weight gradients (mode 3, fp32 epilogues): optional column sums of the B operand over the K range (the bias
  // gradient colsum(dY) of the layer whose dW = X^T dY this is), += atomically by the first M-tile row of tiles
  // from the B fragments already in registers, so dY is not read a second time
  float* bsum;
  // E_F32_STORE: optional sum of squares of the stored values (this weight gradient's share of the global gradient
  // norm the optimizer's clip needs), += atomically into one of 64 slots, so the norm pass can skip these gradients
  float* gsq;
  // implicit-GEMM convolution (csrc/conv_nhwc.hip): GEMM rows are the output pixels (n, h, w) of a conv_h x conv_w
  // image; an operand is gathered from the NHWC source activation [n][conv_sh][conv_sw][conv_c] through the
  // conv_k x conv_k taps with stride conv_s and padding conv_pad -- forward: source (s h + kh - pad, s w + kw - pad);
  // conv_flip (the input gradient, a transposed convolution): source ((h + pad - kh) / s, (w + pad - kw) / s) where
  // divisible.  Taps outside the source image read the 16-B-aligned zero page ``zero``.
  const __bf16* zero;
  int conv_h, conv_w, conv_c, conv_flip;
  int conv_sh, conv_sw, conv_k, conv_s, conv_pad;
  // E_BF16_CS: per-tile column statistics, channel-major over the M / BM row tiles T:
  // cstat[(k * N + col) * T + tm], k = 0 the tile's pivot (its first row's value), 1 sum(v - pivot), 2 sum((v - pivot)^2)
  // over the tile's BM rows -- plain stores, one writer per element (the consumer is the next launch)
  float* cstat;
};

__device__ __forceinline__ void prof_mark(long long* prof, int slot, int e, bool on) {
  if (on) prof[(long)slot * 64 + e] = clock64();
}

typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(3))) i16x4 lds_i16x4_t;
typedef const __attribute__((address_space(1))) void gbl_void_t;

__device__ __forceinline__ void glds16(const __bf16* g, char* lds_wave_base) {
  __builtin_amdgcn_global_load_lds((gbl_void_t*)g, (lds_void_t*)lds_wave_base, 16, 0, 0);
}

// swizzle of a k-major image: 32-B block index XOR f(k-row), chosen so the 16 k-rows {8g + q (+4)} of one
// transpose-read instruction land on 8 distinct 32-B bank slots of the 256-B bank window
template <int R>
__device__ __forceinline__ int kmaj_swz(int kr) {
  if constexpr (R == 128) return (kr & 3) | (((kr >> 3) & 1) << 2);  // 8 blocks per 256-B k-row
  else if constexpr (R == 64) return ((kr >> 1) & 1) | (((kr >> 3) & 1) << 1);  // 4 blocks per 128-B k-row
  else return (kr >> 3) & 1;  // R == 32: 2 blocks per 64-B k-row; k-rows 8g+q of one read -> 2 per bank slot
}

// swizzle of a k-contiguous image: the 16-B chunk slot XOR f(row), so the 16 rows one ds_read_b128 fragment read
// touches land on distinct 16-B bank slots (128-B rows: two rows per 256-B bank window; 256-B rows: one)
template <int BK>
__device__ __forceinline__ int kcont_swz(int row) {
  if constexpr (BK == 128) return row & 15;
  else if constexpr (BK == 32) return (row >> 2) & 3;  // 64-B rows: four rows per 256-B bank window
  else return (row >> 1) & 7;
}

// Stage one operand tile (R rows of the output dimension x BK k) into its LDS image with LDS-DMA.  The per-lane
// source pointers and LDS offsets are computed once per workgroup; staging K-tile kt then costs one 64-bit add per
// DMA instruction (the k offset is uniform).  LEAN keeps ONE per-lane pointer: with an even wave count the XOR
// swizzle of instruction i equals that of instruction 0, so instruction i's source is pointer 0 plus a wave-uniform
// stride (an SGPR add) -- N - 1 fewer VGPR pairs for the register-bound big tiles (gemm_4w.hip).
template <bool KMAJ, int R, int NW = 4, int BK = 64, bool LEAN = false>
struct Stager {
  // LDS-DMA instructions per wave per K-tile: one instruction moves 8 rows x 128 B (k-contiguous, BK = 64), 4 rows x
  // 256 B (BK = 128) or 64 / (R/8) k-rows (k-major); the NW waves of the workgroup split them
  static constexpr int RPI = 1024 / (BK * 2);  // k-contiguous rows per instruction
  static constexpr int N = KMAJ ? BK / (NW * (64 / (R / 8))) : R / (RPI * NW);
  static_assert(N >= 1, "tile too narrow for the workgroup's waves");
  static_assert(!LEAN || NW % 2 == 0, "the lean stager needs an even wave count");
  static constexpr int NP_ = LEAN ? 1 : N;
  const __bf16* ptr[NP_];
  int off[NP_];
  long kstep;  // elements between consecutive K-tiles
  long istep;  // LEAN: elements between consecutive instructions' sources
  int ostep;   // LEAN: bytes between consecutive instructions' LDS offsets

  __device__ __forceinline__ void init(const __bf16* base, long ld, int r0g, int kbeg, int wave, int lane) {
    if constexpr (!KMAJ) {
      // [R][BK] bf16; BK = 64: 128-B rows, one instruction = 8 rows x 8 chunks of 16 B, chunk c of row r at slot
      // c ^ ((r >> 1) & 7); BK = 128: 256-B rows, 4 rows x 16 chunks, chunk c at slot c ^ (r & 15)
      constexpr int CPR = BK / 8;  // 16-B chunks per row
#pragma unroll
      for (int i = 0; i < NP_; ++i) {
        const int r0 = i * RPI * NW + wave * RPI;
        const int row = r0 + lane / CPR;
        const int c = (lane % CPR) ^ kcont_swz<BK>(row);
        ptr[i] = base + (long)(r0g + row) * ld + kbeg + c * 8;
        off[i] = r0 * BK * 2;
      }
      kstep = BK;
      istep = (long)RPI * NW * ld;
      ostep = RPI * NW * BK * 2;
    } else {
      // [64][R] bf16, R*2-B k-rows; one instruction = (64 / (R/8)) k-rows
      constexpr int CH = R / 8;     // 16-B chunks per k-row
      constexpr int KRI = 64 / CH;  // k-rows per instruction
#pragma unroll
      for (int i = 0; i < NP_; ++i) {
        const int kr0 = (i * NW + wave) * KRI;
        const int kr = kr0 + lane / CH;
        const int ch = lane % CH;
        const int col = (((ch >> 1) ^ kmaj_swz<R>(kr)) << 4) + ((ch & 1) << 3);
        ptr[i] = base + (long)(kbeg + kr) * ld + r0g + col;
        off[i] = kr0 * R * 2;
      }
      kstep = (long)BK * ld;
      istep = (long)NW * KRI * ld;
      ostep = NW * KRI * R * 2;
    }
  }

  __device__ __forceinline__ void stage(int kt, char* img) const {
    const long k = kt * kstep;
#pragma unroll
    for (int i = 0; i < N; ++i) {
      if constexpr (LEAN) glds16(ptr[0] + (k + i * istep), img + off[0] + i * ostep);
      else glds16(ptr[i] + k, img + off[i]);
    }
  }
};

// MFMA 16x16x32 operand fragment: lane l gets X[row0 + (l & 15)][kbase + 8 * (l >> 4) + j], j = 0..7.
// The k-major (transpose-read) form is issued as inline asm: hipcc (ROCm 7.2) treats the ds_read_tr builtin as
// possibly aliasing every in-flight LDS-DMA and puts s_waitcnt vmcnt(0) in front of it, which would drain the
// prefetch ring each K-step.  The caller therefore waits lgkmcnt(0) + sched_barrier before using the registers.
__device__ __forceinline__ unsigned lds_addr(const char* p) {
  return (unsigned)(uintptr_t)(const __attribute__((address_space(3))) char*)p;
}

// Wide k-major operands (R > 128 columns, e.g. the 192-column B tile) are staged as R/64 independent 64-column
// panels, each its own [64][64] swizzled image (the k-major image layout above needs R/8 | 64); a k-major operand
// whose width is an odd multiple of 32 (the 96-column tiles) as R/32 panels of [64][32].
template <bool KMAJ, int R>
struct Panels {
  static constexpr bool ON = KMAJ && (R > 128 || R % 64 != 0);
  static constexpr int PR = !ON ? R : (R % 64 == 0 ? 64 : 32);  // columns per panel
  static constexpr int NP = R / PR;
};

template <bool KMAJ, int R, int NW = 4, int BK = 64, bool LEAN = false>
struct OperandStager {
  static constexpr bool PANELS = Panels<KMAJ, R>::ON;
  static constexpr int NP = Panels<KMAJ, R>::NP;
  static constexpr int PR = Panels<KMAJ, R>::PR;        // columns per panel
  static constexpr int N = NP * Stager<KMAJ, PR, NW, BK, LEAN>::N;  // LDS-DMA instructions per wave per K-tile
  Stager<KMAJ, PR, NW, BK, LEAN> st[NP];

  __device__ __forceinline__ void init(const __bf16* base, long ld, int r0g, int kbeg, int wave, int lane) {
#pragma unroll
    for (int q = 0; q < NP; ++q) st[q].init(base, ld, r0g + q * PR, kbeg, wave, lane);
  }
  __device__ __forceinline__ void stage(int kt, char* img) const {
#pragma unroll
    for (int q = 0; q < NP; ++q) st[q].stage(kt, img + q * PR * BK * 2);
  }
};

// Fragment reads are split into an *issue* (asm LDS reads into raw registers) and a *use* (combine into the
// MFMA operand) so the main loop can keep the next sub-step's reads in flight under the current MFMAs.  hipcc
// does not track asm-issued LDS reads, so the loop waits lgkmcnt(0) (+ sched_barrier) before any use.
typedef int i32x4 __attribute__((ext_vector_type(4)));
template <bool KMAJ> struct RawFrag;
template <> struct RawFrag<false> { i32x4 v; };
template <> struct RawFrag<true> { i16x4 lo, hi; };

template <bool KMAJ, int R, int BK = 64>
__device__ __forceinline__ void frag_issue(const char* img, int row0, int kbase, int lane, RawFrag<KMAJ>& f) {
  if constexpr (!KMAJ) {
    const int row = row0 + (lane & 15);
    const int c = (kbase >> 3) + (lane >> 4);
    const unsigned a = lds_addr(img + row * (BK * 2) + ((c ^ kcont_swz<BK>(row)) << 4));
    asm volatile("ds_read_b128 %0, %1" : "=v"(f.v) : "v"(a));
  } else {
    const int g = lane >> 4, q = (lane >> 2) & 3, pp = lane & 3;
    const int kr = kbase + 8 * g + q;
    const int col = row0 + 4 * pp;
    const unsigned a0 = lds_addr(img + kr * (R * 2) + ((((col >> 4) ^ kmaj_swz<R>(kr))) << 5) + ((col & 15) << 1));
    asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(f.lo) : "v"(a0));
    asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(f.hi) : "v"(a0), "i"(4 * R * 2));
  }
}

// fragment of rows/columns [row0, row0 + 16) of an operand tile staged by OperandStager<KMAJ, R>
template <bool KMAJ, int R, int BK = 64>
__device__ __forceinline__ void frag_issue_t(const char* img, int row0, int kbase, int lane, RawFrag<KMAJ>& f) {
  using PN = Panels<KMAJ, R>;
  if constexpr (PN::ON) {
    frag_issue<KMAJ, PN::PR, BK>(img + (row0 / PN::PR) * PN::PR * BK * 2, row0 % PN::PR, kbase, lane, f);
  } else {
    frag_issue<KMAJ, R, BK>(img, row0, kbase, lane, f);
  }
}

template <bool KMAJ>
__device__ __forceinline__ bf16x8 frag_use(const RawFrag<KMAJ>& f) {
  if constexpr (!KMAJ) {
    return __builtin_bit_cast(bf16x8, f.v);
  } else {
    const i16x8 w = __builtin_shufflevector(f.lo, f.hi, 0, 1, 2, 3, 4, 5, 6, 7);
    return __builtin_bit_cast(bf16x8, w);
  }
}

// One 16x16x32 product into an output block's accumulator.  TR = false: C = A B, lane l holds rows 4 (l >> 4) + r
// of column l & 15 (the MFMA's native layout).  TR = true: the operands enter swapped, the MFMA computes the block
// of C^T, so lane l holds row l & 15, COLUMNS 4 (l >> 4) + r -- four consecutive outputs of one row, which the
// epilogue moves into its row-major LDS tile with ONE 16-byte write per accumulator instead of four 4-byte ones.
template <bool TR>
__device__ __forceinline__ f32x4 mfma_tile(const bf16x8 a, const bf16x8 b, const f32x4 c) {
  if constexpr (TR) return __builtin_amdgcn_mfma_f32_16x16x32_bf16(b, a, c, 0, 0, 0);
  else return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int xcd = bid % 8;
  const int q = nwg / 8, r = nwg % 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + bid / 8;
}

// Tile order inside an XCD's contiguous range: column-major groups of up to GM M-tiles.  GM = 1 is the plain
// row-major order (an XCD runs whole rows of output tiles: each A row panel lives in one XCD's L2, the B column
// panels in all of them); larger GM makes each XCD's concurrent tiles a compact block that shares both (see the
// call site for the measured choice).
__device__ __forceinline__ void grouped_tile(int t, int tiles_m, int tiles_n, int& tm, int& tn, int GM = 8) {
  const int per_group = GM * tiles_n;
  const int first_m = (t / per_group) * GM;
  const int gsize = min(tiles_m - first_m, GM);
  const int r = t % per_group;
  tm = first_m + r % gsize;
  tn = r / gsize;
}

__device__ __forceinline__ float gelu_new_dev(float x) { return gelu_new_f(x); }

__device__ __forceinline__ void add8v(float* v, const float4 x, const float4 y) {
  v[0] += x.x; v[1] += x.y; v[2] += x.z; v[3] += x.w;
  v[4] += y.x; v[5] += y.y; v[6] += y.z; v[7] += y.w;
}

__device__ __forceinline__ void add8(float* v, const float* b) {
  const float4 x = *(const float4*)b, y = *(const float4*)(b + 4);
  v[0] += x.x; v[1] += x.y; v[2] += x.z; v[3] += x.w;
  v[4] += y.x; v[5] += y.y; v[6] += y.z; v[7] += y.w;
}

__device__ __forceinline__ void store16(void* dst, const f32x4 x, int mode) {
  if (mode == 1) {
    __builtin_nontemporal_store(x, (f32x4*)dst);
  } else if (mode == 2) {
    asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(dst), "v"(x) : "memory");
  } else {
    *(f32x4*)dst = x;
  }
}

__device__ __forceinline__ void store8_bf16(void* dst, const float* v, int mode = 0) {
  bf16x8 o;
#pragma unroll
  for (int e = 0; e < 8; ++e) o[e] = f2bf(v[e]);
  store16(dst, __builtin_bit_cast(f32x4, o), mode);
}

__device__ __forceinline__ void store8_f32(void* dst, const float* v, int mode = 0) {
  store16(dst, f32x4{v[0], v[1], v[2], v[3]}, mode);
  store16((float*)dst + 4, f32x4{v[4], v[5], v[6], v[7]}, mode);
}

// s_waitcnt vmcnt(N) with N chosen at run time from {0, L, ..., 7L} (an immediate is required; deep rings keep up
// to NS - 1 K-tiles in flight, capped by the 6-bit vmcnt)
template <int L>
__device__ __forceinline__ void wait_tiles(int tiles_in_flight) {
  constexpr int CAP = 63 / L;
  if (tiles_in_flight > CAP) tiles_in_flight = CAP;
  if (tiles_in_flight >= 7) asm volatile("s_waitcnt vmcnt(%0)" ::"n"((7 * L) < 63 ? 7 * L : 63) : "memory");
  else if (tiles_in_flight == 6) asm volatile("s_waitcnt vmcnt(%0)" ::"n"((6 * L) < 63 ? 6 * L : 63) : "memory");
  else if (tiles_in_flight == 5) asm volatile("s_waitcnt vmcnt(%0)" ::"n"((5 * L) < 63 ? 5 * L : 63) : "memory");
  else if (tiles_in_flight == 4) asm volatile("s_waitcnt vmcnt(%0)" ::"n"((4 * L) < 63 ? 4 * L : 63) : "memory");
  else if (tiles_in_flight == 3) asm volatile("s_waitcnt vmcnt(%0)" ::"n"((3 * L) < 63 ? 3 * L : 63) : "memory");
  else if (tiles_in_flight == 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * L) : "memory");
  else if (tiles_in_flight == 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(L) : "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// OCC = workgroups co-resident per CU the kernel is built for (LDS <= 160 KiB / OCC, registers <= 512 / OCC per lane
// for 4-wave groups): with OCC = 2 one workgroup's prologue / epilogue (operand fill, output stores) overlaps the
// other's MFMA main loop -- the per-launch fixed cost that one lock-stepped tile per CU leaves exposed.
template <int BM, int BN, int NS, int NW, int BK, int OCC>
struct GldsSmem {
  static constexpr int STAGE = (BM + BN) * BK * 2;
  static constexpr int EPS = BN + 4;
  static constexpr int LDS_BUDGET = 160 * 1024 / OCC;
  static constexpr int ECH = BM * EPS * 4 > LDS_BUDGET ? 2 : 1;
  static constexpr int EPI_BYTES = BM / ECH * EPS * 4;
  static constexpr int BYTES = NS * STAGE > EPI_BYTES ? NS * STAGE : EPI_BYTES;
};

// The epilogue of an output tile, shared by the LDS-DMA kernels: the fp32 accumulators go through LDS in ECH row
// chunks of BM / ECH rows (``write_acc(E, ch)`` stores this thread's accumulators of chunk ``ch`` into the row-major
// [BM / ECH][EPS] fp32 tile E), then each thread owns 8 consecutive columns of a row: 16-B / 32-B vector loads of
// bias / residual / accumulator and vector stores with the fused epilogue (bias, residual, gelu, dgelu + column sums,
// fp32 accumulate / store + sum of squares).
template <int BM, int BN, int EPI, int NT, int ECH, int EPS, class WriteAcc>
__device__ __forceinline__ void glds_epilogue(const G2Args& p, char* smem, const int m0, const int n0, const int lin,
                                              WriteAcc&& write_acc) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  constexpr int NW = NT / 64;
  float* E = (float*)smem;
  constexpr int ER = BM / ECH;  // rows per chunk
  constexpr int CPR = BN / 8;                      // 8-column chunks per row
  constexpr int ITEMS = (ER * CPR + NT - 1) / NT;  // chunks per thread per row chunk
  // the epilogue's streamed global operand (residual, accumulator, saved pre-activation) is loaded for all of a
  // thread's items up front, before the LDS tile is complete: ITEMS loads in flight instead of one per round trip
  constexpr bool PF32 = EPI == E_F32_RESID || EPI == E_F32_ACC;
  constexpr bool PF16 = EPI == E_DGELU || EPI == E_DGELU_ERF;
  float sq = 0.f;  // E_F32_STORE with ``gsq``: this thread's sum of squares of the stored values
  float cpiv = 0.f, cs1 = 0.f, cs2 = 0.f;  // E_BF16_CS: this thread's column group (pivot, sum d, sum d^2)
  for (int ch = 0; ch < ECH; ++ch) {
  float4 pf[PF32 ? 2 * ITEMS : 1];
  bf16x8 pb[PF16 ? ITEMS : 1];
#pragma unroll
  for (int k = 0; k < ITEMS; ++k) {
    const int id = tid + k * NT;
    if (id < ER * CPR) {
      const int row = m0 + ch * ER + id / CPR, col = n0 + (id % CPR) * 8;
      if constexpr (EPI == E_F32_RESID) {
        const float* src = p.resid + (long)row * p.ldr + col;
        pf[2 * k] = *(const float4*)src;
        pf[2 * k + 1] = *(const float4*)(src + 4);
      } else if constexpr (EPI == E_F32_ACC) {
        const float* src = (const float*)p.C + (long)row * p.ldc + col;
        pf[2 * k] = *(const float4*)src;
        pf[2 * k + 1] = *(const float4*)(src + 4);
      } else if constexpr (PF16) {
        pb[k] = *(const bf16x8*)((const __bf16*)p.C2 + (long)row * p.ldc2 + col);
      }
    }
  }
  __syncthreads();  // staging buffers / the previous chunk are done before the LDS is (re)written
  write_acc(E, ch);
  __syncthreads();
#pragma unroll
  for (int k = 0; k < ITEMS; ++k) {
    const int id = tid + k * NT;
    if (id >= ER * CPR) break;
    const int lr = id / CPR, lc = (id % CPR) * 8;
    const int row = m0 + ch * ER + lr, col = n0 + lc;
    float v[8];
    {
      const float4 x = *(const float4*)(E + lr * EPS + lc), y = *(const float4*)(E + lr * EPS + lc + 4);
      v[0] = x.x; v[1] = x.y; v[2] = x.z; v[3] = x.w; v[4] = y.x; v[5] = y.y; v[6] = y.z; v[7] = y.w;
    }
    if constexpr (EPI == E_BF16) {
      if (p.bias0) add8(v, p.bias0 + col);
      store8_bf16((__bf16*)p.C + (long)row * p.ldc + col, v, p.store_mode);
    } else if constexpr (EPI == E_BF16_CS) {
      if (p.bias0) add8(v, p.bias0 + col);
      store8_bf16((__bf16*)p.C + (long)row * p.ldc + col, v, p.store_mode);
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = bf2f(f2bf(v[e]));  // the statistics of what the consumer reads
      // this thread's own chunk of E: no other thread touches it before the barrier below
      *(float4*)(E + lr * EPS + lc) = make_float4(v[0], v[1], v[2], v[3]);
      *(float4*)(E + lr * EPS + lc + 4) = make_float4(v[4], v[5], v[6], v[7]);
    } else if constexpr (EPI == E_BF16_BIAS3) {
      const int w = col / p.bias_cols, o = col - w * p.bias_cols;
      const float* bb = w == 0 ? p.bias0 : (w == 1 ? p.bias1 : p.bias2);
      if (bb) add8(v, bb + o);
      store8_bf16((__bf16*)p.C + (long)row * p.ldc + col, v, p.store_mode);
    } else if constexpr (EPI == E_F32_RESID) {
      if (p.bias0) add8(v, p.bias0 + col);
      add8v(v, pf[2 * k], pf[2 * k + 1]);
      store8_f32((float*)p.C + (long)row * p.ldc + col, v, p.store_mode);
    } else if constexpr (EPI == E_GELU || EPI == E_GELU_ERF) {
      if (p.bias0) add8(v, p.bias0 + col);
      // pre (C2) is only kept for the backward: inference forwards pass C2 = null and skip its store
      if (p.C2) store8_bf16((__bf16*)p.C2 + (long)row * p.ldc2 + col, v, p.store_mode);
      float g[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) {  // gelu of the stored (bf16) pre, which the backward reads
        const float x = bf2f(f2bf(v[e]));
        g[e] = EPI == E_GELU ? gelu_new_dev(x) : gelu_erf_f(x);
      }
      store8_bf16((__bf16*)p.C + (long)row * p.ldc + col, g, p.store_mode);
    } else if constexpr (EPI == E_DGELU || EPI == E_DGELU_ERF) {
      const bf16x8 pr = pb[k];
#pragma unroll
      for (int e = 0; e < 8; ++e) {  // the stored value
        const float x = bf2f(pr[e]);
        v[e] = bf2f(f2bf(v[e] * (EPI == E_DGELU ? gelu_new_grad_f(x) : gelu_erf_grad_f(x))));
      }
      store8_bf16((__bf16*)p.C + (long)row * p.ldc + col, v, p.store_mode);
      if (p.csum) {  // this thread's own chunk of E: no other thread touches it before the barrier below
        *(float4*)(E + lr * EPS + lc) = make_float4(v[0], v[1], v[2], v[3]);
        *(float4*)(E + lr * EPS + lc + 4) = make_float4(v[4], v[5], v[6], v[7]);
      }
    } else if constexpr (EPI == E_F32_ACC) {
      float* dst = (float*)p.C + (long)row * p.ldc + col;
      add8v(v, pf[2 * k], pf[2 * k + 1]);
      store8_f32(dst, v, p.store_mode);
    } else {  // E_F32_STORE
      if (p.bias0) add8(v, p.bias0 + col);
      store8_f32((float*)p.C + (long)row * p.ldc + col, v, p.store_mode);
      if (p.gsq) {
#pragma unroll
        for (int e = 0; e < 8; ++e) sq += v[e] * v[e];
      }
    }
  }
  if constexpr (EPI == E_DGELU || EPI == E_DGELU_ERF) {
    if (p.csum) {  // column sums of this chunk's ER rows: G row groups per column, one atomic each
      __syncthreads();
      constexpr int G = NT / BN > 0 ? NT / BN : 1;
      for (int c = tid; c < BN * G; c += NT) {
        const int col = c % BN, g = c / BN;
        float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};  // 8 independent chains: the LDS reads pipeline
#pragma unroll
        for (int r0 = g; r0 < ER; r0 += 8 * G)
#pragma unroll
          for (int u = 0; u < 8; ++u)
            if (r0 + u * G < ER) s[u] += E[(r0 + u * G) * EPS + col];
        atomicAdd(p.csum + n0 + col, ((s[0] + s[1]) + (s[2] + s[3])) + ((s[4] + s[5]) + (s[6] + s[7])));
      }
    }
  }
  if constexpr (EPI == E_BF16_CS) {  // this chunk's rows into the thread's column-group sums (one group per thread)
    __syncthreads();
    static_assert(NT % BN == 0, "column groups");
    constexpr int G = NT / BN;
    const int col = tid % BN, g = tid / BN;
    if (ch == 0) cpiv = E[col];  // the tile's first row: the pivot (sums of v - pivot do not cancel)
    for (int r = g; r < ER; r += G) {
      const float d = E[r * EPS + col] - cpiv;
      cs1 += d;
      cs2 = __builtin_fmaf(d, d, cs2);
    }
  }
  }  // chunk
  if constexpr (EPI == E_BF16_CS) {  // the G groups of each column summed in a fixed order, one record per tile
    constexpr int G = NT / BN;
    float* red = (float*)smem;
    __syncthreads();  // every thread is done with the epilogue's LDS tile
    red[tid] = cs1;
    red[NT + tid] = cs2;
    __syncthreads();
    if (tid < BN) {
      float a = 0.f, b = 0.f;
#pragma unroll
      for (int g = 0; g < G; ++g) {
        a += red[g * BN + tid];
        b += red[NT + g * BN + tid];
      }
      const long T = p.M / BM, tm = m0 / BM, c = n0 + tid;
      p.cstat[c * T + tm] = cpiv;
      p.cstat[((long)p.N + c) * T + tm] = a;
      p.cstat[(2L * p.N + c) * T + tm] = b;
    }
  }
  if constexpr (EPI == E_F32_STORE) {
    if (p.gsq) {  // one atomic per workgroup (the waves' sums meet in LDS): thousands of tiles share 64 slots
      sq = wave_sum(sq);
      float* red = (float*)smem;
      __syncthreads();  // every thread is done with the epilogue's LDS tile
      if (lane == 0) red[wave] = sq;
      __syncthreads();
      if (tid == 0) {
        float t = 0.f;
#pragma unroll
        for (int w = 0; w < NW; ++w) t += red[w];
        atomicAdd(p.gsq + (lin & 63), t);
      }
    }
  }
}

// One output tile of one GEMM problem: workgroup ``lin`` of the ``nlin`` tiles of K-split ``split`` of ``nsplit``
// (a single-problem launch passes its block index and grid size; the dual launch in gemm_dual.hip maps its
// workgroups onto two problems).  ``smem`` is the launch's one LDS object of at least GldsSmem<...>::BYTES.
template <int BM, int BN, int NS, bool AKM, bool BKM, int EPI, int NW, int BK = 64, int OCC = 1, bool LEAN = false,
          class ASTG = void, class BSTG = void>
__device__ __forceinline__ void gemm_glds_body(const G2Args& p, const int lin, const int nlin, const int split,
                                               const int nsplit, char* smem) {
  // ASTG / BSTG: operand stagers other than the strided-matrix one (the convolution's implicit im2col rows /
  // columns); they take their geometry from ``p`` and must fill the same LDS image as OperandStager<...>
  using SA = std::conditional_t<std::is_void_v<ASTG>, OperandStager<AKM, BM, NW, BK, LEAN>, ASTG>;
  using SB = std::conditional_t<std::is_void_v<BSTG>, OperandStager<BKM, BN, NW, BK, LEAN>, BSTG>;
  constexpr int HALVES = BK / 64;  // a 128-deep K-tile is two 64-deep halves of two 32-deep MFMA sub-steps each
  constexpr int NT = NW * 64;                    // threads
  constexpr int WMR = NW / 2;                    // wave rows (waves form a WMR x 2 grid)
  constexpr int WM = BM / WMR, WN = BN / 2;
  constexpr int TM = WM / 16, TN = WN / 16;
  constexpr int A_BYTES = BM * BK * 2, B_BYTES = BN * BK * 2;
  constexpr int STAGE = A_BYTES + B_BYTES;
  constexpr int LOADS = SA::N + SB::N;  // DMA / wave / K-tile
  using SM = GldsSmem<BM, BN, NS, NW, BK, OCC>;
  constexpr int EPS = SM::EPS;  // fp32 epilogue row stride (floats)
  // the fp32 epilogue tile goes through LDS in row chunks (one per wave row) when the whole tile would not fit
  constexpr int ECH = SM::ECH;
  static_assert(SM::BYTES <= SM::LDS_BUDGET, "LDS budget");
  static_assert(STAGE == SM::STAGE, "stage size");

  // transposed accumulators (mfma_tile) for every epilogue that goes through the LDS tile; the atomic split-K
  // partials of E_F32_ACC keep the native layout (16 consecutive columns per lane group, 64-B atomic segments)
  constexpr bool TR = EPI != E_F32_ACC;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;  // wave (wm, wn) of the WMR x 2 grid
  const int tiles_n = p.N / BN;
  const int t = xcd_remap(lin, nlin);
  int tm, tn;
  // XCD-local order, 8-high column groups.  Whole rows of output tiles per XCD (group height 1: each activation
  // panel in ONE XCD's L2) are 3-8 % faster in isolation on every single-pass shape but 0.03-0.08 ms/step slower
  // inside the training step, same box (profiles/gemm_tile_order_r3.txt); ``group_m`` (IIT_GEMM_GROUP_M) overrides.
  grouped_tile(t, p.M / BM, tiles_n, tm, tn, p.group_m > 0 ? p.group_m : 8);
  const int m0 = tm * BM, n0 = tn * BN;
  const int kbeg = split * p.k_per_split;
  const int nt = p.k_per_split / BK;
  const bool prof_on = p.prof != nullptr && tid == 0;
  const int prof_slot = split * nlin + lin;
  if (prof_on) {
    p.prof[(long)prof_slot * 64 + 63] = wall_clock64();
    prof_mark(p.prof, prof_slot, 0, true);
  }

  f32x4 acc[TM][TN];
  // fused column sums of B (``bsum``): lane l's B fragment holds B[8 (l >> 4) + e][l & 15] of its 16-column block,
  // so the waves of the first wave row of the first M-tile row add their fragments' 8 values per lane on the VALU
  // (beside the MFMAs) into one float per block; the 4 k-groups are combined with lane shuffles at the end
  constexpr bool CS = AKM && BKM && (EPI == E_F32_ACC || EPI == E_F32_STORE);
  const bool do_cs = CS && p.bsum != nullptr && tm == 0 && wm == 0;  // wave-uniform
  float cs[CS ? TN : 1];
#pragma unroll
  for (int j = 0; j < (CS ? TN : 1); ++j) cs[j] = 0.f;
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // Software pipeline (one wave per SIMD, so the wave itself must hide the LDS latency):
  //  * LDS-DMA ring of NS K-tiles: slot kt % NS holds K-tile kt; NS tiles are staged up front and tile kt + NS
  //    is staged as soon as every wave has finished reading tile kt;
  //  * register double buffer: the fragments of the next 32-deep sub-step (possibly in the next K-tile) are
  //    issued before the 16 MFMAs of the current one, so their LDS latency hides under the matrix work;
  //  * one raw s_barrier per K-tile, placed before the last sub-step's MFMAs: it publishes tile kt+1 (every
  //    wave's counted vmcnt) and retires all reads of tile kt, so those MFMAs overlap the next DMA issue.
  RawFrag<AKM> ca[TM], na[TM];
  RawFrag<BKM> cb[TN], nb[TN];
  SA stA;
  SB stB;
  if constexpr (std::is_void_v<ASTG>) stA.init(p.A, p.lda, m0, kbeg, wave, lane);
  else stA.init(p, m0, kbeg, wave, lane);
  if constexpr (std::is_void_v<BSTG>) stB.init(p.B, p.ldb, n0, kbeg, wave, lane);
  else stB.init(p, n0, kbeg, wave, lane);
#pragma unroll
  for (int s = 0; s < NS; ++s)
    if (s < nt) {
      char* buf = smem + s * STAGE;
      stA.stage(s, buf);
      stB.stage(s, buf + A_BYTES);
    }
  wait_tiles<LOADS>(min(NS - 1, nt - 1));
  __builtin_amdgcn_s_barrier();
  prof_mark(p.prof, prof_slot, 1, prof_on);
#pragma unroll
  for (int i = 0; i < TM; ++i) frag_issue_t<AKM, BM, BK>(smem, wm * WM + i * 16, 0, lane, ca[i]);
#pragma unroll
  for (int j = 0; j < TN; ++j) frag_issue_t<BKM, BN, BK>(smem + A_BYTES, wn * WN + j * 16, 0, lane, cb[j]);

  for (int kt = 0; kt < nt; ++kt) {
    const char* sa = smem + (kt % NS) * STAGE;
    const char* sb = sa + A_BYTES;
#pragma unroll
    for (int h = 0; h < HALVES; ++h) {
    // ---- sub-step 0 of half h of tile kt: operands in ca/cb; issue sub-step 1 into na/nb
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int i = 0; i < TM; ++i) frag_issue_t<AKM, BM, BK>(sa, wm * WM + i * 16, h * 64 + 32, lane, na[i]);
#pragma unroll
    for (int j = 0; j < TN; ++j) frag_issue_t<BKM, BN, BK>(sb, wn * WN + j * 16, h * 64 + 32, lane, nb[j]);
    __builtin_amdgcn_sched_barrier(0);
    {
      bf16x8 a[TM], b[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) a[i] = frag_use<AKM>(ca[i]);
#pragma unroll
      for (int j = 0; j < TN; ++j) b[j] = frag_use<BKM>(cb[j]);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = mfma_tile<TR>(a[i], b[j], acc[i][j]);
      if constexpr (CS) {
        if (do_cs) {
#pragma unroll
          for (int j = 0; j < TN; ++j) {
            const i32x4 w = __builtin_bit_cast(i32x4, b[j]);
            float t = 0.f;
#pragma unroll
            for (int q = 0; q < 4; ++q)
              t += __builtin_bit_cast(float, (unsigned)w[q] << 16) + __builtin_bit_cast(float, (unsigned)w[q] & 0xffff0000u);
            cs[j] += t;
          }
        }
      }
    }
    __builtin_amdgcn_sched_barrier(0);
    // ---- sub-step 1: operands in na/nb; issue the next half of this tile into ca/cb, or (last half) publish tile
    // kt+1, restage slot kt % NS and issue (kt+1, 0) into ca/cb
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    if (h + 1 < HALVES) {
#pragma unroll
      for (int i = 0; i < TM; ++i) frag_issue_t<AKM, BM, BK>(sa, wm * WM + i * 16, (h + 1) * 64, lane, ca[i]);
#pragma unroll
      for (int j = 0; j < TN; ++j) frag_issue_t<BKM, BN, BK>(sb, wn * WN + j * 16, (h + 1) * 64, lane, cb[j]);
    } else if (kt + 1 < nt) {
      wait_tiles<LOADS>(min(NS - 2, nt - 2 - kt));
      __builtin_amdgcn_s_barrier();
      if (kt + 2 < 61) prof_mark(p.prof, prof_slot, kt + 2, prof_on);
      if (kt + NS < nt) {
        char* buf = smem + (kt % NS) * STAGE;
        stA.stage(kt + NS, buf);
        stB.stage(kt + NS, buf + A_BYTES);
      }
      const char* ta = smem + ((kt + 1) % NS) * STAGE;
#pragma unroll
      for (int i = 0; i < TM; ++i) frag_issue_t<AKM, BM, BK>(ta, wm * WM + i * 16, 0, lane, ca[i]);
#pragma unroll
      for (int j = 0; j < TN; ++j) frag_issue_t<BKM, BN, BK>(ta + A_BYTES, wn * WN + j * 16, 0, lane, cb[j]);
    }
    __builtin_amdgcn_sched_barrier(0);
    {
      bf16x8 a[TM], b[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) a[i] = frag_use<AKM>(na[i]);
#pragma unroll
      for (int j = 0; j < TN; ++j) b[j] = frag_use<BKM>(nb[j]);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = mfma_tile<TR>(a[i], b[j], acc[i][j]);
      if constexpr (CS) {
        if (do_cs) {
#pragma unroll
          for (int j = 0; j < TN; ++j) {
            const i32x4 w = __builtin_bit_cast(i32x4, b[j]);
            float t = 0.f;
#pragma unroll
            for (int q = 0; q < 4; ++q)
              t += __builtin_bit_cast(float, (unsigned)w[q] << 16) + __builtin_bit_cast(float, (unsigned)w[q] & 0xffff0000u);
            cs[j] += t;
          }
        }
      }
    }
    __builtin_amdgcn_sched_barrier(0);
    }  // half
  }
  prof_mark(p.prof, prof_slot, 61, prof_on);
  if constexpr (CS) {
    if (do_cs) {
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        float v = cs[j];
        v += __shfl_xor(v, 16);
        v += __shfl_xor(v, 32);
        if (lane < 16) atomicAdd(p.bsum + n0 + wn * WN + j * 16 + lane, v);
      }
    }
  }
  if constexpr (EPI == E_F32_ACC || EPI == E_F32_STORE || EPI == E_F32_RESID || EPI == E_BF16 || EPI == E_BF16_CS) {
    if (p.ws != nullptr) {
      // Partial tile in MFMA register order (one 16-B chunk per lane per accumulator: 1 KiB coalesced per wave),
      // published without any L2 writeback / invalidate: write-through (sc1) stores, drained with vmcnt(0) before
      // the ticket, and sc1 loads on the reading side (the XCDs' L2s are not coherent with each other; a
      // device-scope fence here would write back / invalidate whole L2s under every other tile's main loop).
      const long tile_elems = (long)BM * BN;
      f32x4* mine = (f32x4*)(p.ws + ((long)split * nlin + t) * tile_elems);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(mine + (i * TN + j) * NT + tid), "v"(acc[i][j])
                       : "memory");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();  // every thread's partial has landed; also retires the main loop's LDS use
      int* flag = (int*)smem;
      if (tid == 0) {
        const int last = atomicAdd(p.counters + t, 1) == nsplit - 1;
        // every split has arrived: re-arm the ticket for the next launch (a device-coherent store, like the ticket)
        if (last) __hip_atomic_store(p.counters + t, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        flag[0] = last;
      }
      __syncthreads();
      if (!flag[0]) return;
      f32x4 sum[TM][TN];
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) sum[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
      for (int sp = 0; sp < nsplit; ++sp) {  // fixed order: bit-identical whoever arrives last
        if (sp == split) {
#pragma unroll
          for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j) sum[i][j] += acc[i][j];
          continue;
        }
        const f32x4* other = (const f32x4*)(p.ws + ((long)sp * nlin + t) * tile_elems);
        f32x4 v[TM][TN];
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            asm volatile("global_load_dwordx4 %0, %1, off sc1" : "=v"(v[i][j]) : "v"(other + (i * TN + j) * NT + tid)
                         : "memory");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j) sum[i][j] += v[i][j];
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = sum[i][j];
    }
  }
  if constexpr (EPI == E_F32_ACC) {
    if (nsplit > 1 && p.ws == nullptr) {  // split-K partial: atomics straight from the MFMA layout (16 lanes = 16 consecutive
                          // columns, so each wave instruction hits 4 rows x 64 B)
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const int col = n0 + wn * WN + j * 16 + (lane & 15);
          const int row = m0 + wm * WM + i * 16 + 4 * (lane >> 4);
#pragma unroll
          for (int r = 0; r < 4; ++r) unsafeAtomicAdd((float*)p.C + (long)(row + r) * p.ldc + col, acc[i][j][r]);
        }
      return;
    }
  }
  // ---------------------------------------------------------------- epilogue via LDS (ECH row chunks)
  glds_epilogue<BM, BN, EPI, NT, ECH, SM::EPS>(p, smem, m0, n0, lin, [&](float* E, int ch) {
    if (wm / (WMR / ECH) == ch) {
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          if constexpr (TR) {  // lane: row l & 15, columns 4 (l >> 4) .. + 3 -> one 16-B LDS write
            const int col = wn * WN + j * 16 + 4 * (lane >> 4);
            const int row = (wm % (WMR / ECH)) * WM + i * 16 + (lane & 15);
            *(f32x4*)(E + row * EPS + col) = acc[i][j];
          } else {
            const int col = wn * WN + j * 16 + (lane & 15);
            const int row = (wm % (WMR / ECH)) * WM + i * 16 + 4 * (lane >> 4);
#pragma unroll
            for (int r = 0; r < 4; ++r) E[(row + r) * EPS + col] = acc[i][j][r];
          }
        }
    }
  });
  if (p.prof != nullptr) {  // drain this workgroup's stores, then stamp (diagnostic path only)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    prof_mark(p.prof, prof_slot, 62, prof_on);
    if (prof_on) p.prof[(long)prof_slot * 64 + 60] = wall_clock64();
  }
}

}  // namespace
