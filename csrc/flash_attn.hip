// Tiled (flash-style) attention for long sequences on gfx950 MFMA: forward + backward, causal or bidirectional,
// grouped-query heads (Hkv divides Hq), head dims 64 and 128, and the interchange-splice head mask of the
// short-sequence kernel (csrc/attn_mfma.hip): heads in ``head_mask`` take z := src and get zero q/k/v gradients.
//
// Never materialises [S, S]: 64x64 score tiles live in registers, the softmax is the online (running max / sum)
// form, and the backward recomputes P from the saved log-sum-exp (SURVEY.md §2.3 K04, §7.3 kernel 3).
//
// All products are v_mfma_f32_16x16x32_bf16 tiles.  Layouts (lane l = 16 g + c):
//   A fragment  X[m0 + c][k0 + 8g + j]        (16-B LDS row read, or straight from global memory)
//   B fragment  Y[k0 + 8g + j][n0 + c]
//   C           lane holds rows m0 + 4g + r (r = 0..3) of column n0 + c
// A C tile over two consecutive 16-row blocks (rows 4g+r and 16+4g+r) becomes the B operand of the next product
// with no lane movement when that product's reduction index is permuted the same way, kk(g, j) = 4g + j (j < 4),
// 16 + 4g + (j - 4) (j >= 4); the partner A operand is read transposed from LDS with ds_read_b64_tr_b16 at exactly
// those rows (frag_tr_perm).  That keeps P / dS in registers:
//   forward   S^T = K Q^T (keys x queries), online softmax per query column, O^T += V^T P^T
//   dK, dV    S = Q K^T, dP = dO V^T (queries x keys), dS = P (dP - D); dV^T += dO^T P, dK^T += Q^T dS
//   dQ        S^T = K Q^T, dP^T = V dO^T, dS^T = P^T (dP^T - D); dQ^T += K^T dS^T
// with D = rowsum(dO o O) from a small prep kernel.  dK/dV workgroups own 64 keys of one KV head and loop over every
// query head of its group (GQA needs no atomics); dQ workgroups own 64 queries.
//
// General interchange splice of ``hook_z`` (``use_sp``; any patch-spec index over z [B][S][Hq][dh], the range table
// of csrc/splice_spec.h): the forward's output store writes the source's value into the spliced elements (no separate
// splice pass over z), and every backward load of dO zeroes the spliced elements (the spliced z is a constant: its
// elements carry no gradient into q / k / v) -- the prep kernel's D = rowsum(dO o O), the dK/dV kernel's dO tiles and
// the dQ kernel's dO fragments, so no masked copy of dO is written either.
#include "common.h"
#include "splice_spec.h"
#include <stdlib.h>

typedef __attribute__((address_space(3))) i16x4 lds_i16x4_t;

namespace {

struct FaArgs {
  const __bf16* q; const __bf16* k; const __bf16* v;
  long qb, qs, qh, kb, ks, kh, vb, vs, vh;           // element strides (batch, position, head); unit stride on d
  __bf16* z; long zb, zs, zh;                        // forward output
  float* lse;                                        // [B][Hq][S] (scaled units)
  const __bf16* src; long sb, ss, sh;                // splice source, z layout
  unsigned long long head_mask;
  const __bf16* dz; long db, ds, dh_;                // backward: dO
  float* dd;                                         // D = rowsum(dO o O), [B][Hq][S]
  __bf16* dq; __bf16* dk; __bf16* dv;
  long gqb, gqs, gqh, gkb, gks, gkh, gvb, gvs, gvh;  // gradient strides
  int B, S, Hq, Hkv, causal;
  float scale;
  int use_sp;     // general z splice: sp over [B][S][Hq][dh], source a.src with sp.sstride element strides
  SpliceSpec sp;
};

// is (b, row, h) of z inside the splice's first three dimensions
__device__ __forceinline__ bool sp_row(const FaArgs& a, int b, int row, int h) {
  return a.use_sp && in_ranges(a.sp, 0, b) && in_ranges(a.sp, 1, row) && in_ranges(a.sp, 2, h);
}

// dO elements d0 .. d0 + 7 of a row inside the splice (``row_in``) read as zero
__device__ __forceinline__ bf16x8 sp_mask8(bf16x8 v, const FaArgs& a, bool row_in, int d0) {
  if (!row_in) return v;
  i16x8 w = __builtin_bit_cast(i16x8, v);
#pragma unroll
  for (int e = 0; e < 8; ++e)
    if (in_ranges(a.sp, 3, d0 + e)) w[e] = 0;
  return __builtin_bit_cast(bf16x8, w);
}

constexpr int T64 = 64;

// [64][DH] bf16 LDS image, 16-B chunks XOR-swizzled per row (conflict-free 16-B row reads)
template <int DH>
__device__ __forceinline__ int ioff(int row, int col) {
  const int sw = DH == 64 ? ((row >> 1) & 7) : (row & 15);
  return row * DH + ((((col >> 3) ^ sw) << 3) | (col & 7));
}

template <int DH>
__device__ __forceinline__ void load_tile(__bf16* img, const __bf16* base, long stride, int r0, int S, int tid) {
  constexpr int CPR = DH / 8;
#pragma unroll
  for (int i = tid; i < T64 * CPR; i += 256) {
    const int r = i / CPR, ch = i % CPR;
    uint4 val = make_uint4(0u, 0u, 0u, 0u);
    if (r0 + r < S) val = *(const uint4*)(base + (long)(r0 + r) * stride + ch * 8);
    *(uint4*)(img + ioff<DH>(r, ch * 8)) = val;
  }
}

// load_tile of dO rows with the splice mask applied (rows r0.. of batch b, query head h)
template <int DH>
__device__ __forceinline__ void load_tile_dz(__bf16* img, const __bf16* base, long stride, int r0, int S, int tid,
                                             const struct FaArgs& a, int b, int h);

__device__ __forceinline__ bf16x8 zero8() {
  const i16x8 z = {0, 0, 0, 0, 0, 0, 0, 0};
  return __builtin_bit_cast(bf16x8, z);
}

__device__ __forceinline__ bf16x8 gload8(const __bf16* p, bool ok) { return ok ? *(const bf16x8*)p : zero8(); }

template <int DH>
__device__ __forceinline__ void load_tile_dz(__bf16* img, const __bf16* base, long stride, int r0, int S, int tid,
                                             const FaArgs& a, int b, int h) {
  constexpr int CPR = DH / 8;
#pragma unroll
  for (int i = tid; i < T64 * CPR; i += 256) {
    const int r = i / CPR, ch = i % CPR;
    bf16x8 val = zero8();
    if (r0 + r < S) val = sp_mask8(*(const bf16x8*)(base + (long)(r0 + r) * stride + ch * 8), a, sp_row(a, b, r0 + r, h), ch * 8);
    *(bf16x8*)(img + ioff<DH>(r, ch * 8)) = val;
  }
}

template <int DH>
__device__ __forceinline__ bf16x8 frag_rows(const __bf16* img, int m0, int k0, int lane) {
  return *(const bf16x8*)(img + ioff<DH>(m0 + (lane & 15), k0 + 8 * (lane >> 4)));
}

// lane receives X[kk(g, j)][n0 + c] of the [64][DH] image X, kk permuted as in the header (rows kb + ...)
template <int DH>
__device__ __forceinline__ bf16x8 frag_tr_perm(const __bf16* img, int kb, int n0, int lane) {
  const int g = lane >> 4, q = (lane >> 2) & 3, pp = lane & 3;
  const int col = n0 + 4 * pp;
  const i16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_i16x4_t*)(img + ioff<DH>(kb + 4 * g + q, col)));
  const i16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_i16x4_t*)(img + ioff<DH>(kb + 16 + 4 * g + q, col)));
  return __builtin_bit_cast(bf16x8, (i16x8)__builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
}

__device__ __forceinline__ bf16x8 pack_perm(const float* a, const float* b) {
  bf16x8 o = {f2bf(a[0]), f2bf(a[1]), f2bf(a[2]), f2bf(a[3]), f2bf(b[0]), f2bf(b[1]), f2bf(b[2]), f2bf(b[3])};
  return o;
}

__device__ __forceinline__ f32x4 mfma(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ void store4(__bf16* dst, const f32x4 v, float s) {
  bf16x4 o = {f2bf(v[0] * s), f2bf(v[1] * s), f2bf(v[2] * s), f2bf(v[3] * s)};
  *(bf16x4*)dst = o;
}

// ------------------------------------------------------------------------------------------------ forward
// Each wave owns QB blocks of 16 queries (QB * 64 queries per workgroup): every K / V fragment read from LDS feeds
// QB MFMAs, halving (QB = 2) the LDS traffic per FLOP -- with one 16-query block per wave the kernel is LDS-bound
// (16 x 64 x DH MACs per 2 x 64 x DH x 2 bytes read).  Softmax runs in the log2 domain (scale * log2(e) folded
// into one multiply, exp2 on the hardware v_exp_f32); the saved log-sum-exp is converted back to natural units.
constexpr float kLog2e = 1.4426950408889634f;
constexpr float kLn2 = 0.6931471805599453f;

template <int DH, int QB>
__global__ __launch_bounds__(256, 2) void fa_fwd_kernel(FaArgs a) {
  __shared__ __attribute__((aligned(16))) __bf16 Ks[T64 * DH];
  __shared__ __attribute__((aligned(16))) __bf16 Vs[T64 * DH];
  const int tid = threadIdx.x, wave = tid >> 6, l = tid & 63, g = l >> 4, c = l & 15;
  const int qblk = blockIdx.x, h = blockIdx.y, b = blockIdx.z;
  const int S = a.S;
  constexpr int QW = T64 * QB;  // queries per workgroup
  const int q0 = qblk * QW + 16 * QB * wave;  // this wave's first query; block j covers q0 + 16 j + [0, 16)
  if ((a.head_mask >> h) & 1ull) {  // spliced head: z := src, lse unused by the backward (zero gradients)
    constexpr int CPR = DH / 8;
    for (int i = tid; i < QW * CPR; i += 256) {
      const int r = qblk * QW + i / CPR, ch = i % CPR;
      if (r < S)
        *(uint4*)(a.z + b * a.zb + (long)r * a.zs + h * a.zh + ch * 8) =
            *(const uint4*)(a.src + b * a.sb + (long)r * a.ss + h * a.sh + ch * 8);
    }
    return;
  }
  const int hk = h / (a.Hq / a.Hkv);
  const __bf16* kbase = a.k + b * a.kb + hk * a.kh;
  const __bf16* vbase = a.v + b * a.vb + hk * a.vh;
  const float sl2 = a.scale * kLog2e;
  bf16x8 qf[QB][DH / 32];
  f32x4 o[QB][DH / 16];
  float m[QB], lsum[QB];  // running max (log2 units) of column qi; this lane's partial sum
#pragma unroll
  for (int j = 0; j < QB; ++j) {
    const int qi = q0 + 16 * j + c;
#pragma unroll
    for (int s = 0; s < DH / 32; ++s)
      qf[j][s] = gload8(a.q + b * a.qb + (long)qi * a.qs + h * a.qh + 32 * s + 8 * g, qi < S);
#pragma unroll
    for (int t = 0; t < DH / 16; ++t) o[j][t] = f32x4{0.f, 0.f, 0.f, 0.f};
    m[j] = -INFINITY;
    lsum[j] = 0.f;
  }
  const int kend = a.causal ? min(S, (qblk + 1) * QW) : S;
  for (int k0 = 0; k0 < kend; k0 += T64) {
    __syncthreads();
    load_tile<DH>(Ks, kbase, a.ks, k0, S, tid);
    load_tile<DH>(Vs, vbase, a.vs, k0, S, tid);
    __syncthreads();
    if (a.causal && k0 > q0 + 16 * QB - 1) continue;  // every key of this tile is after this wave's queries
    float p[QB][4][4];
    float mb[QB];
#pragma unroll
    for (int j = 0; j < QB; ++j) mb[j] = -INFINITY;
#pragma unroll
    for (int kb4 = 0; kb4 < 4; ++kb4) {
      f32x4 acc[QB];
#pragma unroll
      for (int j = 0; j < QB; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < DH / 32; ++s) {
        const bf16x8 kf = frag_rows<DH>(Ks, 16 * kb4, 32 * s, l);
#pragma unroll
        for (int j = 0; j < QB; ++j) acc[j] = mfma(kf, qf[j][s], acc[j]);
      }
#pragma unroll
      for (int j = 0; j < QB; ++j) {
        const int qi = q0 + 16 * j + c;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int kj = k0 + 16 * kb4 + 4 * g + r;
          const bool ok = kj < S && (!a.causal || kj <= qi);
          p[j][kb4][r] = ok ? acc[j][r] * sl2 : -INFINITY;
          mb[j] = fmaxf(mb[j], p[j][kb4][r]);
        }
      }
    }
#pragma unroll
    for (int j = 0; j < QB; ++j) {
      mb[j] = fmaxf(mb[j], __shfl_xor(mb[j], 16, 64));
      mb[j] = fmaxf(mb[j], __shfl_xor(mb[j], 32, 64));
      const float mn = fmaxf(m[j], mb[j]);
      const float alpha = mn == -INFINITY ? 1.f : __builtin_amdgcn_exp2f(m[j] - mn);
      m[j] = mn;
      lsum[j] *= alpha;
#pragma unroll
      for (int t = 0; t < DH / 16; ++t) o[j][t] *= alpha;
#pragma unroll
      for (int kb4 = 0; kb4 < 4; ++kb4)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float e = p[j][kb4][r] == -INFINITY ? 0.f : __builtin_amdgcn_exp2f(p[j][kb4][r] - mn);
          p[j][kb4][r] = e;
          lsum[j] += e;
        }
    }
#pragma unroll
    for (int ch = 0; ch < 2; ++ch) {
      bf16x8 pb[QB];
#pragma unroll
      for (int j = 0; j < QB; ++j) pb[j] = pack_perm(p[j][2 * ch], p[j][2 * ch + 1]);
#pragma unroll
      for (int t = 0; t < DH / 16; ++t) {
        const bf16x8 vf = frag_tr_perm<DH>(Vs, 32 * ch, 16 * t, l);
#pragma unroll
        for (int j = 0; j < QB; ++j) o[j][t] = mfma(vf, pb[j], o[j][t]);
      }
    }
  }
#pragma unroll
  for (int j = 0; j < QB; ++j) {
    float ls = lsum[j];
    ls += __shfl_xor(ls, 16, 64);
    ls += __shfl_xor(ls, 32, 64);
    const int qi = q0 + 16 * j + c;
    if (qi < S) {
      const float inv = ls > 0.f ? 1.f / ls : 0.f;
      __bf16* zr = a.z + b * a.zb + (long)qi * a.zs + h * a.zh;
      if (sp_row(a, b, qi, h)) {  // spliced row of z: the source's value in the spliced elements
        const __bf16* sr = a.src + b * a.sp.sstride[0] + (long)qi * a.sp.sstride[1] + h * a.sp.sstride[2];
#pragma unroll
        for (int t = 0; t < DH / 16; ++t) {
          bf16x4 ov;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int d = 16 * t + 4 * g + e;
            ov[e] = in_ranges(a.sp, 3, d) ? sr[d * a.sp.sstride[3]] : f2bf(o[j][t][e] * inv);
          }
          *(bf16x4*)(zr + 16 * t + 4 * g) = ov;
        }
      } else {
#pragma unroll
        for (int t = 0; t < DH / 16; ++t) store4(zr + 16 * t + 4 * g, o[j][t], inv);
      }
      if (g == 0 && a.lse) a.lse[((long)b * a.Hq + h) * S + qi] = (m[j] + __log2f(ls)) * kLn2;
    }
  }
}

// ------------------------------------------------------------------------------------------------ backward
// D[b][h][i] = sum_d dO[i][d] * O[i][d]  (one thread per row)
template <int DH>
__global__ __launch_bounds__(256) void fa_bwd_prep_kernel(FaArgs a) {
  const long row = (long)blockIdx.x * 256 + threadIdx.x;
  const long rows = (long)a.B * a.Hq * a.S;
  if (row >= rows) return;
  const int i = row % a.S;
  const int h = (row / a.S) % a.Hq;
  const int b = row / ((long)a.S * a.Hq);
  const __bf16* o = a.z + b * a.zb + (long)i * a.zs + h * a.zh;
  const __bf16* g = a.dz + b * a.db + (long)i * a.ds + h * a.dh_;
  float acc = 0.f;
  const bool row_in = sp_row(a, b, i, h);
#pragma unroll
  for (int ch = 0; ch < DH / 8; ++ch) {
    const bf16x8 x = *(const bf16x8*)(o + ch * 8), y = sp_mask8(*(const bf16x8*)(g + ch * 8), a, row_in, ch * 8);
#pragma unroll
    for (int e = 0; e < 8; ++e) acc += bf2f(x[e]) * bf2f(y[e]);
  }
  a.dd[row] = acc;
}

// dK / dV: each wave owns NB blocks of 16 keys, so every Q / dO fragment read from LDS feeds NB MFMAs (NB = 2 halves
// the LDS traffic per FLOP, as in the forward).
template <int DH, int NB>
__global__ __launch_bounds__(256, 2) void fa_bwd_dkdv_kernel(FaArgs a) {
  __shared__ __attribute__((aligned(16))) __bf16 Qs[T64 * DH];
  __shared__ __attribute__((aligned(16))) __bf16 Gs[T64 * DH];
  __shared__ float Ls[T64], Ds[T64];
  const int tid = threadIdx.x, wave = tid >> 6, l = tid & 63, g = l >> 4, c = l & 15;
  const int kblk = blockIdx.x, hk = blockIdx.y, b = blockIdx.z;
  const int S = a.S, rep = a.Hq / a.Hkv;
  constexpr int KW = T64 * NB;  // keys per workgroup
  const int k0 = kblk * KW + 16 * NB * wave;  // this wave's first key; block j covers k0 + 16 j + [0, 16)
  bf16x8 kf[NB][DH / 32], vf[NB][DH / 32];
  f32x4 dk[NB][DH / 16], dv[NB][DH / 16];
#pragma unroll
  for (int j = 0; j < NB; ++j) {
    const int kj = k0 + 16 * j + c;  // this lane's key (B-operand / C column)
#pragma unroll
    for (int s = 0; s < DH / 32; ++s) {
      kf[j][s] = gload8(a.k + b * a.kb + (long)kj * a.ks + hk * a.kh + 32 * s + 8 * g, kj < S);
      vf[j][s] = gload8(a.v + b * a.vb + (long)kj * a.vs + hk * a.vh + 32 * s + 8 * g, kj < S);
    }
#pragma unroll
    for (int t = 0; t < DH / 16; ++t) dk[j][t] = dv[j][t] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  const int qbeg = a.causal ? kblk * KW : 0;
  for (int hh = 0; hh < rep; ++hh) {
    const int h = hk * rep + hh;
    if ((a.head_mask >> h) & 1ull) continue;  // spliced head: constant z, no gradient
    const __bf16* qbase = a.q + b * a.qb + h * a.qh;
    const __bf16* gbase = a.dz + b * a.db + h * a.dh_;
    const float* lse = a.lse + ((long)b * a.Hq + h) * S;
    const float* D = a.dd + ((long)b * a.Hq + h) * S;
    for (int i0 = qbeg; i0 < S; i0 += T64) {
      __syncthreads();
      load_tile<DH>(Qs, qbase, a.qs, i0, S, tid);
      if (a.use_sp) load_tile_dz<DH>(Gs, gbase, a.ds, i0, S, tid, a, b, h);
      else load_tile<DH>(Gs, gbase, a.ds, i0, S, tid);
      if (tid < T64) {
        Ls[tid] = i0 + tid < S ? lse[i0 + tid] : 0.f;
        Ds[tid] = i0 + tid < S ? D[i0 + tid] : 0.f;
      }
      __syncthreads();
      if (a.causal && i0 + T64 - 1 < k0) continue;  // every query of this tile precedes this wave's keys
      float P[NB][4][4], dS[NB][4][4];
#pragma unroll
      for (int qm = 0; qm < 4; ++qm) {
        f32x4 sa[NB], pa[NB];
#pragma unroll
        for (int j = 0; j < NB; ++j) sa[j] = pa[j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s < DH / 32; ++s) {
          const bf16x8 qfr = frag_rows<DH>(Qs, 16 * qm, 32 * s, l), gfr = frag_rows<DH>(Gs, 16 * qm, 32 * s, l);
#pragma unroll
          for (int j = 0; j < NB; ++j) {
            sa[j] = mfma(qfr, kf[j][s], sa[j]);  // S[q][key]
            pa[j] = mfma(gfr, vf[j][s], pa[j]);  // dP[q][key]
          }
        }
#pragma unroll
        for (int j = 0; j < NB; ++j) {
          const int kj = k0 + 16 * j + c;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int il = 16 * qm + 4 * g + r, i = i0 + il;
            const bool ok = i < S && kj < S && (!a.causal || kj <= i);
            const float pv = ok ? __expf(sa[j][r] * a.scale - Ls[il]) : 0.f;
            P[j][qm][r] = pv;
            dS[j][qm][r] = pv * (pa[j][r] - Ds[il]);
          }
        }
      }
#pragma unroll
      for (int ch = 0; ch < 2; ++ch) {
        bf16x8 pb[NB], sb[NB];
#pragma unroll
        for (int j = 0; j < NB; ++j) {
          pb[j] = pack_perm(P[j][2 * ch], P[j][2 * ch + 1]);
          sb[j] = pack_perm(dS[j][2 * ch], dS[j][2 * ch + 1]);
        }
#pragma unroll
        for (int t = 0; t < DH / 16; ++t) {
          const bf16x8 gtr = frag_tr_perm<DH>(Gs, 32 * ch, 16 * t, l), qtr = frag_tr_perm<DH>(Qs, 32 * ch, 16 * t, l);
#pragma unroll
          for (int j = 0; j < NB; ++j) {
            dv[j][t] = mfma(gtr, pb[j], dv[j][t]);  // dV^T[d][key] += dO^T P
            dk[j][t] = mfma(qtr, sb[j], dk[j][t]);  // dK^T[d][key] += Q^T dS
          }
        }
      }
    }
  }
#pragma unroll
  for (int j = 0; j < NB; ++j) {
    const int kj = k0 + 16 * j + c;
    if (kj < S) {
      __bf16* dkr = a.dk + b * a.gkb + (long)kj * a.gks + hk * a.gkh;
      __bf16* dvr = a.dv + b * a.gvb + (long)kj * a.gvs + hk * a.gvh;
#pragma unroll
      for (int t = 0; t < DH / 16; ++t) {
        store4(dkr + 16 * t + 4 * g, dk[j][t], a.scale);
        store4(dvr + 16 * t + 4 * g, dv[j][t], 1.f);
      }
    }
  }
}

// dQ: each wave owns NB blocks of 16 queries (K / V fragment reads shared by NB MFMAs).
template <int DH, int NB>
__global__ __launch_bounds__(256, 2) void fa_bwd_dq_kernel(FaArgs a) {
  __shared__ __attribute__((aligned(16))) __bf16 Ks[T64 * DH];
  __shared__ __attribute__((aligned(16))) __bf16 Vs[T64 * DH];
  const int tid = threadIdx.x, wave = tid >> 6, l = tid & 63, g = l >> 4, c = l & 15;
  const int qblk = blockIdx.x, h = blockIdx.y, b = blockIdx.z;
  const int S = a.S;
  constexpr int QW = T64 * NB;
  const int q0 = qblk * QW + 16 * NB * wave;
  if ((a.head_mask >> h) & 1ull) {
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      const int qi = q0 + 16 * j + c;
      if (qi < S) {
        __bf16* dqr = a.dq + b * a.gqb + (long)qi * a.gqs + h * a.gqh;
#pragma unroll
        for (int t = 0; t < DH / 16; ++t) store4(dqr + 16 * t + 4 * g, f32x4{0.f, 0.f, 0.f, 0.f}, 1.f);
      }
    }
    return;
  }
  const int hk = h / (a.Hq / a.Hkv);
  const __bf16* kbase = a.k + b * a.kb + hk * a.kh;
  const __bf16* vbase = a.v + b * a.vb + hk * a.vh;
  const long hrow = ((long)b * a.Hq + h) * S;
  bf16x8 qf[NB][DH / 32], gf[NB][DH / 32];
  float lse_q[NB], D_q[NB];
  f32x4 dq[NB][DH / 16];
#pragma unroll
  for (int j = 0; j < NB; ++j) {
    const int qi = q0 + 16 * j + c;
#pragma unroll
    for (int s = 0; s < DH / 32; ++s) {
      qf[j][s] = gload8(a.q + b * a.qb + (long)qi * a.qs + h * a.qh + 32 * s + 8 * g, qi < S);
      gf[j][s] = sp_mask8(gload8(a.dz + b * a.db + (long)qi * a.ds + h * a.dh_ + 32 * s + 8 * g, qi < S), a,
                          qi < S && sp_row(a, b, qi, h), 32 * s + 8 * g);
    }
    lse_q[j] = qi < S ? a.lse[hrow + qi] : 0.f;
    D_q[j] = qi < S ? a.dd[hrow + qi] : 0.f;
#pragma unroll
    for (int t = 0; t < DH / 16; ++t) dq[j][t] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  const int kend = a.causal ? min(S, (qblk + 1) * QW) : S;
  for (int k0 = 0; k0 < kend; k0 += T64) {
    __syncthreads();
    load_tile<DH>(Ks, kbase, a.ks, k0, S, tid);
    load_tile<DH>(Vs, vbase, a.vs, k0, S, tid);
    __syncthreads();
    if (a.causal && k0 > q0 + 16 * NB - 1) continue;  // every key of this tile is after this wave's queries
    float dS[NB][4][4];
#pragma unroll
    for (int kb4 = 0; kb4 < 4; ++kb4) {
      f32x4 sa[NB], pa[NB];
#pragma unroll
      for (int j = 0; j < NB; ++j) sa[j] = pa[j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < DH / 32; ++s) {
        const bf16x8 kfr = frag_rows<DH>(Ks, 16 * kb4, 32 * s, l), vfr = frag_rows<DH>(Vs, 16 * kb4, 32 * s, l);
#pragma unroll
        for (int j = 0; j < NB; ++j) {
          sa[j] = mfma(kfr, qf[j][s], sa[j]);  // S^T[key][q]
          pa[j] = mfma(vfr, gf[j][s], pa[j]);  // dP^T[key][q]
        }
      }
#pragma unroll
      for (int j = 0; j < NB; ++j) {
        const int qi = q0 + 16 * j + c;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int kj = k0 + 16 * kb4 + 4 * g + r;
          const bool ok = qi < S && kj < S && (!a.causal || kj <= qi);
          const float pv = ok ? __expf(sa[j][r] * a.scale - lse_q[j]) : 0.f;
          dS[j][kb4][r] = pv * (pa[j][r] - D_q[j]);
        }
      }
    }
#pragma unroll
    for (int ch = 0; ch < 2; ++ch) {
      bf16x8 sb[NB];
#pragma unroll
      for (int j = 0; j < NB; ++j) sb[j] = pack_perm(dS[j][2 * ch], dS[j][2 * ch + 1]);
#pragma unroll
      for (int t = 0; t < DH / 16; ++t) {
        const bf16x8 ktr = frag_tr_perm<DH>(Ks, 32 * ch, 16 * t, l);
#pragma unroll
        for (int j = 0; j < NB; ++j) dq[j][t] = mfma(ktr, sb[j], dq[j][t]);
      }
    }
  }
#pragma unroll
  for (int j = 0; j < NB; ++j) {
    const int qi = q0 + 16 * j + c;
    if (qi < S) {
      __bf16* dqr = a.dq + b * a.gqb + (long)qi * a.gqs + h * a.gqh;
#pragma unroll
      for (int t = 0; t < DH / 16; ++t) store4(dqr + 16 * t + 4 * g, dq[j][t], a.scale);
    }
  }
}

bool args_ok(const FaArgs& a, int dh) {
  if (!(dh == 64 || dh == 128) || a.S <= 0 || a.B <= 0 || a.Hq <= 0 || a.Hkv <= 0 || a.Hq % a.Hkv) return false;
  if (a.head_mask && a.Hq > 64) return false;
  const long strides[] = {a.qs, a.qh, a.qb, a.ks, a.kh, a.kb, a.vs, a.vh, a.vb};
  for (long s : strides)
    if (s % 8) return false;
  const uintptr_t al = (uintptr_t)a.q | (uintptr_t)a.k | (uintptr_t)a.v;
  return (al & 15) == 0;
}

}  // namespace

// q [B,S,Hq,dh], k/v [B,S,Hkv,dh] (bf16, any batch/position/head strides that keep 16-B rows), z [B,S,Hq,dh] bf16,
// lse [B,Hq,S] fp32.  ``scale`` multiplies the scores (1/sqrt(dh) for standard attention).
IIT_EXPORT int iit_flash_fwd(const void* q, const void* k, const void* v, const long* strides9, void* z,
                             const long* zstrides3, float* lse, const void* src, const long* sstrides3,
                             unsigned long long head_mask, int B, int S, int Hq, int Hkv, int dh, float scale,
                             int causal, const void* spec, void* stream) {
  FaArgs a = {};
  a.q = (const __bf16*)q; a.k = (const __bf16*)k; a.v = (const __bf16*)v;
  a.qb = strides9[0]; a.qs = strides9[1]; a.qh = strides9[2];
  a.kb = strides9[3]; a.ks = strides9[4]; a.kh = strides9[5];
  a.vb = strides9[6]; a.vs = strides9[7]; a.vh = strides9[8];
  a.z = (__bf16*)z; a.zb = zstrides3[0]; a.zs = zstrides3[1]; a.zh = zstrides3[2];
  a.lse = lse;
  a.src = (const __bf16*)src;
  if (src && sstrides3) { a.sb = sstrides3[0]; a.ss = sstrides3[1]; a.sh = sstrides3[2]; }
  // a general splice spec (over [B][S][Hq][dh], source strides inside) replaces the head mask
  if (spec && src) { a.sp = *(const SpliceSpec*)spec; a.use_sp = 1; }
  a.head_mask = src && !a.use_sp ? head_mask : 0ull;
  if (a.use_sp && (a.sp.shape[0] != B || a.sp.shape[1] != S || a.sp.shape[2] != Hq || a.sp.shape[3] != dh))
    return (int)hipErrorInvalidValue;
  a.B = B; a.S = S; a.Hq = Hq; a.Hkv = Hkv; a.causal = causal; a.scale = scale;
  if (!args_ok(a, dh) || a.zs % 8 || a.zh % 8 || ((uintptr_t)z & 15)) return (int)hipErrorInvalidValue;
  // query blocks per wave: 2 halves the LDS traffic per FLOP but halves the workgroup count -- taken when that
  // still leaves >= 2 workgroups per CU (IIT_FLASH_QB=1|2 forces a choice)
  static const int qb_env = getenv("IIT_FLASH_QB") ? atoi(getenv("IIT_FLASH_QB")) : 0;
  const long wg2 = (long)((S + 2 * T64 - 1) / (2 * T64)) * Hq * B;
  const int QB = qb_env == 1 ? 1 : (qb_env == 2 ? 2 : (wg2 >= 512 ? 2 : 1));
  dim3 grid((S + T64 * QB - 1) / (T64 * QB), Hq, B);
  hipStream_t s = (hipStream_t)stream;
  if (dh == 64) {
    if (QB == 2) hipLaunchKernelGGL((fa_fwd_kernel<64, 2>), grid, dim3(256), 0, s, a);
    else hipLaunchKernelGGL((fa_fwd_kernel<64, 1>), grid, dim3(256), 0, s, a);
  } else {
    if (QB == 2) hipLaunchKernelGGL((fa_fwd_kernel<128, 2>), grid, dim3(256), 0, s, a);
    else hipLaunchKernelGGL((fa_fwd_kernel<128, 1>), grid, dim3(256), 0, s, a);
  }
  return (int)hipGetLastError();
}

// dz/z [B,S,Hq,dh] (z = the forward output), dd [B,Hq,S] fp32 scratch; dq/dk/dv with their own strides.
IIT_EXPORT int iit_flash_bwd(const void* q, const void* k, const void* v, const long* strides9, const void* z,
                             const long* zstrides3, const void* dz, const long* dzstrides3, const float* lse,
                             float* dd, void* dq, void* dk, void* dv, const long* gstrides9,
                             unsigned long long head_mask, int B, int S, int Hq, int Hkv, int dh, float scale,
                             int causal, const void* spec, void* stream) {
  FaArgs a = {};
  a.q = (const __bf16*)q; a.k = (const __bf16*)k; a.v = (const __bf16*)v;
  a.qb = strides9[0]; a.qs = strides9[1]; a.qh = strides9[2];
  a.kb = strides9[3]; a.ks = strides9[4]; a.kh = strides9[5];
  a.vb = strides9[6]; a.vs = strides9[7]; a.vh = strides9[8];
  a.z = (__bf16*)z; a.zb = zstrides3[0]; a.zs = zstrides3[1]; a.zh = zstrides3[2];
  a.dz = (const __bf16*)dz; a.db = dzstrides3[0]; a.ds = dzstrides3[1]; a.dh_ = dzstrides3[2];
  if (spec) {
    a.sp = *(const SpliceSpec*)spec;
    a.use_sp = 1;
    if (a.sp.shape[0] != B || a.sp.shape[1] != S || a.sp.shape[2] != Hq || a.sp.shape[3] != dh)
      return (int)hipErrorInvalidValue;
  }
  a.lse = (float*)lse; a.dd = dd;
  a.dq = (__bf16*)dq; a.dk = (__bf16*)dk; a.dv = (__bf16*)dv;
  a.gqb = gstrides9[0]; a.gqs = gstrides9[1]; a.gqh = gstrides9[2];
  a.gkb = gstrides9[3]; a.gks = gstrides9[4]; a.gkh = gstrides9[5];
  a.gvb = gstrides9[6]; a.gvs = gstrides9[7]; a.gvh = gstrides9[8];
  a.head_mask = a.use_sp ? 0ull : head_mask;
  a.B = B; a.S = S; a.Hq = Hq; a.Hkv = Hkv; a.causal = causal; a.scale = scale;
  if (!args_ok(a, dh) || a.ds % 8 || a.dh_ % 8 || a.zs % 8 || a.zh % 8 || ((uintptr_t)dz & 15) || ((uintptr_t)z & 15))
    return (int)hipErrorInvalidValue;
  for (int i = 0; i < 9; ++i)
    if (gstrides9[i] % 4) return (int)hipErrorInvalidValue;  // 8-byte stores
  hipStream_t s = (hipStream_t)stream;
  const long rows = (long)B * Hq * S;
  dim3 gp((rows + 255) / 256);
  // blocks per wave as in the forward: 2 when the grid keeps >= 2 workgroups per CU (IIT_FLASH_QB forces);
  // the dK/dV kernel keeps one block per wave at dh 128 (its accumulators would not fit two waves per SIMD)
  static const int qb_env = getenv("IIT_FLASH_QB") ? atoi(getenv("IIT_FLASH_QB")) : 0;
  const int tiles2 = (S + 2 * T64 - 1) / (2 * T64);
  const int nbq = qb_env == 1 ? 1 : (qb_env == 2 ? 2 : ((long)tiles2 * Hq * B >= 512 ? 2 : 1));
  const int nbk = dh == 128 ? 1 : (qb_env == 1 ? 1 : (qb_env == 2 ? 2 : ((long)tiles2 * Hkv * B >= 512 ? 2 : 1)));
  dim3 gkv((S + T64 * nbk - 1) / (T64 * nbk), Hkv, B), gq((S + T64 * nbq - 1) / (T64 * nbq), Hq, B);
  if (dh == 64) {
    hipLaunchKernelGGL(fa_bwd_prep_kernel<64>, gp, dim3(256), 0, s, a);
    if (nbk == 2) hipLaunchKernelGGL((fa_bwd_dkdv_kernel<64, 2>), gkv, dim3(256), 0, s, a);
    else hipLaunchKernelGGL((fa_bwd_dkdv_kernel<64, 1>), gkv, dim3(256), 0, s, a);
    if (nbq == 2) hipLaunchKernelGGL((fa_bwd_dq_kernel<64, 2>), gq, dim3(256), 0, s, a);
    else hipLaunchKernelGGL((fa_bwd_dq_kernel<64, 1>), gq, dim3(256), 0, s, a);
  } else {
    hipLaunchKernelGGL(fa_bwd_prep_kernel<128>, gp, dim3(256), 0, s, a);
    hipLaunchKernelGGL((fa_bwd_dkdv_kernel<128, 1>), gkv, dim3(256), 0, s, a);
    if (nbq == 2) hipLaunchKernelGGL((fa_bwd_dq_kernel<128, 2>), gq, dim3(256), 0, s, a);
    else hipLaunchKernelGGL((fa_bwd_dq_kernel<128, 1>), gq, dim3(256), 0, s, a);
  }
  return (int)hipGetLastError();
}
