// Causal self-attention for short sequences (S <= 16) on gfx950 MFMA.
//
// One wave64 per (batch, head), four per workgroup.  All products are
// v_mfma_f32_16x16x32_bf16 tiles (K padded to 32 with zeros where the reduction
// is over <= 16 positions), the softmax runs in registers:
//
//   forward   S^T = K Q^T           lane (g,c) holds S^T[kj=4g+r][qi=c]  (r = 0..3)
//             softmax over kj       4 registers + shfl_xor 16/32
//             Z^T = V^T P^T         P^T feeds the B operand with no lane movement
//                                   (k index 8g+j <-> kj 4g+j, j < 4; j >= 4 zero);
//                                   V^T comes from LDS through ds_read_b64_tr_b16
//   backward  P, P^T recomputed from the saved log-sum-exp; dP, dP^T by MFMA;
//             dV^T = dZ^T P,  dK^T = Q^T dS,  dQ^T = K^T dS^T  (tr16 A operands)
//
// Heads selected by ``head_mask`` are interchange-spliced: z := zsrc and their
// q/k/v gradients are zero (the spliced value is a constant).
#include "common.h"
#include "splice_spec.h"

typedef __attribute__((address_space(3))) i16x4 lds_i16x4_t;

__device__ __forceinline__ bf16x8 half_frag(const i16x4 v) {
  const i16x4 z = {0, 0, 0, 0};
  return __builtin_bit_cast(bf16x8, (i16x8)__builtin_shufflevector(v, z, 0, 1, 2, 3, 4, 5, 6, 7));
}

__device__ __forceinline__ bf16x8 regs_frag(float a, float b, float c, float d) {
  bf16x8 o = {f2bf(a), f2bf(b), f2bf(c), f2bf(d), f2bf(0.f), f2bf(0.f), f2bf(0.f), f2bf(0.f)};
  return o;
}

__device__ __forceinline__ bf16x8 load8(const __bf16* p, bool ok) {
  if (!ok) {
    const i16x8 z = {0, 0, 0, 0, 0, 0, 0, 0};
    return __builtin_bit_cast(bf16x8, z);
  }
  return *(const bf16x8*)p;
}

// tr16 read of the 4-row x 16-column block (rows 4g.., columns col0..) of a [16][LDSR] bf16 LDS image:
// lane c of group g receives column col0+c of rows 4g..4g+3.
template <int LDSR>
__device__ __forceinline__ i16x4 tr_block(const __bf16* img, int g, int lane_in_group, int col0) {
  const int q = lane_in_group >> 2, p = lane_in_group & 3;
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_i16x4_t*)(img + (4 * g + q) * LDSR + col0 + 4 * p));
}


// Paired source + base rows (iit_amd/ops/hip_ops.py Paired): sequences [0, pair_seqs) are base rows, the rest source
// rows.  Heads in ``pair_mask`` are spliced from source into base: the base wave of such a head computes nothing (its
// z is the source's, its gradient zero) and the source wave stores its z into both rows.  ``z2`` (nullable) receives
// a second copy of every stored z row (a whole-layer splice whose base z is the source z).
template <int DH, bool SP>
__global__ __launch_bounds__(256) void attn_mfma_fwd_kernel(const __bf16* __restrict__ qkv, __bf16* __restrict__ z,
                                                            float* __restrict__ lse, const __bf16* __restrict__ zsrc,
                                                            unsigned long long head_mask, int BH, int S, int H,
                                                            long ld_qkv, long ld_z, long ld_src, float scale,
                                                            int causal, __bf16* __restrict__ z2, int pair_seqs,
                                                            unsigned long long pair_mask, SpliceSpec sp, int use_sp) {
  constexpr int LDSR = DH + 8;
  __shared__ __attribute__((aligned(16))) __bf16 smem[4][16 * LDSR];
  const int wave = threadIdx.x >> 6, l = threadIdx.x & 63, g = l >> 4, c = l & 15;
  const int bh = blockIdx.x * 4 + wave;
  const bool valid = bh < BH;
  const int b = valid ? bh / H : 0, h = valid ? bh % H : 0;
  const int HD = H * DH;
  const long row0 = (long)b * S;
  const bool patched = valid && ((head_mask >> h) & 1ull);
  const bool mirrored = valid && pair_seqs > 0 && ((pair_mask >> h) & 1ull);
  const bool mirror_base = mirrored && b < pair_seqs;  // this base head takes the source's z
  const bool mirror_src = mirrored && b >= pair_seqs;  // ... which this source wave also stores there
  __bf16* Vs = smem[wave];
  if (valid && !patched && !mirror_base) {
    for (int i = l; i < 16 * DH / 8; i += 64) {
      const int r = i / (DH / 8), ch = i % (DH / 8);
      *(bf16x8*)(Vs + r * LDSR + ch * 8) = load8(qkv + (row0 + r) * ld_qkv + 2 * HD + h * DH + ch * 8, r < S);
    }
  }
  __syncthreads();
  if (!valid) return;
  if (mirror_base) {
    if (lse && l < S) lse[(long)bh * S + l] = 0.f;
    return;
  }
  if (patched) {
    for (int i = l; i < S * DH / 8; i += 64) {
      const int r = i / (DH / 8), ch = i % (DH / 8);
      const uint4 v = *(const uint4*)(zsrc + (row0 + r) * ld_src + h * DH + ch * 8);
      *(uint4*)(z + (row0 + r) * ld_z + h * DH + ch * 8) = v;
      if (z2) *(uint4*)(z2 + (row0 + r) * ld_z + h * DH + ch * 8) = v;
    }
    if (lse && l < S) lse[(long)bh * S + l] = 0.f;
    return;
  }
  // S^T = K Q^T
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int s = 0; s < DH / 32; ++s) {
    const long off = (row0 + c) * ld_qkv + h * DH + 32 * s + 8 * g;
    const bf16x8 kf = load8(qkv + off + HD, c < S);
    const bf16x8 qf = load8(qkv + off, c < S);
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf, qf, acc, 0, 0, 0);
  }
  float sc[4];
  float m = -INFINITY;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int kj = 4 * g + r;
    const bool ok = kj < S && (!causal || kj <= c);
    sc[r] = ok ? acc[r] * scale : -INFINITY;
    m = fmaxf(m, sc[r]);
  }
  m = fmaxf(m, __shfl_xor(m, 16, 64));
  m = fmaxf(m, __shfl_xor(m, 32, 64));
  float p[4], sum = 0.f;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    p[r] = sc[r] == -INFINITY ? 0.f : __expf(sc[r] - m);
    sum += p[r];
  }
  sum += __shfl_xor(sum, 16, 64);
  sum += __shfl_xor(sum, 32, 64);
  const float inv = sum > 0.f ? 1.f / sum : 0.f;
  if (lse && g == 0 && c < S) lse[(long)bh * S + c] = m + __logf(sum);
  const bf16x8 bp = regs_frag(p[0] * inv, p[1] * inv, p[2] * inv, p[3] * inv);
  f32x4 o[DH / 16];
#pragma unroll
  for (int t = 0; t < DH / 16; ++t) {
    const bf16x8 av = half_frag(tr_block<LDSR>(Vs, g, c, 16 * t));
    const f32x4 zero = {0.f, 0.f, 0.f, 0.f};
    o[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, bp, zero, 0, 0, 0);  // Z^T[e][qi=c]
  }
  // z rows out through this wave's LDS image (V is consumed) as 16-byte chunks, as in the backward
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
  for (int t = 0; t < DH / 16; ++t)
    *(bf16x4*)(Vs + c * LDSR + 16 * t + 4 * g) = bf16x4{f2bf(o[t][0]), f2bf(o[t][1]), f2bf(o[t][2]), f2bf(o[t][3])};
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
  for (int i = l; i < 16 * DH / 8; i += 64) {
    const int r = i / (DH / 8), ch = i % (DH / 8);
    if (r < S) {
      const bf16x8 v = *(const bf16x8*)(Vs + r * LDSR + ch * 8);
      __bf16* zo = z + (row0 + r) * ld_z + h * DH + ch * 8;
      if (SP && use_sp && pair_seqs > 0) {
        // general patch spec over the base rows' z [pair_seqs][S][H][DH]: the source wave of (b, h) also stores the
        // selected elements of its row into the base row; the base wave stores only the unselected ones (disjoint
        // writes, no ordering between the two waves needed).  A partly selected 16-B chunk goes out element-wise.
        const bool base = b < pair_seqs;
        const int bb = base ? b : b - pair_seqs;
        const bool rowsel = in_ranges(sp, 0, bb) && in_ranges(sp, 1, r) && in_ranges(sp, 2, h);
        unsigned m = 0;
        if (rowsel) {
#pragma unroll
          for (int e = 0; e < 8; ++e) m |= (unsigned)in_ranges(sp, 3, ch * 8 + e) << e;
        }
        if (base) {
          if (m == 0) *(bf16x8*)zo = v;
          else if (m != 0xffu) {
#pragma unroll
            for (int e = 0; e < 8; ++e)
              if (!((m >> e) & 1u)) zo[e] = v[e];
          }
        } else {
          *(bf16x8*)zo = v;
          __bf16* zb = z + (row0 - (long)pair_seqs * S + r) * ld_z + h * DH + ch * 8;
          if (m == 0xffu) *(bf16x8*)zb = v;
          else if (m) {
#pragma unroll
            for (int e = 0; e < 8; ++e)
              if ((m >> e) & 1u) zb[e] = v[e];
          }
        }
        continue;
      }
      *(bf16x8*)zo = v;
      if (z2) *(bf16x8*)(z2 + (row0 + r) * ld_z + h * DH + ch * 8) = v;
      if (mirror_src) *(bf16x8*)(z + (row0 - (long)pair_seqs * S + r) * ld_z + h * DH + ch * 8) = v;
    }
  }
}

template <int DH, bool SP>
__global__ __launch_bounds__(256) void attn_mfma_bwd_kernel(const __bf16* __restrict__ qkv, const __bf16* __restrict__ dz,
                                                            const float* __restrict__ lse, __bf16* __restrict__ dqkv,
                                                            unsigned long long head_mask, int BH, int S, int H,
                                                            long ld_qkv, long ld_dz, float scale, int causal,
                                                            SpliceSpec sp, int use_sp) {
  constexpr int LDSR = DH + 8;
  __shared__ __attribute__((aligned(16))) __bf16 smem[4][3][16 * LDSR];
  __shared__ float Dsh[4][16];
  const int wave = threadIdx.x >> 6, l = threadIdx.x & 63, g = l >> 4, c = l & 15;
  const int bh = blockIdx.x * 4 + wave;
  const bool valid = bh < BH;
  const int b = valid ? bh / H : 0, h = valid ? bh % H : 0;
  const int HD = H * DH;
  const long row0 = (long)b * S;
  const bool patched = valid && ((head_mask >> h) & 1ull);
  const bool work = valid && !patched;
  __bf16* Qs = smem[wave][0];
  __bf16* Ks = smem[wave][1];
  __bf16* Gs = smem[wave][2];
  // fragments of row c (zero beyond S) and LDS images for the transposed operands
  bf16x8 qf[DH / 32], kf[DH / 32], vf[DH / 32], gf[DH / 32];
#pragma unroll
  for (int s = 0; s < DH / 32; ++s) {
    const long off = (row0 + c) * ld_qkv + h * DH + 32 * s + 8 * g;
    const bool ok = work && c < S;
    qf[s] = load8(qkv + off, ok);
    kf[s] = load8(qkv + off + HD, ok);
    vf[s] = load8(qkv + off + 2 * HD, ok);
    gf[s] = load8(dz + (row0 + c) * ld_dz + h * DH + 32 * s + 8 * g, ok);
    if (SP && use_sp && ok && in_ranges(sp, 0, b) && in_ranges(sp, 1, c) && in_ranges(sp, 2, h)) {
      // spliced elements of z are the source's (a constant): their gradient is zero
#pragma unroll
      for (int e = 0; e < 8; ++e)
        if (in_ranges(sp, 3, 32 * s + 8 * g + e)) gf[s][e] = f2bf(0.f);
    }
    if (work) {
      *(bf16x8*)(Qs + c * LDSR + 32 * s + 8 * g) = qf[s];
      *(bf16x8*)(Ks + c * LDSR + 32 * s + 8 * g) = kf[s];
      *(bf16x8*)(Gs + c * LDSR + 32 * s + 8 * g) = gf[s];
    }
  }
  f32x4 Sa = {0.f, 0.f, 0.f, 0.f}, STa = Sa, dPa = Sa, dPTa = Sa;
#pragma unroll
  for (int s = 0; s < DH / 32; ++s) {
    Sa = __builtin_amdgcn_mfma_f32_16x16x32_bf16(qf[s], kf[s], Sa, 0, 0, 0);     // S[qi=4g+r][kj=c]
    STa = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf[s], qf[s], STa, 0, 0, 0);   // S^T[kj=4g+r][qi=c]
    dPa = __builtin_amdgcn_mfma_f32_16x16x32_bf16(gf[s], vf[s], dPa, 0, 0, 0);   // dP[qi=4g+r][kj=c]
    dPTa = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vf[s], gf[s], dPTa, 0, 0, 0); // dP^T[kj=4g+r][qi=c]
  }
  float P[4], PT[4], Dr[4];
  const float lse_c = (work && c < S) ? lse[(long)bh * S + c] : 0.f;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int qi = 4 * g + r, kj = c;
    const bool ok = work && qi < S && kj < S && (!causal || kj <= qi);
    P[r] = ok ? __expf(Sa[r] * scale - lse[(long)bh * S + qi]) : 0.f;
    const int kj2 = 4 * g + r, qi2 = c;
    const bool ok2 = work && qi2 < S && kj2 < S && (!causal || kj2 <= qi2);
    PT[r] = ok2 ? __expf(STa[r] * scale - lse_c) : 0.f;
    float d = P[r] * dPa[r];
    d += __shfl_xor(d, 1, 64);
    d += __shfl_xor(d, 2, 64);
    d += __shfl_xor(d, 4, 64);
    d += __shfl_xor(d, 8, 64);
    Dr[r] = d;  // D[qi = 4g + r]
  }
  if (c == 0) {
#pragma unroll
    for (int r = 0; r < 4; ++r) Dsh[wave][4 * g + r] = Dr[r];
  }
  __syncthreads();
  if (!valid) return;
  __bf16* dq = dqkv + h * DH;
  __bf16* dk = dqkv + HD + h * DH;
  __bf16* dv = dqkv + 2 * HD + h * DH;
  if (patched) {
    for (int i = l; i < S * DH / 8; i += 64) {
      const int r = i / (DH / 8), ch = i % (DH / 8);
      const uint4 zz = make_uint4(0, 0, 0, 0);
      *(uint4*)(dq + (row0 + r) * ld_qkv + ch * 8) = zz;
      *(uint4*)(dk + (row0 + r) * ld_qkv + ch * 8) = zz;
      *(uint4*)(dv + (row0 + r) * ld_qkv + ch * 8) = zz;
    }
    return;
  }
  const float Dc = Dsh[wave][c];
  float dS[4], dST[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    dS[r] = P[r] * (dPa[r] - Dr[r]) * scale;   // dS[qi=4g+r][kj=c]
    dST[r] = PT[r] * (dPTa[r] - Dc) * scale;   // dS^T[kj=4g+r][qi=c]
  }
  const bf16x8 bP = regs_frag(P[0], P[1], P[2], P[3]);
  const bf16x8 bdS = regs_frag(dS[0], dS[1], dS[2], dS[3]);
  const bf16x8 bdST = regs_frag(dST[0], dST[1], dST[2], dST[3]);
  const f32x4 zero = {0.f, 0.f, 0.f, 0.f};
  f32x4 dvT[DH / 16], dkT[DH / 16], dqT[DH / 16];
#pragma unroll
  for (int t = 0; t < DH / 16; ++t) {
    const bf16x8 aG = half_frag(tr_block<LDSR>(Gs, g, c, 16 * t));  // dZ^T[e][qi=4g+j]
    const bf16x8 aQ = half_frag(tr_block<LDSR>(Qs, g, c, 16 * t));  // Q^T[e][qi=4g+j]
    const bf16x8 aK = half_frag(tr_block<LDSR>(Ks, g, c, 16 * t));  // K^T[e][kj=4g+j]
    dvT[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(aG, bP, zero, 0, 0, 0);   // dV^T[e][kj=c]
    dkT[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(aQ, bdS, zero, 0, 0, 0);  // dK^T[e][kj=c]
    dqT[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(aK, bdST, zero, 0, 0, 0); // dQ^T[e][qi=c]
  }
  // Coalesced writes: the transposed results go through this wave's (now free) LDS images as [16][DH] rows, then
  // out as 16-byte row chunks (the MFMA layout would give 8-byte stores scattered over 16 rows per instruction).
  // Only this wave touches its images, so an lgkmcnt drain orders its LDS writes before its reads.
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
  for (int t = 0; t < DH / 16; ++t) {
    const int o = c * LDSR + 16 * t + 4 * g;
    *(bf16x4*)(Gs + o) = bf16x4{f2bf(dvT[t][0]), f2bf(dvT[t][1]), f2bf(dvT[t][2]), f2bf(dvT[t][3])};
    *(bf16x4*)(Ks + o) = bf16x4{f2bf(dkT[t][0]), f2bf(dkT[t][1]), f2bf(dkT[t][2]), f2bf(dkT[t][3])};
    *(bf16x4*)(Qs + o) = bf16x4{f2bf(dqT[t][0]), f2bf(dqT[t][1]), f2bf(dqT[t][2]), f2bf(dqT[t][3])};
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  constexpr int CPR = DH / 8;  // 16-byte chunks per row
#pragma unroll
  for (int i = l; i < 16 * CPR; i += 64) {
    const int r = i / CPR, ch = i % CPR;
    if (r < S) {
      const long o = (row0 + r) * ld_qkv + ch * 8;
      *(bf16x8*)(dv + o) = *(const bf16x8*)(Gs + r * LDSR + ch * 8);
      *(bf16x8*)(dk + o) = *(const bf16x8*)(Ks + r * LDSR + ch * 8);
      *(bf16x8*)(dq + o) = *(const bf16x8*)(Qs + r * LDSR + ch * 8);
    }
  }
}

IIT_EXPORT int iit_attn_mfma_fwd_pair(const void* qkv, void* z, float* lse, const void* zsrc,
                                      unsigned long long head_mask, int B, int S, int H, int dh, long ld_qkv, long ld_z,
                                      long ld_src, float scale, int causal, void* z2, int pair_seqs,
                                      unsigned long long pair_mask, void* stream);

IIT_EXPORT int iit_attn_mfma_fwd(const void* qkv, void* z, float* lse, const void* zsrc, unsigned long long head_mask,
                                 int B, int S, int H, int dh, long ld_qkv, long ld_z, long ld_src, float scale,
                                 int causal, void* stream) {
  return iit_attn_mfma_fwd_pair(qkv, z, lse, zsrc, head_mask, B, S, H, dh, ld_qkv, ld_z, ld_src, scale, causal,
                                nullptr, 0, 0ull, stream);
}

// the same with the paired-row options of attn_mfma_fwd_kernel (``z2`` copy, ``pair_mask`` heads of the first
// ``pair_seqs`` sequences taken from the sequences ``pair_seqs`` later)
static int attn_fwd_launch(const void* qkv, void* z, float* lse, const void* zsrc, unsigned long long head_mask,
                           int B, int S, int H, int dh, long ld_qkv, long ld_z, long ld_src, float scale, int causal,
                           void* z2, int pair_seqs, unsigned long long pair_mask, const SpliceSpec& sp, int use_sp,
                           void* stream);

IIT_EXPORT int iit_attn_mfma_fwd_pair(const void* qkv, void* z, float* lse, const void* zsrc,
                                      unsigned long long head_mask, int B, int S, int H, int dh, long ld_qkv, long ld_z,
                                      long ld_src, float scale, int causal, void* z2, int pair_seqs,
                                      unsigned long long pair_mask, void* stream) {
  const SpliceSpec none{};
  return attn_fwd_launch(qkv, z, lse, zsrc, head_mask, B, S, H, dh, ld_qkv, ld_z, ld_src, scale, causal, z2,
                         pair_seqs, pair_mask, none, 0, stream);
}

// Paired rows with a general interchange splice of ``hook_z`` (host SpliceSpec over the base rows' [B][S][H][dh]
// z, e.g. one position of some heads): applied in the kernel's store (see attn_mfma_fwd_kernel); no head mirroring
IIT_EXPORT int iit_attn_mfma_fwd_spec(const void* qkv, void* z, float* lse, int B, int S, int H, int dh, long ld_qkv,
                                      long ld_z, float scale, int causal, int pair_seqs, const void* spec,
                                      void* stream) {
  if (pair_seqs <= 0) return (int)hipErrorInvalidValue;
  return attn_fwd_launch(qkv, z, lse, nullptr, 0ull, B, S, H, dh, ld_qkv, ld_z, 0, scale, causal, nullptr, pair_seqs,
                         0ull, *(const SpliceSpec*)spec, 1, stream);
}

static int attn_fwd_launch(const void* qkv, void* z, float* lse, const void* zsrc, unsigned long long head_mask,
                           int B, int S, int H, int dh, long ld_qkv, long ld_z, long ld_src, float scale, int causal,
                           void* z2, int pair_seqs, unsigned long long pair_mask, const SpliceSpec& sp, int use_sp,
                           void* stream) {
  if (S > 16) return (int)hipErrorInvalidValue;
  if (pair_seqs < 0 || (pair_seqs > 0 && 2 * pair_seqs != B)) return (int)hipErrorInvalidValue;
  const int BH = B * H;
  dim3 grid((BH + 3) / 4), block(256);
  hipStream_t s = (hipStream_t)stream;
#define AF(D)                                                                                                       \
  hipLaunchKernelGGL((use_sp ? attn_mfma_fwd_kernel<D, true> : attn_mfma_fwd_kernel<D, false>), grid, block, 0, s,    \
                     (const __bf16*)qkv, (__bf16*)z, lse,                                                           \
                     (const __bf16*)zsrc, head_mask, BH, S, H, ld_qkv, ld_z, ld_src, scale, causal, (__bf16*)z2,    \
                     pair_seqs, pair_mask, sp, use_sp)
  if (dh == 32) AF(32);
  else if (dh == 64) AF(64);
  else if (dh == 96) AF(96);
  else if (dh == 128) AF(128);
  else return (int)hipErrorInvalidValue;
#undef AF
  return hipGetLastError();
}

static int attn_bwd_launch(const void* qkv, const void* dz, const float* lse, void* dqkv, unsigned long long head_mask,
                           int B, int S, int H, int dh, long ld_qkv, long ld_dz, float scale, int causal,
                           const SpliceSpec& sp, int use_sp, void* stream);

IIT_EXPORT int iit_attn_mfma_bwd(const void* qkv, const void* dz, const float* lse, void* dqkv,
                                 unsigned long long head_mask, int B, int S, int H, int dh, long ld_qkv, long ld_dz,
                                 float scale, int causal, void* stream) {
  const SpliceSpec none{};
  return attn_bwd_launch(qkv, dz, lse, dqkv, head_mask, B, S, H, dh, ld_qkv, ld_dz, scale, causal, none, 0, stream);
}

// the backward of iit_attn_mfma_fwd_spec's base rows: the spliced elements of dz are zeroed as they are loaded
IIT_EXPORT int iit_attn_mfma_bwd_spec(const void* qkv, const void* dz, const float* lse, void* dqkv, int B, int S,
                                      int H, int dh, long ld_qkv, long ld_dz, float scale, int causal,
                                      const void* spec, void* stream) {
  return attn_bwd_launch(qkv, dz, lse, dqkv, 0ull, B, S, H, dh, ld_qkv, ld_dz, scale, causal,
                         *(const SpliceSpec*)spec, 1, stream);
}

static int attn_bwd_launch(const void* qkv, const void* dz, const float* lse, void* dqkv, unsigned long long head_mask,
                           int B, int S, int H, int dh, long ld_qkv, long ld_dz, float scale, int causal,
                           const SpliceSpec& sp, int use_sp, void* stream) {
  if (S > 16) return (int)hipErrorInvalidValue;
  const int BH = B * H;
  dim3 grid((BH + 3) / 4), block(256);
  hipStream_t s = (hipStream_t)stream;
#define AB(D)                                                                                                       \
  hipLaunchKernelGGL((use_sp ? attn_mfma_bwd_kernel<D, true> : attn_mfma_bwd_kernel<D, false>), grid, block, 0, s,    \
                     (const __bf16*)qkv, (const __bf16*)dz, lse,                                                    \
                     (__bf16*)dqkv, head_mask, BH, S, H, ld_qkv, ld_dz, scale, causal, sp, use_sp)
  if (dh == 32) AB(32);
  else if (dh == 64) AB(64);
  else if (dh == 96) AB(96);
  else if (dh == 128) AB(128);
  else return (int)hipErrorInvalidValue;
#undef AB
  return hipGetLastError();
}
