// Non-GEMM kernels of the iit_amd engine for gfx950 (MI355X).  All wave64-native.
//
//  embed_pos_fwd / embed_bwd / pos_bwd     token+position embedding (fp32 residual stream)
//  ln_fwd / ln_bwd                          LN / LNPre, one wave per row, fp32 stats
//  attn_small_fwd / attn_small_bwd          causal attention for S <= 64, dh <= 128, one
//                                           workgroup per (batch, head); per-head splice of
//                                           hook_z inside the kernel (patched heads copy the
//                                           source z and get zero q/k/v gradient)
//  ce_fwd / ce_bwd                          row-wise cross entropy over the vocab (+argmax)
//  sumsq_partial / adam_flat                global-norm clip + Adam over the flat arena
//  shadow_refresh                           fp32 master -> bf16 compute copies (+transposes)
//  colsum_accum, dgelu, add_f32, cast       small elementwise / reduction helpers
#include "common.h"
#include <stdlib.h>

// ============================================================================ embedding
__global__ void embed_pos_fwd_kernel(const long* __restrict__ tok, const float* __restrict__ WE,
                                     const float* __restrict__ Wpos, float* __restrict__ out, int T, int S, int d) {
  const int t = blockIdx.x;
  if (t >= T) return;
  const long v = tok[t];
  const int s = t % S;
  const float4* e = (const float4*)(WE + v * (long)d);
  const float4* p = (const float4*)(Wpos + (long)s * d);
  float4* o = (float4*)(out + (long)t * d);
  for (int i = threadIdx.x; i < d / 4; i += blockDim.x) {
    float4 a = e[i], b = p[i];
    o[i] = make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w);
  }
}

IIT_EXPORT int iit_embed_pos_fwd(const long* tok, const float* WE, const float* Wpos, float* out, int T, int S,
                                 int d, void* stream) {
  hipLaunchKernelGGL(embed_pos_fwd_kernel, dim3(T), dim3(d >= 256 ? 64 : 64), 0, (hipStream_t)stream, tok, WE, Wpos,
                     out, T, S, d);
  return hipGetLastError();
}

// dW_E[tok[t]] += g[t]   (fp32 atomics, one 256-B segment per wave-instruction)
__global__ void embed_bwd_kernel(const long* __restrict__ tok, const float* __restrict__ g, float* __restrict__ dWE,
                                 int T, int d) {
  const int t = blockIdx.x;
  const long v = tok[t];
  for (int i = threadIdx.x; i < d; i += blockDim.x) atomicAdd(dWE + v * (long)d + i, g[(long)t * d + i]);
}

// Position-major form: block = (position s, 256-column slab, chunk of EB sequences); each thread walks its column
// down the chunk's sequences at position s and adds runs of EQUAL tokens in a register, one atomic per run.  IIT
// batches repeat template tokens at a position across the batch (IOI: every word but the names), so the atomics on
// a contended row drop from B to B / EB per column; distinct tokens cost what the token-major kernel costs.
constexpr int EB = 32;
__global__ __launch_bounds__(256) void embed_bwd_pos_kernel(const long* __restrict__ tok, const float* __restrict__ g,
                                                            float* __restrict__ dWE, int B, int S, int d) {
  const int s = blockIdx.x, c = blockIdx.y * 256 + threadIdx.x, b0 = blockIdx.z * EB;
  if (c >= d) return;
  const int b1 = min(B, b0 + EB);
  long cur = -1;
  float acc = 0.f;
  // 8 rows' token ids and gradients loaded before the first is used: the loop was one dependent load round trip
  // per row (latency-bound)
  for (int bb = b0; bb < b1; bb += 8) {
    long vv[8];
    float xx[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int b = bb + k;
      vv[k] = -1;
      xx[k] = 0.f;
      if (b < b1) {
        const long t = (long)b * S + s;
        vv[k] = tok[t];
        xx[k] = g[t * d + c];
      }
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      if (vv[k] < 0) break;
      if (vv[k] != cur) {
        if (cur >= 0) atomicAdd(dWE + cur * (long)d + c, acc);
        cur = vv[k];
        acc = xx[k];
      } else {
        acc += xx[k];
      }
    }
  }
  if (cur >= 0) atomicAdd(dWE + cur * (long)d + c, acc);
}

// dW_pos[s] += sum_b g[b, s].  Block = (position s, 256-column slab); 4 waves split the batch, LDS combine.
__global__ __launch_bounds__(256) void pos_bwd_kernel(const float* __restrict__ g, float* __restrict__ dWpos, int B,
                                                      int S, int d) {
  __shared__ float part[4][64 * 4];
  const int s = blockIdx.x, w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int c = blockIdx.y * 256 + lane * 4;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  if (c < d)
#pragma unroll 8  // independent row loads in flight (the loop was one round trip per row)
    for (int b = w; b < B; b += 4) {
      const float4 v = *(const float4*)(g + ((long)b * S + s) * d + c);
      acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
    }
  *(float4*)&part[w][lane * 4] = acc;
  __syncthreads();
  const int col = blockIdx.y * 256 + threadIdx.x;
  if (col < d)
    dWpos[(long)s * d + col] += part[0][threadIdx.x] + part[1][threadIdx.x] + part[2][threadIdx.x] + part[3][threadIdx.x];
}

__global__ void pos_bwd_scalar_kernel(const float* __restrict__ g, float* __restrict__ dWpos, int B, int S, int d) {
  const int s = blockIdx.x;
  for (int i = threadIdx.x; i < d; i += blockDim.x) {
    float acc = 0.f;
    for (int b = 0; b < B; ++b) acc += g[((long)b * S + s) * d + i];
    dWpos[(long)s * d + i] += acc;
  }
}

IIT_EXPORT int iit_embed_pos_bwd(const long* tok, const float* g, float* dWE, float* dWpos, int B, int S, int d,
                                 void* stream) {
  hipStream_t st = (hipStream_t)stream;
  // (an LDS-combining variant -- 64-position chunks adding equal tokens' rows before one global atomic per distinct
  // token -- measured 54 us against this kernel's 30 us on the IOI batch: fewer, longer blocks; not kept)
  static const bool pos_major = [] {
    const char* e = getenv("IIT_EMBED_BWD_POS");
    return !(e && e[0] == '0');
  }();
  if (dWE && pos_major)
    hipLaunchKernelGGL(embed_bwd_pos_kernel, dim3(S, (d + 255) / 256, (B + EB - 1) / EB), dim3(256), 0, st, tok, g,
                       dWE, B, S, d);
  else if (dWE)
    hipLaunchKernelGGL(embed_bwd_kernel, dim3(B * S), dim3(256), 0, st, tok, g, dWE, B * S, d);
  if (dWpos) {
    if (d % 4 == 0 && (((uintptr_t)g) & 15) == 0)
      hipLaunchKernelGGL(pos_bwd_kernel, dim3(S, (d + 255) / 256), dim3(256), 0, st, g, dWpos, B, S, d);
    else
      hipLaunchKernelGGL(pos_bwd_scalar_kernel, dim3(S), dim3(256), 0, st, g, dWpos, B, S, d);
  }
  return hipGetLastError();
}

// ============================================================================ layer norm
// Row select: the interchange splice of whole positions of an LN output inside the LN kernel itself (a paired
// source+base forward, iit_amd/models/bert.py forward_paired: MQNLI's ``hook_normalized_resid_post`` position
// sites).  Rows [0, Tb) are the base rows, [Tb, 2 Tb) the source rows at the same (batch, position); a base row
// whose position s has bit s of ``mask`` set normalises the SOURCE row instead (out[idx] = src[idx] for whole
// rows), and in the backward the same base rows get no gradient (the spliced slice is a constant).  mask == 0:
// plain LN.
struct RowSel {
  unsigned long long mask;
  int S;
  int Tb;
};

__device__ __forceinline__ bool sel_hit(const RowSel& sel, int row) {
  return sel.mask != 0ull && row < sel.Tb && ((sel.mask >> (row % sel.S)) & 1ull);
}

// One wave per row; each lane owns V4 float4 column groups (c4 = lane + 64*i), so every load is a 16-B
// vector and a wave instruction moves 1 KB (fp32) / 512 B (bf16).  Requires d % 4 == 0 and 16-B aligned
// rows; the scalar kernels below cover everything else.  Stats in fp32.
template <int V4>
__global__ __launch_bounds__(256) void ln_fwd_vec_kernel(const float* __restrict__ x, const float* __restrict__ w,
                                                         const float* __restrict__ b, __bf16* __restrict__ y,
                                                         float* __restrict__ mean_out, float* __restrict__ rstd_out,
                                                         int T, int d, float eps, RowSel sel,
                                                         float* __restrict__ y32 = nullptr) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= T) return;
  const int d4 = d >> 2;
  const int xrow = sel_hit(sel, row) ? row + sel.Tb : row;
  const float4* xr = (const float4*)(x + (long)xrow * d);
  float4 v[V4];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < V4; ++i) {
    const int c = lane + i * 64;
    v[i] = c < d4 ? xr[c] : make_float4(0.f, 0.f, 0.f, 0.f);
    s += (v[i].x + v[i].y) + (v[i].z + v[i].w);
  }
  const float mu = wave_sum(s) / d;
  float s2 = 0.f;
#pragma unroll
  for (int i = 0; i < V4; ++i) {
    const int c = lane + i * 64;
    if (c < d4) {
      v[i].x -= mu; v[i].y -= mu; v[i].z -= mu; v[i].w -= mu;
      s2 += (v[i].x * v[i].x + v[i].y * v[i].y) + (v[i].z * v[i].z + v[i].w * v[i].w);
    }
  }
  const float rstd = rsqrtf(wave_sum(s2) / d + eps);
  bf16x4* yr = (bf16x4*)(y + (long)row * d);
#pragma unroll
  for (int i = 0; i < V4; ++i) {
    const int c = lane + i * 64;
    if (c < d4) {
      float4 o = make_float4(v[i].x * rstd, v[i].y * rstd, v[i].z * rstd, v[i].w * rstd);
      if (w) {
        const float4 ww = ((const float4*)w)[c], bb = ((const float4*)b)[c];
        o = make_float4(o.x * ww.x + bb.x, o.y * ww.y + bb.y, o.z * ww.z + bb.z, o.w * ww.w + bb.w);
      }
      bf16x4 ob = {f2bf(o.x), f2bf(o.y), f2bf(o.z), f2bf(o.w)};
      yr[c] = ob;
      if (y32)  // the fp32 twin of the rounded output (a post-norm block's residual operand: no separate cast pass)
        ((float4*)(y32 + (long)row * d))[c] = make_float4(bf2f(ob[0]), bf2f(ob[1]), bf2f(ob[2]), bf2f(ob[3]));
    }
  }
  if (lane == 0) {
    mean_out[row] = mu;
    rstd_out[row] = rstd;
  }
}

// scalar fallback: y = (x - mean) * rstd  (* w + b);   one wave per row, up to VPL floats per lane
template <int VPL>
__global__ __launch_bounds__(256) void ln_fwd_kernel(const float* __restrict__ x, const float* __restrict__ w,
                                                     const float* __restrict__ b, __bf16* __restrict__ y,
                                                     float* __restrict__ mean_out, float* __restrict__ rstd_out,
                                                     int T, int d, float eps, RowSel sel) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= T) return;
  const float* xr = x + (long)(sel_hit(sel, row) ? row + sel.Tb : row) * d;
  float v[VPL];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < VPL; ++i) {
    const int c = lane + i * 64;
    v[i] = c < d ? xr[c] : 0.f;
    s += v[i];
  }
  const float mu = wave_sum(s) / d;
  float s2 = 0.f;
#pragma unroll
  for (int i = 0; i < VPL; ++i) {
    const int c = lane + i * 64;
    const float z = c < d ? v[i] - mu : 0.f;
    v[i] = z;
    s2 += z * z;
  }
  const float rstd = rsqrtf(wave_sum(s2) / d + eps);
  __bf16* yr = y + (long)row * d;
#pragma unroll
  for (int i = 0; i < VPL; ++i) {
    const int c = lane + i * 64;
    if (c < d) {
      float o = v[i] * rstd;
      if (w) o = o * w[c] + b[c];
      yr[c] = f2bf(o);
    }
  }
  if (lane == 0) {
    mean_out[row] = mu;
    rstd_out[row] = rstd;
  }
}

static inline bool aligned16(const void* p) { return (((uintptr_t)p) & 15) == 0; }

IIT_EXPORT int iit_ln_fwd_sel(const float* x, const float* w, const float* b, void* y, float* mean, float* rstd,
                              int T, int d, float eps, unsigned long long pos_mask, int S, int Tb, void* stream);

IIT_EXPORT int iit_ln_fwd(const float* x, const float* w, const float* b, void* y, float* mean, float* rstd, int T,
                          int d, float eps, void* stream) {
  return iit_ln_fwd_sel(x, w, b, y, mean, rstd, T, d, eps, 0ull, 1, 0, stream);
}

// iit_ln_fwd that also writes ``y32`` = fp32(y) (vector layout only: d % 4 == 0, d <= 4096, 16-B aligned rows)
IIT_EXPORT int iit_ln_fwd_twin(const float* x, const float* w, const float* b, void* y, float* y32, float* mean,
                               float* rstd, int T, int d, float eps, void* stream) {
  const bool vec = d % 4 == 0 && d <= 4096 && aligned16(x) && (((uintptr_t)y) & 7) == 0 && aligned16(y32) &&
                   (!w || (aligned16(w) && aligned16(b)));
  if (!vec) return (int)hipErrorInvalidValue;
  const RowSel sel{0ull, 1, 0};
  dim3 grid((T + 3) / 4), block(256);
  hipStream_t s = (hipStream_t)stream;
#define LNT(V) hipLaunchKernelGGL((ln_fwd_vec_kernel<V>), grid, block, 0, s, x, w, b, (__bf16*)y, mean, rstd, T, d, eps, sel, y32)
  const int v4 = (d / 4 + 63) / 64;
  if (v4 <= 1) LNT(1); else if (v4 <= 2) LNT(2); else if (v4 <= 3) LNT(3); else if (v4 <= 4) LNT(4);
  else if (v4 <= 6) LNT(6); else if (v4 <= 8) LNT(8); else if (v4 <= 12) LNT(12); else LNT(16);
#undef LNT
  return hipGetLastError();
}

// ``pos_mask`` (RowSel): base rows [0, Tb) at positions with their bit set normalise the source row row + Tb
IIT_EXPORT int iit_ln_fwd_sel(const float* x, const float* w, const float* b, void* y, float* mean, float* rstd,
                              int T, int d, float eps, unsigned long long pos_mask, int S, int Tb, void* stream) {
  const RowSel sel{pos_mask, S > 0 ? S : 1, Tb};
  if (pos_mask && (S <= 0 || S > 64 || 2 * (long)Tb > T)) return (int)hipErrorInvalidValue;
  dim3 grid((T + 3) / 4), block(256);
  hipStream_t s = (hipStream_t)stream;
  const bool vec = d % 4 == 0 && aligned16(x) && (((uintptr_t)y) & 7) == 0 && (!w || (aligned16(w) && aligned16(b)));
  if (vec && d <= 4096) {
#define LNF(V) hipLaunchKernelGGL((ln_fwd_vec_kernel<V>), grid, block, 0, s, x, w, b, (__bf16*)y, mean, rstd, T, d, eps, sel)
    const int v4 = (d / 4 + 63) / 64;
    if (v4 <= 1) LNF(1); else if (v4 <= 2) LNF(2); else if (v4 <= 3) LNF(3); else if (v4 <= 4) LNF(4);
    else if (v4 <= 6) LNF(6); else if (v4 <= 8) LNF(8); else if (v4 <= 12) LNF(12); else LNF(16);
#undef LNF
    return hipGetLastError();
  }
  if (d <= 256) hipLaunchKernelGGL((ln_fwd_kernel<4>), grid, block, 0, s, x, w, b, (__bf16*)y, mean, rstd, T, d, eps, sel);
  else if (d <= 1024) hipLaunchKernelGGL((ln_fwd_kernel<16>), grid, block, 0, s, x, w, b, (__bf16*)y, mean, rstd, T, d, eps, sel);
  else if (d <= 2048) hipLaunchKernelGGL((ln_fwd_kernel<32>), grid, block, 0, s, x, w, b, (__bf16*)y, mean, rstd, T, d, eps, sel);
  else if (d <= 4096) hipLaunchKernelGGL((ln_fwd_kernel<64>), grid, block, 0, s, x, w, b, (__bf16*)y, mean, rstd, T, d, eps, sel);
  else return (int)hipErrorInvalidValue;
  return hipGetLastError();
}

// dx = rstd * (g - mean(g) - xhat * mean(g * xhat)) (+ dres),  g = dy * w.
// ``dres`` (nullable) is the residual stream's skip-connection gradient: fusing it here saves autograd's
// separate gradient-sum pass over the fp32 residual.  ``dx16`` (nullable) receives a bf16 copy of dx: the
// next backward GEMMs (W_O / W_out dX and dW) read bf16, so the cast rides along with this pass.
// The affine gradients dw/db are NOT done here (see ln_dwdb_kernel: per-block partial sums, few atomics).
// XH16: ``x`` is the forward's bf16 output xhat of a norm without affine parameters (LNPre): 2 bytes per element
// instead of the fp32 input, and no mean
template <int V4, bool DY_F32, bool XH16 = false>
__global__ __launch_bounds__(256) void ln_bwd_vec_kernel(const void* __restrict__ dy_, const float* __restrict__ x,
                                                         const float* __restrict__ mean, const float* __restrict__ rstd,
                                                         const float* __restrict__ w, float* __restrict__ dx,
                                                         const float* __restrict__ dres, __bf16* __restrict__ dx16,
                                                         int T, int d, int accumulate, RowSel sel) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= T) return;
  const int d4 = d >> 2;
  const bool dead = sel_hit(sel, row);  // a spliced row: its output came from the source row (no gradient here)
  const float mu = mean[row], rs = rstd[row];
  float4 g[V4], xh[V4];
  float sg = 0.f, sgx = 0.f;
#pragma unroll
  for (int i = 0; i < V4; ++i) {
    const int c = lane + i * 64;
    float4 dy = make_float4(0.f, 0.f, 0.f, 0.f), xv = dy;
    if (c < d4 && !dead) {
      if (DY_F32) {
        dy = ((const float4*)dy_)[(long)row * d4 + c];
      } else {
        const bf16x4 t = ((const bf16x4*)dy_)[(long)row * d4 + c];
        dy = make_float4(bf2f(t[0]), bf2f(t[1]), bf2f(t[2]), bf2f(t[3]));
      }
      if constexpr (XH16) {
        const bf16x4 t = ((const bf16x4*)x)[(long)row * d4 + c];
        xv = make_float4(bf2f(t[0]), bf2f(t[1]), bf2f(t[2]), bf2f(t[3]));
      } else {
        const float4 xx = ((const float4*)x)[(long)row * d4 + c];
        xv = make_float4((xx.x - mu) * rs, (xx.y - mu) * rs, (xx.z - mu) * rs, (xx.w - mu) * rs);
      }
      if (w) {
        const float4 ww = ((const float4*)w)[c];
        dy.x *= ww.x; dy.y *= ww.y; dy.z *= ww.z; dy.w *= ww.w;
      }
    }
    g[i] = dy;
    xh[i] = xv;
    sg += (dy.x + dy.y) + (dy.z + dy.w);
    sgx += (dy.x * xv.x + dy.y * xv.y) + (dy.z * xv.z + dy.w * xv.w);
  }
  sg = wave_sum(sg) / d;
  sgx = wave_sum(sgx) / d;
#pragma unroll
  for (int i = 0; i < V4; ++i) {
    const int c = lane + i * 64;
    if (c < d4) {
      float4 o = make_float4(rs * (g[i].x - sg - xh[i].x * sgx), rs * (g[i].y - sg - xh[i].y * sgx),
                             rs * (g[i].z - sg - xh[i].z * sgx), rs * (g[i].w - sg - xh[i].w * sgx));
      if (dres) {
        const float4 r = ((const float4*)dres)[(long)row * d4 + c];
        o.x += r.x; o.y += r.y; o.z += r.z; o.w += r.w;
      }
      float4* p = (float4*)dx + (long)row * d4 + c;
      if (accumulate) {
        const float4 q = *p;
        o.x += q.x; o.y += q.y; o.z += q.z; o.w += q.w;
      }
      *p = o;
      if (dx16) {
        bf16x4 ob = {f2bf(o.x), f2bf(o.y), f2bf(o.z), f2bf(o.w)};
        ((bf16x4*)dx16)[(long)row * d4 + c] = ob;
      }
    }
  }
}

// Affine LN parameter gradients: dw[c] += sum_t dy[t][c] * xhat[t][c], db[c] += sum_t dy[t][c].
// Block = 64 columns x 256 rows (4 waves x 64 rows), LDS combine, one atomic per column per block.
template <bool DY_F32>
__global__ __launch_bounds__(256) void ln_dwdb_kernel(const void* __restrict__ dy_, const float* __restrict__ x,
                                                      const float* __restrict__ mean, const float* __restrict__ rstd,
                                                      float* __restrict__ dw, float* __restrict__ db, int T, int d,
                                                      RowSel sel) {
  __shared__ float pw[4][64], pb[4][64];
  const int c = blockIdx.x * 64 + (threadIdx.x & 63), wv = threadIdx.x >> 6;
  const int t0 = blockIdx.y * 256;
  float sw = 0.f, sb = 0.f;
  if (c < d)
    for (int i = 0; i < 64; ++i) {
      const int t = t0 + wv * 64 + i;
      if (t >= T) break;
      if (sel_hit(sel, t)) continue;
      const float dy = DY_F32 ? ((const float*)dy_)[(long)t * d + c] : bf2f(((const __bf16*)dy_)[(long)t * d + c]);
      sw += dy * (x[(long)t * d + c] - mean[t]) * rstd[t];
      sb += dy;
    }
  pw[wv][threadIdx.x & 63] = sw;
  pb[wv][threadIdx.x & 63] = sb;
  __syncthreads();
  if (wv == 0 && c < d) {
    const int l = threadIdx.x;
    atomicAdd(dw + c, pw[0][l] + pw[1][l] + pw[2][l] + pw[3][l]);
    atomicAdd(db + c, pb[0][l] + pb[1][l] + pb[2][l] + pb[3][l]);
  }
}

// Vectorised affine gradients (d % 4 == 0, 16-B aligned rows): a wave covers 256 columns as float4 lanes, the block's 4
// waves take interleaved rows of a 32-row chunk with all 8 rows' loads issued before the first use, and the waves meet
// in LDS for one atomic per column per block.  ~700 blocks at T = 7680 (the 64-column kernel above ran 180-360
// blocks of 64 serial dependent loads per thread: 29 us for [7680][768], profiles/mqnli_step_breakdown_r4.txt).
constexpr int LN_DWDB_ROWS = 32;
template <bool DY_F32>
__global__ __launch_bounds__(256) void ln_dwdb_vec_kernel(const void* __restrict__ dy_, const float* __restrict__ x,
                                                          const float* __restrict__ mean,
                                                          const float* __restrict__ rstd, float* __restrict__ dw,
                                                          float* __restrict__ db, int T, int d, RowSel sel) {
  __shared__ float4 pw[4][64], pb[4][64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int d4 = d >> 2;
  const int c4 = blockIdx.x * 64 + lane;
  const int r0 = blockIdx.y * LN_DWDB_ROWS;
  float4 sw = make_float4(0.f, 0.f, 0.f, 0.f), sb = sw;
  if (c4 < d4) {
    constexpr int R = LN_DWDB_ROWS / 4;
    float4 g[R], xv[R];
    float mu[R], rs[R];
#pragma unroll
    for (int i = 0; i < R; ++i) {
      const int t = r0 + wv + 4 * i;
      const bool live = t < T && !sel_hit(sel, t);
      g[i] = make_float4(0.f, 0.f, 0.f, 0.f);
      xv[i] = g[i];
      mu[i] = 0.f;
      rs[i] = 0.f;
      if (live) {
        if (DY_F32) {
          g[i] = ((const float4*)dy_)[(long)t * d4 + c4];
        } else {
          const bf16x4 b = ((const bf16x4*)dy_)[(long)t * d4 + c4];
          g[i] = make_float4(bf2f(b[0]), bf2f(b[1]), bf2f(b[2]), bf2f(b[3]));
        }
        xv[i] = ((const float4*)x)[(long)t * d4 + c4];
        mu[i] = mean[t];
        rs[i] = rstd[t];
      }
    }
#pragma unroll
    for (int i = 0; i < R; ++i) {
      sw.x += g[i].x * (xv[i].x - mu[i]) * rs[i];
      sw.y += g[i].y * (xv[i].y - mu[i]) * rs[i];
      sw.z += g[i].z * (xv[i].z - mu[i]) * rs[i];
      sw.w += g[i].w * (xv[i].w - mu[i]) * rs[i];
      sb.x += g[i].x; sb.y += g[i].y; sb.z += g[i].z; sb.w += g[i].w;
    }
  }
  pw[wv][lane] = sw;
  pb[wv][lane] = sb;
  __syncthreads();
  if (wv == 0 && c4 < d4) {
    const float4 a = pw[0][lane], b = pw[1][lane], c = pw[2][lane], e = pw[3][lane];
    const float4 p = pb[0][lane], q = pb[1][lane], r = pb[2][lane], u = pb[3][lane];
    float* w4 = dw + 4 * c4;
    float* b4 = db + 4 * c4;
    atomicAdd(w4 + 0, (a.x + b.x) + (c.x + e.x));
    atomicAdd(w4 + 1, (a.y + b.y) + (c.y + e.y));
    atomicAdd(w4 + 2, (a.z + b.z) + (c.z + e.z));
    atomicAdd(w4 + 3, (a.w + b.w) + (c.w + e.w));
    atomicAdd(b4 + 0, (p.x + q.x) + (r.x + u.x));
    atomicAdd(b4 + 1, (p.y + q.y) + (r.y + u.y));
    atomicAdd(b4 + 2, (p.z + q.z) + (r.z + u.z));
    atomicAdd(b4 + 3, (p.w + q.w) + (r.w + u.w));
  }
}

// ln_bwd_vec_kernel with the affine gradients fused: each wave takes R rows (row = block * 4R + 4 r + wave), so a
// lane keeps the same float4 columns for all of them and sums dy * xhat and dy in registers; the block's 4 waves
// meet in LDS and write ONE partial row pair (dw part, db part) to ``part[block][2 d]`` with plain stores -- no
// atomics here (the separate ln_dwdb kernels re-read dy and x and did one memory-side fp32 atomic per column per
// 32 rows: ~17 us for [3840][768], profiles/mqnli_step_breakdown_r5.txt).  ln_part_reduce_kernel sums the partials.
// R = rows per wave (the block covers 4 R rows): IIT_LN_PART_R = 1 / 2 / 4, default 1 -- the MQNLI (BERT-base)
// step measured 11.93-11.96 ms at R = 1, 12.03-12.04 at 2 and 12.38-12.40 at 4 (interleaved, one box;
// profiles/mqnli_native_r6.txt): more, shorter blocks beat the smaller partial array
static int ln_part_r() {
  static const int r = [] {
    const char* e = getenv("IIT_LN_PART_R");
    const int v = e ? atoi(e) : 1;
    return (v == 2 || v == 4) ? v : 1;
  }();
  return r;
}
template <int V4, bool DY_F32, int LN_FUSED_R>
__global__ __launch_bounds__(256) void ln_bwd_part_vec_kernel(const void* __restrict__ dy_, const float* __restrict__ x,
                                                              const float* __restrict__ mean,
                                                              const float* __restrict__ rstd,
                                                              const float* __restrict__ w, float* __restrict__ dx,
                                                              const float* __restrict__ dres,
                                                              __bf16* __restrict__ dx16, float* __restrict__ part,
                                                              int T, int d, int accumulate, RowSel sel,
                                                              const float* __restrict__ dy2) {
  __shared__ float4 red[2][4][64 * V4];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int d4 = d >> 2;
  float4 pw[V4], pb[V4];
#pragma unroll
  for (int i = 0; i < V4; ++i) pw[i] = pb[i] = make_float4(0.f, 0.f, 0.f, 0.f);
  float4 ww[V4];
#pragma unroll
  for (int i = 0; i < V4; ++i) {
    const int c = lane + i * 64;
    ww[i] = (w && c < d4) ? ((const float4*)w)[c] : make_float4(1.f, 1.f, 1.f, 1.f);
  }
  // every row's operands are loaded before the first is used: the R rows' memory latency overlaps
  float4 dyv[LN_FUSED_R][V4], xvv[LN_FUSED_R][V4];
  float muv[LN_FUSED_R], rsv[LN_FUSED_R];
#pragma unroll
  for (int r = 0; r < LN_FUSED_R; ++r) {
    const int row = blockIdx.x * 4 * LN_FUSED_R + 4 * r + wave;
    const bool live = row < T && !sel_hit(sel, row);
    muv[r] = row < T ? mean[row] : 0.f;
    rsv[r] = row < T ? rstd[row] : 0.f;
#pragma unroll
    for (int i = 0; i < V4; ++i) {
      const int c = lane + i * 64;
      dyv[r][i] = make_float4(0.f, 0.f, 0.f, 0.f);
      xvv[r][i] = dyv[r][i];
      if (c < d4 && live) {
        if (DY_F32) {
          dyv[r][i] = ((const float4*)dy_)[(long)row * d4 + c];
        } else {
          const bf16x4 t = ((const bf16x4*)dy_)[(long)row * d4 + c];
          dyv[r][i] = make_float4(bf2f(t[0]), bf2f(t[1]), bf2f(t[2]), bf2f(t[3]));
        }
        if (dy2) {  // the fp32 twin output's gradient (LayerNormTwinFn): dy = dy + dy2
          const float4 e = ((const float4*)dy2)[(long)row * d4 + c];
          dyv[r][i].x += e.x; dyv[r][i].y += e.y; dyv[r][i].z += e.z; dyv[r][i].w += e.w;
        }
        xvv[r][i] = ((const float4*)x)[(long)row * d4 + c];
      }
    }
  }
#pragma unroll
  for (int r = 0; r < LN_FUSED_R; ++r) {
    const int row = blockIdx.x * 4 * LN_FUSED_R + 4 * r + wave;
    if (row >= T) break;
    const bool dead = sel_hit(sel, row);
    const float mu = muv[r], rs = rsv[r];
    float4 g[V4], xh[V4];
    float sg = 0.f, sgx = 0.f;
#pragma unroll
    for (int i = 0; i < V4; ++i) {
      float4 dy = dyv[r][i];
      const float4 xx = xvv[r][i];
      const float4 xv = dead ? make_float4(0.f, 0.f, 0.f, 0.f)
                             : make_float4((xx.x - mu) * rs, (xx.y - mu) * rs, (xx.z - mu) * rs, (xx.w - mu) * rs);
      // affine partials from the raw dy (dw += dy * xhat, db += dy), then g = dy * w
      pw[i].x += dy.x * xv.x; pw[i].y += dy.y * xv.y; pw[i].z += dy.z * xv.z; pw[i].w += dy.w * xv.w;
      pb[i].x += dy.x; pb[i].y += dy.y; pb[i].z += dy.z; pb[i].w += dy.w;
      dy.x *= ww[i].x; dy.y *= ww[i].y; dy.z *= ww[i].z; dy.w *= ww[i].w;
      g[i] = dy;
      xh[i] = xv;
      sg += (dy.x + dy.y) + (dy.z + dy.w);
      sgx += (dy.x * xv.x + dy.y * xv.y) + (dy.z * xv.z + dy.w * xv.w);
    }
    sg = wave_sum(sg) / d;
    sgx = wave_sum(sgx) / d;
#pragma unroll
    for (int i = 0; i < V4; ++i) {
      const int c = lane + i * 64;
      if (c < d4) {
        float4 o = make_float4(rs * (g[i].x - sg - xh[i].x * sgx), rs * (g[i].y - sg - xh[i].y * sgx),
                               rs * (g[i].z - sg - xh[i].z * sgx), rs * (g[i].w - sg - xh[i].w * sgx));
        if (dres) {
          const float4 q = ((const float4*)dres)[(long)row * d4 + c];
          o.x += q.x; o.y += q.y; o.z += q.z; o.w += q.w;
        }
        float4* p = (float4*)dx + (long)row * d4 + c;
        if (accumulate) {
          const float4 q = *p;
          o.x += q.x; o.y += q.y; o.z += q.z; o.w += q.w;
        }
        *p = o;
        if (dx16) {
          bf16x4 ob = {f2bf(o.x), f2bf(o.y), f2bf(o.z), f2bf(o.w)};
          ((bf16x4*)dx16)[(long)row * d4 + c] = ob;
        }
      }
    }
  }
#pragma unroll
  for (int i = 0; i < V4; ++i) {
    red[0][wave][lane + i * 64] = pw[i];
    red[1][wave][lane + i * 64] = pb[i];
  }
  __syncthreads();
  // 256 threads write the block's 2 x d4 float4 partials
  float4* out = (float4*)(part + (long)blockIdx.x * 2 * d);
  for (int k = threadIdx.x; k < 2 * d4; k += 256) {
    const int which = k >= d4, c = which ? k - d4 : k;
    const float4 a = red[which][0][c], b = red[which][1][c], e = red[which][2][c], f = red[which][3][c];
    out[k] = make_float4((a.x + b.x) + (e.x + f.x), (a.y + b.y) + (e.y + f.y), (a.z + b.z) + (e.z + f.z),
                         (a.w + b.w) + (e.w + f.w));
  }
}

// dw[c] += sum_b part[b][c], db[c] += sum_b part[b][d + c]: thread = one float4 column of the 2 d, blockIdx.y = one of
// G groups of partial rows; one fp32 atomic per element per group (G <= 32)
__global__ __launch_bounds__(256) void ln_part_reduce_kernel(const float* __restrict__ part, int nblk, int d,
                                                             float* __restrict__ dw, float* __restrict__ db) {
  const int k = blockIdx.x * 256 + threadIdx.x;
  const int d4 = d >> 2;
  if (k >= 2 * d4) return;
  const int G = gridDim.y;
  const int per = (nblk + G - 1) / G, b0 = blockIdx.y * per, b1 = min(nblk, b0 + per);
  if (b1 <= b0) return;
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
  int b = b0;
  for (; b + 4 <= b1; b += 4) {  // four independent loads in flight
    const float4 v0 = ((const float4*)(part + (long)b * 2 * d))[k];
    const float4 v1 = ((const float4*)(part + (long)(b + 1) * 2 * d))[k];
    const float4 v2 = ((const float4*)(part + (long)(b + 2) * 2 * d))[k];
    const float4 v3 = ((const float4*)(part + (long)(b + 3) * 2 * d))[k];
    s.x += (v0.x + v1.x) + (v2.x + v3.x);
    s.y += (v0.y + v1.y) + (v2.y + v3.y);
    s.z += (v0.z + v1.z) + (v2.z + v3.z);
    s.w += (v0.w + v1.w) + (v2.w + v3.w);
  }
  for (; b < b1; ++b) {
    const float4 v = ((const float4*)(part + (long)b * 2 * d))[k];
    s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
  }
  float* dst = k < d4 ? dw + 4 * k : db + 4 * (k - d4);
  atomicAdd(dst + 0, s.x);
  atomicAdd(dst + 1, s.y);
  atomicAdd(dst + 2, s.z);
  atomicAdd(dst + 3, s.w);
}

// scalar fallback (any d <= 4096, any alignment)
template <int VPL, bool DY_F32>
__global__ __launch_bounds__(256) void ln_bwd_kernel(const void* __restrict__ dy_, const float* __restrict__ x,
                                                     const float* __restrict__ mean, const float* __restrict__ rstd,
                                                     const float* __restrict__ w, float* __restrict__ dx,
                                                     const float* __restrict__ dres, __bf16* __restrict__ dx16,
                                                     int T, int d, int accumulate, RowSel sel) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= T) return;
  const bool dead = sel_hit(sel, row);
  const float mu = mean[row], rs = rstd[row];
  float g[VPL], xh[VPL];
  float sg = 0.f, sgx = 0.f;
#pragma unroll
  for (int i = 0; i < VPL; ++i) {
    const int c = lane + i * 64;
    float dy = 0.f, xv = 0.f;
    if (c < d && !dead) {
      dy = DY_F32 ? ((const float*)dy_)[(long)row * d + c] : bf2f(((const __bf16*)dy_)[(long)row * d + c]);
      xv = (x[(long)row * d + c] - mu) * rs;
      if (w) dy *= w[c];
    }
    g[i] = dy;
    xh[i] = xv;
    sg += dy;
    sgx += dy * xv;
  }
  sg = wave_sum(sg) / d;
  sgx = wave_sum(sgx) / d;
#pragma unroll
  for (int i = 0; i < VPL; ++i) {
    const int c = lane + i * 64;
    if (c < d) {
      float o = rs * (g[i] - sg - xh[i] * sgx);
      if (dres) o += dres[(long)row * d + c];
      float* p = dx + (long)row * d + c;
      o = accumulate ? *p + o : o;
      *p = o;
      if (dx16) dx16[(long)row * d + c] = f2bf(o);
    }
  }
}

IIT_EXPORT int iit_ln_bwd_sel(const void* dy, int dy_f32, const float* x, const float* mean, const float* rstd,
                              const float* w, float* dx, const float* dres, void* dx16, float* dw, float* db, int T,
                              int d, int accumulate, unsigned long long pos_mask, int S, void* stream);
IIT_EXPORT int iit_ln_bwd_part(const void* dy, int dy_f32, const float* x, const float* mean, const float* rstd,
                               const float* w, float* dx, const float* dres, void* dx16, float* dw, float* db,
                               float* part, int T, int d, int accumulate, unsigned long long pos_mask, int S,
                               const float* dy2, void* stream);

IIT_EXPORT int iit_ln_bwd(const void* dy, int dy_f32, const float* x, const float* mean, const float* rstd,
                          const float* w, float* dx, const float* dres, void* dx16, float* dw, float* db, int T, int d,
                          int accumulate, void* stream) {
  return iit_ln_bwd_sel(dy, dy_f32, x, mean, rstd, w, dx, dres, dx16, dw, db, T, d, accumulate, 0ull, 1, stream);
}

// rows per block of the fused affine-gradient backward (the caller sizes ``part`` as blocks x 2 d floats)
IIT_EXPORT int iit_ln_bwd_part_rows() { return 4 * ln_part_r(); }

// iit_ln_bwd_sel with dw / db fused into the dx pass (ln_bwd_part_vec_kernel + ln_part_reduce_kernel); ``part``:
// ceil(T / iit_ln_bwd_part_rows()) x 2 d floats of scratch; ``dy2`` (nullable, fp32 [T, d]) is added to dy.  Falls
// back to iit_ln_bwd_sel when the vector layout does not apply (refused with a ``dy2``: the caller sums first).
IIT_EXPORT int iit_ln_bwd_part(const void* dy, int dy_f32, const float* x, const float* mean, const float* rstd,
                               const float* w, float* dx, const float* dres, void* dx16, float* dw, float* db,
                               float* part, int T, int d, int accumulate, unsigned long long pos_mask, int S,
                               const float* dy2, void* stream) {
  const bool vec = part && dw && db && d % 4 == 0 && d <= 1024 && aligned16(x) && aligned16(dx) &&
                   (!dres || aligned16(dres)) && (!w || aligned16(w)) && aligned16(dw) && aligned16(db) &&
                   aligned16(part) && (dy_f32 ? aligned16(dy) : (((uintptr_t)dy) & 7) == 0) &&
                   (((uintptr_t)dx16) & 7) == 0 && (!dy2 || aligned16(dy2));
  if (dy2 && !vec) return (int)hipErrorInvalidValue;
  if (!vec || T <= 0)
    return iit_ln_bwd_sel(dy, dy_f32, x, mean, rstd, w, dx, dres, dx16, dw, db, T, d, accumulate, pos_mask, S, stream);
  if (pos_mask && (S <= 0 || S > 64)) return (int)hipErrorInvalidValue;
  const RowSel sel{pos_mask, S > 0 ? S : 1, T};
  const int R = ln_part_r();
  const int nblk = (T + 4 * R - 1) / (4 * R);
  hipStream_t s = (hipStream_t)stream;
  __bf16* d16 = (__bf16*)dx16;
#define LNPR(V, RR)                                                                                              \
  if (dy_f32) hipLaunchKernelGGL((ln_bwd_part_vec_kernel<V, true, RR>), dim3(nblk), dim3(256), 0, s, dy, x, mean, rstd, w, dx, dres, d16, part, T, d, accumulate, sel, dy2); \
  else hipLaunchKernelGGL((ln_bwd_part_vec_kernel<V, false, RR>), dim3(nblk), dim3(256), 0, s, dy, x, mean, rstd, w, dx, dres, d16, part, T, d, accumulate, sel, dy2);
#define LNP(V) if (R == 1) { LNPR(V, 1) } else if (R == 4) { LNPR(V, 4) } else { LNPR(V, 2) }
  const int v4 = (d / 4 + 63) / 64;
  if (v4 <= 1) { LNP(1) } else if (v4 <= 2) { LNP(2) } else if (v4 <= 3) { LNP(3) } else { LNP(4) }
#undef LNP
#undef LNPR
  static const int gcap = [] {  // IIT_LN_REDUCE_G: most groups of partial rows (default 32)
    const char* e = getenv("IIT_LN_REDUCE_G");
    const int v = e ? atoi(e) : 32;
    return v >= 1 && v <= 1024 ? v : 32;
  }();
  const int G = max(1, min(gcap, nblk / 8));  // >= ~8 partial rows per thread
  hipLaunchKernelGGL(ln_part_reduce_kernel, dim3((2 * (d / 4) + 255) / 256, G), dim3(256), 0, s, part, nblk, d, dw, db);
  return hipGetLastError();
}

// LNPre backward from the forward's bf16 output (``xh`` = xhat, [T, d]); no affine parameters, no row select
IIT_EXPORT int iit_ln_bwd_xh16(const void* dy, int dy_f32, const void* xh, const float* rstd, float* dx,
                               const float* dres, void* dx16, int T, int d, int accumulate, void* stream) {
  if (d % 4 || d > 4096 || (((uintptr_t)xh) & 7) || !aligned16(dx) || (dres && !aligned16(dres)) ||
      (dy_f32 ? !aligned16(dy) : (((uintptr_t)dy) & 7) != 0) || (((uintptr_t)dx16) & 7))
    return (int)hipErrorInvalidValue;
  const RowSel sel{0ull, 1, T};
  dim3 grid((T + 3) / 4), block(256);
  hipStream_t s = (hipStream_t)stream;
  __bf16* d16 = (__bf16*)dx16;
  const float* x = (const float*)xh;
#define LNBX(V)                                                                                                   \
  if (dy_f32) hipLaunchKernelGGL((ln_bwd_vec_kernel<V, true, true>), grid, block, 0, s, dy, x, rstd, rstd, nullptr, dx, dres, d16, T, d, accumulate, sel); \
  else hipLaunchKernelGGL((ln_bwd_vec_kernel<V, false, true>), grid, block, 0, s, dy, x, rstd, rstd, nullptr, dx, dres, d16, T, d, accumulate, sel);
  const int v4 = (d / 4 + 63) / 64;
  if (v4 <= 1) { LNBX(1) } else if (v4 <= 2) { LNBX(2) } else if (v4 <= 3) { LNBX(3) } else if (v4 <= 4) { LNBX(4) }
  else if (v4 <= 6) { LNBX(6) } else if (v4 <= 8) { LNBX(8) } else if (v4 <= 12) { LNBX(12) } else { LNBX(16) }
#undef LNBX
  return hipGetLastError();
}

// backward of iit_ln_fwd_sel over the base rows (T = Tb): rows at masked positions get dx = dres only and add
// nothing to dw / db
IIT_EXPORT int iit_ln_bwd_sel(const void* dy, int dy_f32, const float* x, const float* mean, const float* rstd,
                              const float* w, float* dx, const float* dres, void* dx16, float* dw, float* db, int T,
                              int d, int accumulate, unsigned long long pos_mask, int S, void* stream) {
  const RowSel sel{pos_mask, S > 0 ? S : 1, T};
  if (pos_mask && (S <= 0 || S > 64)) return (int)hipErrorInvalidValue;
  dim3 grid((T + 3) / 4), block(256);
  hipStream_t s = (hipStream_t)stream;
  __bf16* d16 = (__bf16*)dx16;
  const bool vec = d % 4 == 0 && d <= 4096 && aligned16(x) && aligned16(dx) && (!dres || aligned16(dres)) &&
                   (!w || aligned16(w)) && (dy_f32 ? aligned16(dy) : (((uintptr_t)dy) & 7) == 0) &&
                   (((uintptr_t)dx16) & 7) == 0;
  if (vec) {
#define LNBV(V)                                                                                                   \
  if (dy_f32) hipLaunchKernelGGL((ln_bwd_vec_kernel<V, true>), grid, block, 0, s, dy, x, mean, rstd, w, dx, dres, d16, T, d, accumulate, sel); \
  else hipLaunchKernelGGL((ln_bwd_vec_kernel<V, false>), grid, block, 0, s, dy, x, mean, rstd, w, dx, dres, d16, T, d, accumulate, sel);
    const int v4 = (d / 4 + 63) / 64;
    if (v4 <= 1) { LNBV(1) } else if (v4 <= 2) { LNBV(2) } else if (v4 <= 3) { LNBV(3) } else if (v4 <= 4) { LNBV(4) }
    else if (v4 <= 6) { LNBV(6) } else if (v4 <= 8) { LNBV(8) } else if (v4 <= 12) { LNBV(12) } else { LNBV(16) }
#undef LNBV
  } else {
#define LNB(V)                                                                                                   \
  if (dy_f32) hipLaunchKernelGGL((ln_bwd_kernel<V, true>), grid, block, 0, s, dy, x, mean, rstd, w, dx, dres, d16, T, d, accumulate, sel); \
  else hipLaunchKernelGGL((ln_bwd_kernel<V, false>), grid, block, 0, s, dy, x, mean, rstd, w, dx, dres, d16, T, d, accumulate, sel);
    if (d <= 256) { LNB(4) }
    else if (d <= 1024) { LNB(16) }
    else if (d <= 2048) { LNB(32) }
    else if (d <= 4096) { LNB(64) }
    else return (int)hipErrorInvalidValue;
#undef LNB
  }
  if (dw) {
    const bool v4 = d % 4 == 0 && aligned16(x) && aligned16(dw) && aligned16(db) &&
                    (dy_f32 ? aligned16(dy) : (((uintptr_t)dy) & 7) == 0);
    if (v4) {
      dim3 g2((d / 4 + 63) / 64, (T + LN_DWDB_ROWS - 1) / LN_DWDB_ROWS);
      if (dy_f32) hipLaunchKernelGGL(ln_dwdb_vec_kernel<true>, g2, block, 0, s, dy, x, mean, rstd, dw, db, T, d, sel);
      else hipLaunchKernelGGL(ln_dwdb_vec_kernel<false>, g2, block, 0, s, dy, x, mean, rstd, dw, db, T, d, sel);
    } else {
      dim3 g2((d + 63) / 64, (T + 255) / 256);
      if (dy_f32) hipLaunchKernelGGL(ln_dwdb_kernel<true>, g2, block, 0, s, dy, x, mean, rstd, dw, db, T, d, sel);
      else hipLaunchKernelGGL(ln_dwdb_kernel<false>, g2, block, 0, s, dy, x, mean, rstd, dw, db, T, d, sel);
    }
  }
  return hipGetLastError();
}

// ============================================================================ attention (S <= 64)
// qkv: [B*S, ld_qkv] bf16 with q at column h*dh, k at HD + h*dh, v at 2*HD + h*dh (HD = H*dh).
// z:   [B*S, ld_z] bf16 at column h*dh.  lse: [B*H*S] fp32.
// head_mask bit h set => z[:, h] := zsrc[:, h] (interchange splice of hook_z).
__global__ __launch_bounds__(64) void attn_small_fwd_kernel(const __bf16* __restrict__ qkv, __bf16* __restrict__ z,
                                                            float* __restrict__ lse, const __bf16* __restrict__ zsrc,
                                                            unsigned long long head_mask, int B, int S, int H, int dh,
                                                            long ld_qkv, long ld_z, long ld_src, float scale, int causal) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int bh = blockIdx.x, b = bh / H, h = bh % H;
  const int lane = threadIdx.x;
  const int HD = H * dh;
  const long row0 = (long)b * S;
  if ((head_mask >> h) & 1ull) {
    for (int i = lane; i < S * dh; i += 64) {
      const int s = i / dh, e = i % dh;
      z[(row0 + s) * ld_z + h * dh + e] = zsrc[(row0 + s) * ld_src + h * dh + e];
    }
    if (lse)
      for (int s = lane; s < S; s += 64) lse[(long)bh * S + s] = 0.f;
    return;
  }
  const int P = dh + 1;
  float* q = sm;
  float* k = q + S * P;
  float* v = k + S * P;
  float* pr = v + S * P;  // [S][S+1]
  for (int i = lane; i < S * dh; i += 64) {
    const int s = i / dh, e = i % dh;
    const __bf16* r = qkv + (row0 + s) * ld_qkv + h * dh + e;
    q[s * P + e] = bf2f(r[0]);
    k[s * P + e] = bf2f(r[HD]);
    v[s * P + e] = bf2f(r[2 * HD]);
  }
  __syncthreads();
  const int SP = S + 1;
  for (int i = lane; i < S * S; i += 64) {
    const int qi = i / S, kj = i % S;
    float acc = -INFINITY;
    if (!causal || kj <= qi) {
      acc = 0.f;
      for (int e = 0; e < dh; ++e) acc += q[qi * P + e] * k[kj * P + e];
      acc *= scale;
    }
    pr[qi * SP + kj] = acc;
  }
  __syncthreads();
  for (int qi = lane; qi < S; qi += 64) {
    float m = -INFINITY;
    for (int kj = 0; kj < S; ++kj) m = fmaxf(m, pr[qi * SP + kj]);
    float sum = 0.f;
    for (int kj = 0; kj < S; ++kj) {
      const float e = pr[qi * SP + kj] == -INFINITY ? 0.f : __expf(pr[qi * SP + kj] - m);
      pr[qi * SP + kj] = e;
      sum += e;
    }
    const float inv = sum > 0.f ? 1.f / sum : 0.f;
    for (int kj = 0; kj < S; ++kj) pr[qi * SP + kj] *= inv;
    if (lse) lse[(long)bh * S + qi] = m + __logf(sum);
  }
  __syncthreads();
  for (int i = lane; i < S * dh; i += 64) {
    const int qi = i / dh, e = i % dh;
    float acc = 0.f;
    const int kmax = causal ? qi + 1 : S;
    for (int kj = 0; kj < kmax; ++kj) acc += pr[qi * SP + kj] * v[kj * P + e];
    z[(row0 + qi) * ld_z + h * dh + e] = f2bf(acc);
  }
}

IIT_EXPORT int iit_attn_small_fwd(const void* qkv, void* z, float* lse, const void* zsrc, unsigned long long head_mask,
                                  int B, int S, int H, int dh, long ld_qkv, long ld_z, long ld_src, float scale,
                                  int causal, void* stream) {
  if (S > 64 || dh > 128) return (int)hipErrorInvalidValue;
  const size_t lds = (size_t)(3 * S * (dh + 1) + S * (S + 1)) * sizeof(float);
  hipLaunchKernelGGL(attn_small_fwd_kernel, dim3(B * H), dim3(64), lds, (hipStream_t)stream, (const __bf16*)qkv,
                     (__bf16*)z, lse, (const __bf16*)zsrc, head_mask, B, S, H, dh, ld_qkv, ld_z, ld_src, scale, causal);
  return hipGetLastError();
}

// dqkv written in the qkv layout; patched heads get zero gradient.
__global__ __launch_bounds__(64) void attn_small_bwd_kernel(const __bf16* __restrict__ qkv, const __bf16* __restrict__ dz,
                                                            const float* __restrict__ lse, __bf16* __restrict__ dqkv,
                                                            unsigned long long head_mask, int B, int S, int H, int dh,
                                                            long ld_qkv, long ld_dz, float scale, int causal) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int bh = blockIdx.x, b = bh / H, h = bh % H;
  const int lane = threadIdx.x;
  const int HD = H * dh;
  const long row0 = (long)b * S;
  if ((head_mask >> h) & 1ull) {
    for (int i = lane; i < S * dh; i += 64) {
      const int s = i / dh, e = i % dh;
      __bf16* r = dqkv + (row0 + s) * ld_qkv + h * dh + e;
      r[0] = f2bf(0.f);
      r[HD] = f2bf(0.f);
      r[2 * HD] = f2bf(0.f);
    }
    return;
  }
  const int P = dh + 1, SP = S + 1;
  float* q = sm;
  float* k = q + S * P;
  float* v = k + S * P;
  float* g = v + S * P;   // dz
  float* pm = g + S * P;  // P  [S][S+1]
  float* ds = pm + S * SP; // dS
  for (int i = lane; i < S * dh; i += 64) {
    const int s = i / dh, e = i % dh;
    const __bf16* r = qkv + (row0 + s) * ld_qkv + h * dh + e;
    q[s * P + e] = bf2f(r[0]);
    k[s * P + e] = bf2f(r[HD]);
    v[s * P + e] = bf2f(r[2 * HD]);
    g[s * P + e] = bf2f(dz[(row0 + s) * ld_dz + h * dh + e]);
  }
  __syncthreads();
  // recompute P and dP
  for (int i = lane; i < S * S; i += 64) {
    const int qi = i / S, kj = i % S;
    float p = 0.f, dp = 0.f;
    if (!causal || kj <= qi) {
      float sc = 0.f;
      for (int e = 0; e < dh; ++e) sc += q[qi * P + e] * k[kj * P + e];
      p = __expf(sc * scale - lse[(long)bh * S + qi]);
      for (int e = 0; e < dh; ++e) dp += g[qi * P + e] * v[kj * P + e];
    }
    pm[qi * SP + kj] = p;
    ds[qi * SP + kj] = dp;
  }
  __syncthreads();
  for (int qi = lane; qi < S; qi += 64) {
    float dsum = 0.f;
    for (int kj = 0; kj < S; ++kj) dsum += pm[qi * SP + kj] * ds[qi * SP + kj];
    for (int kj = 0; kj < S; ++kj) ds[qi * SP + kj] = pm[qi * SP + kj] * (ds[qi * SP + kj] - dsum) * scale;
  }
  __syncthreads();
  for (int i = lane; i < S * dh; i += 64) {
    const int s = i / dh, e = i % dh;
    float dq = 0.f, dk = 0.f, dv = 0.f;
    for (int j = 0; j < S; ++j) {
      dq += ds[s * SP + j] * k[j * P + e];   // dQ[s] = sum_kj dS[s][kj] K[kj]
      dk += ds[j * SP + s] * q[j * P + e];   // dK[s] = sum_qi dS[qi][s] Q[qi]
      dv += pm[j * SP + s] * g[j * P + e];   // dV[s] = sum_qi P[qi][s] dZ[qi]
    }
    __bf16* r = dqkv + (row0 + s) * ld_qkv + h * dh + e;
    r[0] = f2bf(dq);
    r[HD] = f2bf(dk);
    r[2 * HD] = f2bf(dv);
  }
}

IIT_EXPORT int iit_attn_small_bwd(const void* qkv, const void* dz, const float* lse, void* dqkv,
                                  unsigned long long head_mask, int B, int S, int H, int dh, long ld_qkv, long ld_dz,
                                  float scale, int causal, void* stream) {
  if (S > 64 || dh > 128) return (int)hipErrorInvalidValue;
  const size_t lds = (size_t)(4 * S * (dh + 1) + 2 * S * (S + 1)) * sizeof(float);
  hipLaunchKernelGGL(attn_small_bwd_kernel, dim3(B * H), dim3(64), lds, (hipStream_t)stream, (const __bf16*)qkv,
                     (const __bf16*)dz, lse, (__bf16*)dqkv, head_mask, B, S, H, dh, ld_qkv, ld_dz, scale, causal);
  return hipGetLastError();
}

// ============================================================================ cross entropy
// Per row: loss = lse - x[label], lse = max + log(sum exp(x - max)), argmax (first index on ties).
// One 1024-thread block per row, a single pass with an online (max, sum) rescale and 16-byte loads.
__device__ __forceinline__ void online_add(float& m, float& s, int& mi, float v, int i) {
  if (v > m) {
    s = s * __expf(m - v) + 1.f;
    m = v;
    mi = i;
  } else {
    s += __expf(v - m);
  }
}

__device__ __forceinline__ void online_merge(float& m, float& s, int& mi, float om, float os, int oi) {
  if (om > m || (om == m && oi < mi)) {
    s = os + (m == -INFINITY ? 0.f : s * __expf(m - om));
    m = om;
    mi = oi;
  } else {
    s += (om == -INFINITY ? 0.f : os * __expf(om - m));
  }
}

__global__ __launch_bounds__(1024) void ce_fwd_kernel(const float* __restrict__ logits, long ld, const long* __restrict__ labels,
                                                      float* __restrict__ loss, float* __restrict__ lse_out,
                                                      long* __restrict__ amax, int V) {
  __shared__ float sm_m[16], sm_s[16];
  __shared__ int sm_i[16];
  const int row = blockIdx.x, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const float* x = logits + (long)row * ld;
  float m = -INFINITY, s = 0.f;
  int mi = 0x7fffffff;
  int head = 0;
  if ((((uintptr_t)x) & 15) == 0) {
    const int v4 = V / 4;
    for (int i = tid; i < v4; i += 1024) {
      const float4 q = ((const float4*)x)[i];
      online_add(m, s, mi, q.x, 4 * i);
      online_add(m, s, mi, q.y, 4 * i + 1);
      online_add(m, s, mi, q.z, 4 * i + 2);
      online_add(m, s, mi, q.w, 4 * i + 3);
    }
    head = v4 * 4;
  }
  for (int i = head + tid; i < V; i += 1024) online_add(m, s, mi, x[i], i);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float om = __shfl_xor(m, o, 64), os = __shfl_xor(s, o, 64);
    const int oi = __shfl_xor(mi, o, 64);
    online_merge(m, s, mi, om, os, oi);
  }
  if (lane == 0) { sm_m[w] = m; sm_s[w] = s; sm_i[w] = mi; }
  __syncthreads();
  if (tid == 0) {
    for (int j = 1; j < 16; ++j) online_merge(m, s, mi, sm_m[j], sm_s[j], sm_i[j]);
    const float l = m + __logf(s);
    if (lse_out) lse_out[row] = l;
    if (loss && labels) loss[row] = l - x[labels[row]];
    if (amax) amax[row] = mi;
  }
}

IIT_EXPORT int iit_ce_fwd(const float* logits, long ld, const long* labels, float* loss, float* lse, long* amax, int R,
                          int V, void* stream) {
  hipLaunchKernelGGL(ce_fwd_kernel, dim3(R), dim3(1024), 0, (hipStream_t)stream, logits, ld, labels, loss, lse, amax, V);
  return hipGetLastError();
}

// dlogits = (softmax - onehot) * gscale[0] * inv_rows   (fp32 or bf16 out, ld_out may be padded; pad columns zeroed)
// ``out16`` (nullable, fp32 ``out`` only): a bf16 copy with the same row stride written in the same pass -- the operand
// the unembed backward GEMMs read, so they need no separate cast / re-pad of the [rows][vocab] gradient
template <typename OUT>
__global__ __launch_bounds__(256) void ce_bwd_kernel(const float* __restrict__ logits, long ld, const long* __restrict__ labels,
                                                     const float* __restrict__ lse, const float* __restrict__ gscale,
                                                     float inv_rows, OUT* __restrict__ out, long ld_out, int V,
                                                     __bf16* __restrict__ out16) {
  const int row = blockIdx.y;
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= ld_out) return;
  float v = 0.f;
  if (i < V) {
    const float p = __expf(logits[(long)row * ld + i] - lse[row]);
    v = (p - (i == labels[row] ? 1.f : 0.f)) * gscale[0] * inv_rows;
  }
  out[(long)row * ld_out + i] = (OUT)v;
  if (out16) out16[(long)row * ld_out + i] = f2bf(v);
}

IIT_EXPORT int iit_ce_bwd(const float* logits, long ld, const long* labels, const float* lse, const float* gscale,
                          float inv_rows, void* out, long ld_out, int R, int V, int out_bf16, void* out16,
                          void* stream) {
  dim3 grid((unsigned)((ld_out + 255) / 256), R);
  if (out_bf16)
    hipLaunchKernelGGL(ce_bwd_kernel<__bf16>, grid, dim3(256), 0, (hipStream_t)stream, logits, ld, labels, lse, gscale,
                       inv_rows, (__bf16*)out, ld_out, V, (__bf16*)nullptr);
  else
    hipLaunchKernelGGL(ce_bwd_kernel<float>, grid, dim3(256), 0, (hipStream_t)stream, logits, ld, labels, lse, gscale,
                       inv_rows, (float*)out, ld_out, V, (__bf16*)out16);
  return hipGetLastError();
}

// ============================================================================ optimizer
// partial sums of g^2 per block (grid-stride over float4)
// Stage 1 of the fused clip+Adam: per-block partial sums of g^2 (skipped when clip == 0) and the
// device-side step counter bump (block 0), so a captured graph replays with the right bias corrections.
// The optimizer walks a table of spans (start, length in float4 units, <= 1024 float4 each) over the arena
// instead of [0, n): rows that can never receive gradient (embedding rows of tokens absent from the dataset,
// positions past the sequence length) are left out -- with zero gradient and zero moments, Adam leaves them
// bit-identical, so skipping them is exact and saves their 30 B/element of HBM traffic.
struct Span {
  long start4;  // parameter / bf16-mirror offset (float4 units) in the arena
  long local4;  // gradient / Adam-moment offset: == start4 for the replicated optimizer; with optimizer-state
                // sharding (ZeRO-1, iit_amd/parallel/zero.py) the offset inside this rank's shard buffers
  int len4;
  int pad;
};

// ``gsq`` (nullable, 64 floats): sums of squares the weight-gradient GEMMs already added for the gradients they stored
// (their spans are left out of ``spans``); block 0 folds them into its partial and re-zeroes the slots for the next
// step
__global__ __launch_bounds__(256) void sumsq_span_kernel(const float* __restrict__ g, const Span* __restrict__ spans,
                                                         int nspans, float* __restrict__ part, int do_norm,
                                                         int* __restrict__ step, float* __restrict__ gsq) {
  __shared__ float sm[4];
  if (blockIdx.x == 0 && threadIdx.x == 0 && step) step[0] += 1;
  float s = 0.f;
  if (gsq && blockIdx.x == 0 && threadIdx.x < 64) {
    s = gsq[threadIdx.x];
    gsq[threadIdx.x] = 0.f;
  }
  if (!do_norm) return;
  const float4* g4 = (const float4*)g;
  for (int e = blockIdx.x; e < nspans; e += gridDim.x) {
    const Span sp = spans[e];
    for (int i = threadIdx.x; i < sp.len4; i += 256) {
      const float4 v = g4[sp.local4 + i];
      s += (v.x * v.x + v.y * v.y) + (v.z * v.z + v.w * v.w);
    }
  }
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) sm[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) part[blockIdx.x] = sm[0] + sm[1] + sm[2] + sm[3];
}

// Adam (torch semantics, amsgrad=False) with the clip coefficient computed on device from the partial sums,
// the bias corrections from the device step counter, and the bf16 mirror of the updated weights written in
// the same pass.  Streams: read g, p, m, v; write p, m, v, mirror (the clipped gradient is not written back).
// U float4 groups per thread per pass (j, j + 256, ...): all 4U loads are issued before the first use, so each thread
// keeps 64U bytes in flight (IIT_ADAM_UNROLL picks U at launch)
template <bool NT, int U>
__global__ __launch_bounds__(256) void adam_span_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                        float* __restrict__ m, float* __restrict__ v,
                                                        __bf16* __restrict__ mirror, const Span* __restrict__ spans,
                                                        int nspans, const float* __restrict__ part, int nparts,
                                                        float clip, float lr, float b1, float b2, float eps, float wd,
                                                        const float* __restrict__ hyper, int* __restrict__ step,
                                                        int* __restrict__ skipped) {
  // ``hyper`` (nullable): device copy of {lr, beta1, beta2, eps, weight_decay}.  A captured graph replays the
  // kernel arguments it saw at capture; reading the hyper-parameters from device memory lets the host change the
  // learning rate (an LR scheduler) between replays with one small copy.
  if (hyper) {
    lr = hyper[0];
    b1 = hyper[1];
    b2 = hyper[2];
    eps = hyper[3];
    wd = hyper[4];
  }
  __shared__ float coef_s;
  __shared__ int bad_s;
  if (threadIdx.x < 64) {
    float s = 0.f;
    if (clip > 0.f || skipped)
      for (int i = threadIdx.x; i < nparts; i += 64) s += part[i];
    s = wave_sum(s);
    if (threadIdx.x == 0) {
      coef_s = clip > 0.f ? fminf(1.f, clip / (sqrtf(s) + 1e-6f)) : 1.f;
      bad_s = skipped != nullptr && !isfinite(s);
    }
  }
  __syncthreads();
  if (bad_s) {  // non-finite gradient: skip the whole update (uniform over the grid), count it, undo the step bump
    if (blockIdx.x == 0 && threadIdx.x == 0) {
      step[0] -= 1;
      skipped[0] += 1;
    }
    return;
  }
  const float coef = coef_s;
  const float t = (float)step[0];
  const float bc1 = 1.f - powf(b1, t);
  const float bc2_sqrt = sqrtf(1.f - powf(b2, t));
  const float stepsz = lr / bc1;
  const float4* g4 = (const float4*)g;
  float4* p4 = (float4*)p;
  float4* m4 = (float4*)m;
  float4* v4 = (float4*)v;
  for (int e = blockIdx.x; e < nspans; e += gridDim.x) {
    const Span sp = spans[e];
    for (int j0 = threadIdx.x; j0 < sp.len4; j0 += 256 * U) {
      float4 gg[U], pp[U], mm[U], vv[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int j = j0 + u * 256;
        if (j < sp.len4) {
          const long i = sp.start4 + j;   // parameter / mirror
          const long li = sp.local4 + j;  // gradient / moments
          pp[u] = p4[i];
          // NT: the gradient and both moments are touched once per step -- stream them past the caches
          if (NT) {
            gg[u] = __builtin_bit_cast(float4, __builtin_nontemporal_load((const f32x4*)g4 + li));
            mm[u] = __builtin_bit_cast(float4, __builtin_nontemporal_load((const f32x4*)m4 + li));
            vv[u] = __builtin_bit_cast(float4, __builtin_nontemporal_load((const f32x4*)v4 + li));
          } else {
            gg[u] = g4[li];
            mm[u] = m4[li];
            vv[u] = v4[li];
          }
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int j = j0 + u * 256;
        if (j >= sp.len4) break;
        const long i = sp.start4 + j;
        const long li = sp.local4 + j;
        float* gs = (float*)&gg[u];
        float* ps = (float*)&pp[u];
        float* ms = (float*)&mm[u];
        float* vs = (float*)&vv[u];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          float gr = gs[k] * coef;
          if (wd != 0.f) gr += wd * ps[k];
          ms[k] = b1 * ms[k] + (1.f - b1) * gr;
          vs[k] = b2 * vs[k] + (1.f - b2) * gr * gr;
          ps[k] -= stepsz * ms[k] / (sqrtf(vs[k]) / bc2_sqrt + eps);
        }
        p4[i] = pp[u];
        if (NT) {
          __builtin_nontemporal_store(__builtin_bit_cast(f32x4, mm[u]), (f32x4*)m4 + li);
          __builtin_nontemporal_store(__builtin_bit_cast(f32x4, vv[u]), (f32x4*)v4 + li);
        } else {
          m4[li] = mm[u];
          v4[li] = vv[u];
        }
        if (mirror) {
          bf16x4 o = {f2bf(ps[0]), f2bf(ps[1]), f2bf(ps[2]), f2bf(ps[3])};
          ((bf16x4*)mirror)[i] = o;
        }
      }
    }
  }
}

// ``spans`` is a device array of ``nspans`` Span records (iit_adam_span_size() bytes each).  ``skipped``
// (nullable) enables the non-finite-gradient guard: the global norm is then always computed and a step whose
// gradient contains inf/nan leaves weights, moments and the step counter untouched.
// ``sq_spans`` / ``n_sq_spans`` (nullable: the Adam spans): the spans the norm pass reads -- the Adam spans minus
// the gradients whose sums of squares the weight-gradient GEMMs added into ``gsq`` (nullable, 64 floats)
IIT_EXPORT int iit_adam_flat(float* p, float* g, float* m, float* v, void* mirror, const void* spans, int nspans,
                             float* part, int nparts, float clip, float lr, float b1, float b2, float eps, float wd,
                             const float* hyper, int* step, int* skipped, const void* sq_spans, int n_sq_spans,
                             float* gsq, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  const bool norm = clip > 0.f || skipped != nullptr;
  const Span* sp = (const Span*)spans;
  const Span* ssp = sq_spans ? (const Span*)sq_spans : sp;
  hipLaunchKernelGGL(sumsq_span_kernel, dim3(norm ? nparts : 1), dim3(256), 0, s, g, ssp,
                     sq_spans ? n_sq_spans : nspans, part, (int)norm, step, gsq);
  // grid: up to 65536 workgroups -- one per span (<= 1024 float4 groups each, ~30 k for GPT-2-small), so the
  // hardware dispatcher balances the ragged spans; a fixed 4096-workgroup grid striding over ~7 spans each measured
  // 0.12 ms per headline step slower (15.851 vs 15.734 ms, two rounds, profiles/launch_knobs_r4s2.txt).  The cap
  // bounds the per-workgroup prologue (the clip coefficient from the norm partials) on 8 B-parameter arenas.
  // IIT_ADAM_MAX_BLOCKS overrides.
  static const int max_blocks = [] {
    const char* e = getenv("IIT_ADAM_MAX_BLOCKS");
    return e ? atoi(e) : 65536;
  }();
  const int blocks = min(nspans, max_blocks);
  static const int nt = [] {
    const char* e = getenv("IIT_ADAM_NT");
    return e ? atoi(e) : 1;
  }();
  static const int unroll = [] {
    const char* e = getenv("IIT_ADAM_UNROLL");
    // 4: with one workgroup per 1024-group span each thread then streams its span share in ONE pass (0.4 % on the
    // headline step over 2, profiles/launch_knobs_r4s2.txt; profiles/adam_microbench_r3s2.txt: 2 and 4 beat 1)
    return e ? atoi(e) : 4;
  }();
#define ADAM_LAUNCH(NT_, U_)                                                                                        \
  hipLaunchKernelGGL((adam_span_kernel<NT_, U_>), dim3(blocks), dim3(256), 0, s, p, g, m, v, (__bf16*)mirror, sp, \
                     nspans, part, nparts, clip, lr, b1, b2, eps, wd, hyper, step, skipped)
  if (nt) {
    if (unroll >= 4) ADAM_LAUNCH(true, 4);
    else if (unroll == 2) ADAM_LAUNCH(true, 2);
    else ADAM_LAUNCH(true, 1);
  } else {
    if (unroll >= 4) ADAM_LAUNCH(false, 4);
    else if (unroll == 2) ADAM_LAUNCH(false, 2);
    else ADAM_LAUNCH(false, 1);
  }
#undef ADAM_LAUNCH
  return hipGetLastError();
}

IIT_EXPORT int iit_adam_span_size() { return (int)sizeof(Span); }

// gsq[slot] += sum of squares of an fp32 [M][N] matrix (row stride ldc): the fused-norm share of a weight gradient
// that a library GEMM stored (the LDS-DMA kernels add theirs in the epilogue)
__global__ __launch_bounds__(256) void sumsq_2d_kernel(const float* __restrict__ c, long ldc, int M, int N,
                                                       float* __restrict__ gsq) {
  // work item = (row, 2048-column chunk); each thread keeps 8 independent loads in flight per item
  __shared__ float sm[4];
  const int chunks = (N + 2047) / 2048;
  float s = 0.f;
  for (long it = blockIdx.x; it < (long)M * chunks; it += gridDim.x) {
    const int r = (int)(it / chunks), c0 = (int)(it % chunks) * 2048;
    const float* row = c + (long)r * ldc;
    float v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int j = c0 + k * 256 + threadIdx.x;
      v[k] = j < N ? row[j] : 0.f;
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) s += v[k] * v[k];
  }
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) sm[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) atomicAdd(gsq + (blockIdx.x & 63), (sm[0] + sm[1]) + (sm[2] + sm[3]));
}

IIT_EXPORT int iit_sumsq_2d(const float* c, long ldc, int M, int N, float* gsq, void* stream) {
  const long items = (long)M * ((N + 2047) / 2048);
  hipLaunchKernelGGL(sumsq_2d_kernel, dim3((unsigned)(items < 2048 ? items : 2048)), dim3(256), 0,
                     (hipStream_t)stream, c, ldc, M, N, gsq);
  return hipGetLastError();
}

// The two stages separately, for the sharded optimizer (ZeRO-1, iit_amd/parallel/zero.py): per-block partial sums
// of g^2 over this rank's shard spans (+ the device step bump), then -- after the host all-reduces the partial total
// into ``total`` (one float) -- the Adam pass over the same spans with the global norm read from ``total``.
IIT_EXPORT int iit_sumsq_spans(const float* g, const void* spans, int nspans, float* part, int nparts, int do_norm,
                               int* step, void* stream) {
  hipLaunchKernelGGL(sumsq_span_kernel, dim3(do_norm ? nparts : 1), dim3(256), 0, (hipStream_t)stream, g,
                     (const Span*)spans, nspans, part, do_norm, step, (float*)nullptr);
  return hipGetLastError();
}

IIT_EXPORT int iit_adam_spans(float* p, const float* g, float* m, float* v, void* mirror, const void* spans,
                              int nspans, const float* total, float clip, float lr, float b1, float b2, float eps,
                              float wd, const float* hyper, int* step, int* skipped, void* stream) {
  // one workgroup per span up to 65536, as the replicated update (iit_adam_flat)
  const int blocks = max(1, min(nspans, 65536));
  // (U = 2: two float4 groups in flight per thread and stream, as the replicated update; profiles/adam_microbench_r3s2.txt)
  hipLaunchKernelGGL((adam_span_kernel<true, 2>), dim3(blocks), dim3(256), 0, (hipStream_t)stream, p, g, m, v,
                     (__bf16*)mirror, (const Span*)spans, nspans, total, 1, clip, lr, b1, b2, eps, wd, hyper, step,
                     skipped);
  return hipGetLastError();
}

// ============================================================================ shadow weights
// dst (bf16) = src (fp32) viewed as [rows][cols]; transpose -> dst[c][r] with leading dim ld.
// element (h, i, j) of src [heads][rows][cols] -> dst[h*dst_hs + i*ld + j]   (or transposed, heads == 1)
struct ShadowDesc {
  const float* src;
  __bf16* dst;
  int rows, cols;
  long ld;
  int heads;
  int transpose;
  long src_hs, dst_hs;
};

__global__ __launch_bounds__(256) void shadow_refresh_kernel(const ShadowDesc* __restrict__ descs) {
  __shared__ float tile[32][33];
  const ShadowDesc d = descs[blockIdx.y];
  if (!d.transpose) {
    const long total = (long)d.heads * d.rows;
    for (long r = blockIdx.x; r < total; r += gridDim.x) {
      const int h = (int)(r / d.rows), i = (int)(r % d.rows);
      const float* s = d.src + h * d.src_hs + (long)i * d.cols;
      __bf16* o = d.dst + h * d.dst_hs + (long)i * d.ld;
      const bool vec = ((((uintptr_t)s) & 15) == 0) && ((((uintptr_t)o) & 7) == 0);
      if (vec) {
        const int c4 = d.cols / 4;
        for (int j = threadIdx.x; j < c4; j += 256) {
          const float4 v = ((const float4*)s)[j];
          bf16x4 b = {f2bf(v.x), f2bf(v.y), f2bf(v.z), f2bf(v.w)};
          *(bf16x4*)(o + 4 * j) = b;
        }
        for (int j = c4 * 4 + threadIdx.x; j < d.cols; j += 256) o[j] = f2bf(s[j]);
      } else {
        for (int j = threadIdx.x; j < d.cols; j += 256) o[j] = f2bf(s[j]);
      }
    }
    return;
  }
  const int tiles_c = (d.cols + 31) / 32;
  const int ntiles = tiles_c * ((d.rows + 31) / 32);
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // 32 x 8
  for (int t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const int r0 = (t / tiles_c) * 32, c0 = (t % tiles_c) * 32;
    {
      for (int i = ty; i < 32; i += 8) {
        const int r = r0 + i, c = c0 + tx;
        tile[i][tx] = (r < d.rows && c < d.cols) ? d.src[(long)r * d.cols + c] : 0.f;
      }
      __syncthreads();
      for (int i = ty; i < 32; i += 8) {
        const int c = c0 + i, r = r0 + tx;
        if (r < d.rows && c < d.cols) d.dst[(long)c * d.ld + r] = f2bf(tile[tx][i]);
      }
      __syncthreads();
    }
  }
}

IIT_EXPORT int iit_shadow_refresh(const void* descs, int n, void* stream) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(shadow_refresh_kernel, dim3(512, n), dim3(256), 0, (hipStream_t)stream, (const ShadowDesc*)descs);
  return hipGetLastError();
}

IIT_EXPORT int iit_shadow_desc_size() { return (int)sizeof(ShadowDesc); }

// ============================================================================ small helpers
// db[n] (+)= sum_t x[t][n]     x bf16 or fp32.  Block = 64 columns x 64 rows, 4 waves each summing
// 16 rows of one coalesced 64-column row segment; LDS combine; one fp32 atomic per column per block.
template <bool F32>
__global__ __launch_bounds__(256) void colsum_kernel(const void* __restrict__ x, long ld, float* __restrict__ out, int T, int N) {
  __shared__ float part[4][64];
  const int c = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int n = blockIdx.x * 64 + c;
  const int t0 = blockIdx.y * 64;
  float s = 0.f;
  if (n < N) {
#pragma unroll 4
    for (int i = 0; i < 16; ++i) {
      const int t = t0 + w + 4 * i;
      if (t < T) s += F32 ? ((const float*)x)[(long)t * ld + n] : bf2f(((const __bf16*)x)[(long)t * ld + n]);
    }
  }
  part[w][c] = s;
  __syncthreads();
  if (w == 0 && n < N) atomicAdd(out + n, part[0][c] + part[1][c] + part[2][c] + part[3][c]);
}

// Vectorised variant: 256 threads = 32 column groups (16 B each: 8 bf16 / 4 fp32 columns) x 8 row groups,
// R rows per block (R % 8 == 0, chosen so the grid fills the 256 CUs); LDS combine over row groups, one fp32
// atomic per column per block.
template <bool F32>
__global__ __launch_bounds__(256) void colsum_vec_kernel(const void* __restrict__ x, long ld, float* __restrict__ out,
                                                         int T, int N, int R) {
  constexpr int CPT = F32 ? 4 : 8;  // columns per thread
  __shared__ float part[8][32 * CPT];
  const int cg = threadIdx.x & 31, rg = threadIdx.x >> 5;
  const int c0 = (blockIdx.x * 32 + cg) * CPT;
  const int t0 = blockIdx.y * R;
  const int t1 = min(T, t0 + R);
  float acc[CPT];
#pragma unroll
  for (int e = 0; e < CPT; ++e) acc[e] = 0.f;
  if (c0 < N) {
#pragma unroll 4
    for (int t = t0 + rg; t < t1; t += 8) {
      if (F32) {
        const float4 v = *(const float4*)((const float*)x + (long)t * ld + c0);
        acc[0] += v.x; acc[1] += v.y; acc[2] += v.z; acc[3] += v.w;
      } else {
        const bf16x8 v = *(const bf16x8*)((const __bf16*)x + (long)t * ld + c0);
#pragma unroll
        for (int e = 0; e < CPT; ++e) acc[e] += bf2f(v[e]);
      }
    }
  }
#pragma unroll
  for (int e = 0; e < CPT; ++e) part[rg][cg * CPT + e] = acc[e];
  __syncthreads();
  for (int col = threadIdx.x; col < 32 * CPT; col += 256) {
    float s = 0.f;
#pragma unroll
    for (int r = 0; r < 8; ++r) s += part[r][col];
    const int n = blockIdx.x * 32 * CPT + col;
    if (n < N) atomicAdd(out + n, s);
  }
}

// Many column sums in one launch (the bias gradients of a whole backward pass, batched by the op backend):
// descriptors by value (capturable, no device table); block b serves descriptor r with cum[r] <= b < cum[r + 1],
// as column block (b - cum[r]) % gx of row block (b - cum[r]) / gx.  Same per-block math as colsum_vec_kernel.
struct ColsumDesc {
  const void* x;
  float* out;
  long ld;
  int T, N, f32, R, gx, pad;
};
#define CS_MAX 32
struct ColsumBatch {
  ColsumDesc d[CS_MAX];
  int cum[CS_MAX + 1];
  int n;
};

template <bool F32>
__device__ __forceinline__ void colsum_block(const ColsumDesc& dsc, int bx, int by, float (*part)[256]) {
  constexpr int CPT = F32 ? 4 : 8;
  const int cg = threadIdx.x & 31, rg = threadIdx.x >> 5;
  const int c0 = (bx * 32 + cg) * CPT;
  const int t0 = by * dsc.R;
  const int t1 = min(dsc.T, t0 + dsc.R);
  float acc[CPT];
#pragma unroll
  for (int e = 0; e < CPT; ++e) acc[e] = 0.f;
  if (c0 < dsc.N) {
#pragma unroll 4
    for (int t = t0 + rg; t < t1; t += 8) {
      if (F32) {
        const float4 v = *(const float4*)((const float*)dsc.x + (long)t * dsc.ld + c0);
        acc[0] += v.x; acc[1] += v.y; acc[2] += v.z; acc[3] += v.w;
      } else {
        const bf16x8 v = *(const bf16x8*)((const __bf16*)dsc.x + (long)t * dsc.ld + c0);
#pragma unroll
        for (int e = 0; e < CPT; ++e) acc[e] += bf2f(v[e]);
      }
    }
  }
#pragma unroll
  for (int e = 0; e < CPT; ++e) part[rg][cg * CPT + e] = acc[e];
  __syncthreads();
  for (int col = threadIdx.x; col < 32 * CPT; col += 256) {
    float sum = 0.f;
#pragma unroll
    for (int r = 0; r < 8; ++r) sum += part[r][col];
    const int n = bx * 32 * CPT + col;
    if (n < dsc.N) atomicAdd(dsc.out + n, sum);
  }
}

__global__ __launch_bounds__(256) void colsum_multi_kernel(const ColsumBatch cb) {
  __shared__ float part[8][256];
  const int b = blockIdx.x;
  int r = 0;
  while (r + 1 < cb.n && cb.cum[r + 1] <= b) ++r;
  const ColsumDesc& dsc = cb.d[r];
  const int local = b - cb.cum[r];
  if (dsc.f32) colsum_block<true>(dsc, local % dsc.gx, local / dsc.gx, part);
  else colsum_block<false>(dsc, local % dsc.gx, local / dsc.gx, part);
}

// descriptors: host arrays (x, out pointers; ld; T; N; f32 flag), all vector-aligned (checked by the caller)
IIT_EXPORT int iit_colsum_multi(const long* xs, const long* outs, const long* lds, const int* Ts, const int* Ns,
                                const int* f32s, int n, void* stream) {
  for (int i0 = 0; i0 < n; i0 += CS_MAX) {
    ColsumBatch cb;
    cb.n = min(CS_MAX, n - i0);
    cb.cum[0] = 0;
    for (int r = 0; r < cb.n; ++r) {
      ColsumDesc& d = cb.d[r];
      const int i = i0 + r;
      d.x = (const void*)xs[i];
      d.out = (float*)outs[i];
      d.ld = lds[i];
      d.T = Ts[i];
      d.N = Ns[i];
      d.f32 = f32s[i];
      d.R = 128;
      d.gx = (d.N + 32 * (d.f32 ? 4 : 8) - 1) / (32 * (d.f32 ? 4 : 8));
      d.pad = 0;
      cb.cum[r + 1] = cb.cum[r] + d.gx * ((d.T + d.R - 1) / d.R);
    }
    if (cb.cum[cb.n] > 0)
      hipLaunchKernelGGL(colsum_multi_kernel, dim3(cb.cum[cb.n]), dim3(256), 0, (hipStream_t)stream, cb);
  }
  return hipGetLastError();
}

IIT_EXPORT int iit_colsum_accum(const void* x, int f32, long ld, float* out, int T, int N, void* stream) {
  const int cpt = f32 ? 4 : 8;
  const bool vec = (N % cpt == 0) && (ld % cpt == 0) && ((((uintptr_t)x) & 15) == 0);
  if (vec) {
    const int gx = (N + 32 * cpt - 1) / (32 * cpt);
    // rows per block: aim for >= ~1024 blocks (4 per CU) without dropping below 32 rows per block
    int R = 256;
    while (R > 32 && (long)gx * ((T + R - 1) / R) < 1024) R >>= 1;
    dim3 grid(gx, (T + R - 1) / R);
    if (f32) hipLaunchKernelGGL(colsum_vec_kernel<true>, grid, dim3(256), 0, (hipStream_t)stream, x, ld, out, T, N, R);
    else hipLaunchKernelGGL(colsum_vec_kernel<false>, grid, dim3(256), 0, (hipStream_t)stream, x, ld, out, T, N, R);
    return hipGetLastError();
  }
  dim3 grid((N + 63) / 64, (T + 63) / 64);
  if (f32) hipLaunchKernelGGL(colsum_kernel<true>, grid, dim3(256), 0, (hipStream_t)stream, x, ld, out, T, N);
  else hipLaunchKernelGGL(colsum_kernel<false>, grid, dim3(256), 0, (hipStream_t)stream, x, ld, out, T, N);
  return hipGetLastError();
}

// out = gelu_new(pre)  (bf16 -> bf16, strided rows; 8 elements / 16 B per thread when aligned)
__device__ __forceinline__ float gelu_new_fast(float x) {
  // tanh(u) = 1 - 2 / (exp(2u) + 1): one exp + one fast reciprocal instead of libm tanhf
  const float u = 0.7978845608028654f * (x + 0.044715f * x * x * x);
  const float t = 1.f - 2.f * __builtin_amdgcn_rcpf(__expf(2.f * u) + 1.f);
  return 0.5f * x * (1.f + t);
}

template <bool ERF>
__global__ __launch_bounds__(256) void gelu_fwd_kernel(const __bf16* __restrict__ pre, long ldp, __bf16* __restrict__ out,
                                                       long ldo, int M, int N) {
  const int n8 = N >> 3;
  const long total = (long)M * n8;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    const int m = (int)(i / n8), c = (int)(i % n8) * 8;
    const bf16x8 x = *(const bf16x8*)(pre + m * ldp + c);
    bf16x8 o;
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = f2bf(ERF ? gelu_erf_f(bf2f(x[e])) : gelu_new_fast(bf2f(x[e])));
    *(bf16x8*)(out + m * ldo + c) = o;
  }
}

template <bool ERF>
__global__ void gelu_fwd_scalar_kernel(const __bf16* __restrict__ pre, long ldp, __bf16* __restrict__ out, long ldo,
                                       int M, int N) {
  const long total = (long)M * N;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    const int m = (int)(i / N), n = (int)(i % N);
    const float x = bf2f(pre[m * ldp + n]);
    out[m * ldo + n] = f2bf(ERF ? gelu_erf_f(x) : gelu_new_fast(x));
  }
}

IIT_EXPORT int iit_gelu_fwd(const void* pre, long ldp, void* out, long ldo, int M, int N, int erf, void* stream) {
  const bool vec = N % 8 == 0 && ldp % 8 == 0 && ldo % 8 == 0 && ((((uintptr_t)pre) | ((uintptr_t)out)) & 15) == 0;
  const long work = vec ? (long)M * (N / 8) : (long)M * N;
  const int blocks = (int)min((work + 255) / 256, 8192L);
  hipStream_t st = (hipStream_t)stream;
  const __bf16* pp = (const __bf16*)pre;
  __bf16* oo = (__bf16*)out;
  if (vec) {
    if (erf) hipLaunchKernelGGL(gelu_fwd_kernel<true>, dim3(blocks), dim3(256), 0, st, pp, ldp, oo, ldo, M, N);
    else hipLaunchKernelGGL(gelu_fwd_kernel<false>, dim3(blocks), dim3(256), 0, st, pp, ldp, oo, ldo, M, N);
  } else {
    if (erf) hipLaunchKernelGGL(gelu_fwd_scalar_kernel<true>, dim3(blocks), dim3(256), 0, st, pp, ldp, oo, ldo, M, N);
    else hipLaunchKernelGGL(gelu_fwd_scalar_kernel<false>, dim3(blocks), dim3(256), 0, st, pp, ldp, oo, ldo, M, N);
  }
  return hipGetLastError();
}

// dpre = dpost * gelu'(pre)   (bf16, contiguous; 8 elements / 16 B per thread when n % 8 == 0); gelu_new or erf
template <bool ERF>
__device__ __forceinline__ float dgelu_of(float x) { return ERF ? gelu_erf_grad_f(x) : gelu_new_grad_f(x); }

template <bool ERF>
__global__ void dgelu_kernel(const __bf16* __restrict__ dpost, const __bf16* __restrict__ pre, __bf16* __restrict__ out, long n) {
  if ((n & 7) == 0) {
    const long n8 = n >> 3;
    for (long i = blockIdx.x * 256L + threadIdx.x; i < n8; i += (long)gridDim.x * 256) {
      const bf16x8 g = ((const bf16x8*)dpost)[i], x = ((const bf16x8*)pre)[i];
      bf16x8 o;
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = f2bf(bf2f(g[e]) * dgelu_of<ERF>(bf2f(x[e])));
      ((bf16x8*)out)[i] = o;
    }
    return;
  }
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256)
    out[i] = f2bf(bf2f(dpost[i]) * dgelu_of<ERF>(bf2f(pre[i])));
}

IIT_EXPORT int iit_dgelu(const void* dpost, const void* pre, void* out, long n, int erf, void* stream) {
  const long work = (n & 7) == 0 ? n / 8 : n;
  const int blocks = (int)min((work + 255) / 256, 8192L);
  if (erf)
    hipLaunchKernelGGL(dgelu_kernel<true>, dim3(blocks), dim3(256), 0, (hipStream_t)stream, (const __bf16*)dpost,
                       (const __bf16*)pre, (__bf16*)out, n);
  else
    hipLaunchKernelGGL(dgelu_kernel<false>, dim3(blocks), dim3(256), 0, (hipStream_t)stream, (const __bf16*)dpost,
                       (const __bf16*)pre, (__bf16*)out, n);
  return hipGetLastError();
}

// out[m][n] = base[m][n] + y[m][n] + bias[n]  (fp32 out/base, bf16 y; base may alias out, bias nullable).
// Completes a library GEMM that wrote bf16 into the fp32 residual / gradient accumulate epilogues.
template <bool VEC>
__global__ __launch_bounds__(256) void add_bf16_kernel(float* __restrict__ out, long ldo, const float* base, long ldb,
                                                       const __bf16* __restrict__ y, long ldy,
                                                       const float* __restrict__ bias, int M, int N) {
  if (VEC) {
    const int n8 = N >> 3;
    const long total = (long)M * n8;
    for (long i = blockIdx.x * 256L + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
      const int m = (int)(i / n8), c = (int)(i % n8) * 8;
      const bf16x8 v = *(const bf16x8*)(y + m * ldy + c);
      const float4 b0 = *(const float4*)(base + m * ldb + c), b1 = *(const float4*)(base + m * ldb + c + 4);
      float4 o0 = make_float4(b0.x + bf2f(v[0]), b0.y + bf2f(v[1]), b0.z + bf2f(v[2]), b0.w + bf2f(v[3]));
      float4 o1 = make_float4(b1.x + bf2f(v[4]), b1.y + bf2f(v[5]), b1.z + bf2f(v[6]), b1.w + bf2f(v[7]));
      if (bias) {
        const float4 c0 = *(const float4*)(bias + c), c1 = *(const float4*)(bias + c + 4);
        o0.x += c0.x; o0.y += c0.y; o0.z += c0.z; o0.w += c0.w;
        o1.x += c1.x; o1.y += c1.y; o1.z += c1.z; o1.w += c1.w;
      }
      *(float4*)(out + m * ldo + c) = o0;
      *(float4*)(out + m * ldo + c + 4) = o1;
    }
    return;
  }
  const long total = (long)M * N;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    const int m = (int)(i / N), n = (int)(i % N);
    out[m * ldo + n] = base[m * ldb + n] + bf2f(y[m * ldy + n]) + (bias ? bias[n] : 0.f);
  }
}

IIT_EXPORT int iit_add_bf16(float* out, long ldo, const float* base, long ldb, const void* y, long ldy,
                            const float* bias, int M, int N, void* stream) {
  const bool vec = (N % 8 == 0) && (ldo % 4 == 0) && (ldb % 4 == 0) && (ldy % 8 == 0) &&
                   ((((uintptr_t)out) | ((uintptr_t)base)) & 15) == 0 && (((uintptr_t)y) & 15) == 0 &&
                   (!bias || (((uintptr_t)bias) & 15) == 0);
  const long work = vec ? (long)M * (N / 8) : (long)M * N;
  const int blocks = (int)min((work + 255) / 256, 8192L);
  if (vec)
    hipLaunchKernelGGL(add_bf16_kernel<true>, dim3(blocks), dim3(256), 0, (hipStream_t)stream, out, ldo, base, ldb,
                       (const __bf16*)y, ldy, bias, M, N);
  else
    hipLaunchKernelGGL(add_bf16_kernel<false>, dim3(blocks), dim3(256), 0, (hipStream_t)stream, out, ldo, base, ldb,
                       (const __bf16*)y, ldy, bias, M, N);
  return hipGetLastError();
}

IIT_EXPORT int iit_device_sync() { return hipDeviceSynchronize(); }

// ---------------------------------------------------------------------------- diagnostics
// probe of ds_read_b64_tr_b16 lane semantics: LDS holds [4 rows][16 cols] of value row*16+col,
// lane 4q+p (within each 16-lane group) addresses row q, columns 4p..4p+3.
__global__ void probe_tr16_kernel(short* out) {
  __shared__ __attribute__((aligned(16))) short lds[64];
  const int l = threadIdx.x;
  lds[l] = (short)l;
  __syncthreads();
  const int li = l & 15, q = li >> 2, p = li & 3;
  typedef __attribute__((address_space(3))) i16x4 lds_i16x4;
  i16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_i16x4*)(lds + q * 16 + 4 * p));
  for (int e = 0; e < 4; ++e) out[l * 4 + e] = v[e];
}

IIT_EXPORT int iit_probe_tr16(void* out, void* stream) {
  hipLaunchKernelGGL(probe_tr16_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, (short*)out);
  return hipGetLastError();
}

// probe 2: LDS [16 rows][16 cols], lane l addresses row 4*(l>>4) + ((l&15)>>2), columns 4*(l&3)
__global__ void probe_tr16b_kernel(short* out) {
  __shared__ __attribute__((aligned(16))) short lds[256];
  const int l = threadIdx.x;
  for (int i = l; i < 256; i += 64) lds[i] = (short)i;
  __syncthreads();
  const int row = 4 * (l >> 4) + ((l & 15) >> 2), col = 4 * (l & 3);
  typedef __attribute__((address_space(3))) i16x4 lds_i16x4;
  i16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_i16x4*)(lds + row * 16 + col));
  for (int e = 0; e < 4; ++e) out[l * 4 + e] = v[e];
}

IIT_EXPORT int iit_probe_tr16b(void* out, void* stream) {
  hipLaunchKernelGGL(probe_tr16b_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, (short*)out);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------- multi-span memset
// Zero many disjoint ranges of one fp32 buffer in a single launch (the flat arena's lazy zero_grad: every
// gradient slot no store-producer owns).  chunks[i] = (start, len) in elements, len <= 65536; one block each.
__global__ __launch_bounds__(256) void zero_chunks_kernel(float* __restrict__ base, const long* __restrict__ chunks) {
  const long start = chunks[2 * blockIdx.x], len = chunks[2 * blockIdx.x + 1];
  float* p = base + start;
  const long head = min(len, (long)((4 - (((uintptr_t)p >> 2) & 3)) & 3));  // scalar stores up to 16-B alignment
  for (long i = threadIdx.x; i < head; i += 256) p[i] = 0.f;
  float4* q = (float4*)(p + head);
  const long n4 = (len - head) >> 2;
  for (long i = threadIdx.x; i < n4; i += 256) q[i] = make_float4(0.f, 0.f, 0.f, 0.f);
  for (long i = head + (n4 << 2) + threadIdx.x; i < len; i += 256) p[i] = 0.f;
}

// Zero up to 64 element ranges of ``base`` in one launch with the ranges passed BY VALUE (kernel arguments are
// copied at launch, and at graph capture): unlike a device range table no host->device copy is needed, so a zero
// plan first built inside a HIP-graph capture is one node instead of a fill per range.  Block b zeroes chunk
// b - cum[r] (ZR_CHUNK floats) of the range r with cum[r] <= b < cum[r + 1].
#define ZR_MAX 128  // 2.6 KB of kernel arguments (limit 4 KB): the GPT-2 arena's ~150-190 ranges in two launches, not three
#define ZR_CHUNK 16384
struct ZeroRanges {
  long start[ZR_MAX];
  long len[ZR_MAX];
  int cum[ZR_MAX + 1];
  int n;
};

__global__ __launch_bounds__(256) void zero_ranges_kernel(float* __restrict__ base, const ZeroRanges zr) {
  const int b = blockIdx.x;
  int r = 0;
  while (r + 1 < zr.n && zr.cum[r + 1] <= b) ++r;
  const long off = (long)(b - zr.cum[r]) * ZR_CHUNK;
  const long len = min((long)ZR_CHUNK, zr.len[r] - off);
  float* p = base + zr.start[r] + off;
  const long head = min(len, (long)((4 - (((uintptr_t)p >> 2) & 3)) & 3));
  for (long i = threadIdx.x; i < head; i += 256) p[i] = 0.f;
  float4* q = (float4*)(p + head);
  const long n4 = (len - head) >> 2;
  for (long i = threadIdx.x; i < n4; i += 256) q[i] = make_float4(0.f, 0.f, 0.f, 0.f);
  for (long i = head + (n4 << 2) + threadIdx.x; i < len; i += 256) p[i] = 0.f;
}

IIT_EXPORT int iit_zero_ranges(float* base, const long* starts, const long* lens, int n, void* stream) {
  for (int i0 = 0; i0 < n; i0 += ZR_MAX) {
    ZeroRanges zr;
    zr.n = min(ZR_MAX, n - i0);
    zr.cum[0] = 0;
    for (int r = 0; r < zr.n; ++r) {
      zr.start[r] = starts[i0 + r];
      zr.len[r] = lens[i0 + r];
      zr.cum[r + 1] = zr.cum[r] + (int)((lens[i0 + r] + ZR_CHUNK - 1) / ZR_CHUNK);
    }
    if (zr.cum[zr.n] > 0)
      hipLaunchKernelGGL(zero_ranges_kernel, dim3(zr.cum[zr.n]), dim3(256), 0, (hipStream_t)stream, base, zr);
  }
  return hipGetLastError();
}

IIT_EXPORT int iit_zero_chunks(float* base, const long* chunks, int n_chunks, void* stream) {
  if (n_chunks <= 0) return 0;
  hipLaunchKernelGGL(zero_chunks_kernel, dim3(n_chunks), dim3(256), 0, (hipStream_t)stream, base, chunks);
  return hipGetLastError();
}

// ------------------------------------------------------------------------------------------------ sweep KL rows
// Evaluation sweeps (iit_amd/utils/eval_metrics.py kl_rows): per row r of the LL output a [R][V] (fp32, row stride
// lda) and the HL target pmf b [R][V] (row stride ldb), ONE pass over both computes
//   out[r] = {sum_v a, logsumexp_v a, sum_v b a, sum_v b log a (terms with b = 0 skipped)}
// -- everything KL(b || a) needs for either reading of a (logits: softmax; already a pmf: used as is), in place of
// the reference's softmax / log / kl_div / sum chain (~10 passes over [R][V] per node).  One workgroup per row; the
// logsumexp is the online (running max) form.
__global__ __launch_bounds__(256) void kl_rows_kernel(const float* __restrict__ a, long lda, const float* __restrict__ b,
                                                      long ldb, int V, float* __restrict__ out) {
  const int r = blockIdx.x;
  const float* ar = a + (long)r * lda;
  const float* br = b + (long)r * ldb;
  float s = 0.f, m = -INFINITY, e = 0.f, dba = 0.f, dbl = 0.f;
  for (int v = threadIdx.x; v < V; v += 256) {
    const float x = ar[v], p = br[v];
    s += x;
    // a -inf logit (masked) adds nothing to the logsumexp: skipped, so it never meets m = -inf (exp(NaN))
    if (x > m) {
      e = e * __expf(m - x) + 1.f;
      m = x;
    } else if (x != -INFINITY) {
      e += __expf(x - m);
    }
    if (p != 0.f) {  // terms with b = 0 contribute 0 (also when a = -inf: no 0 * -inf)
      dba += p * x;
      dbl += p * __logf(x);
    }
  }
  __shared__ float red[5][4];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  // combine (m, e) pairs across the wave, then across waves
  const float mw = wave_max(m);
  e = m == -INFINITY ? 0.f : e * __expf(m - mw);
  e = wave_sum(e);
  s = wave_sum(s);
  dba = wave_sum(dba);
  dbl = wave_sum(dbl);
  if (lane == 0) {
    red[0][w] = s; red[1][w] = mw; red[2][w] = e; red[3][w] = dba; red[4][w] = dbl;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float M = red[1][0];
    for (int i = 1; i < 4; ++i) M = fmaxf(M, red[1][i]);
    float E = 0.f, S = 0.f, DBA = 0.f, DBL = 0.f;
    for (int i = 0; i < 4; ++i) {
      S += red[0][i];
      E += red[1][i] == -INFINITY ? 0.f : red[2][i] * __expf(red[1][i] - M);
      DBA += red[3][i];
      DBL += red[4][i];
    }
    out[4 * r + 0] = S;
    out[4 * r + 1] = M + __logf(E);
    out[4 * r + 2] = DBA;
    out[4 * r + 3] = DBL;
  }
}

IIT_EXPORT int iit_kl_rows(const float* a, long lda, const float* b, long ldb, int R, int V, float* out, void* stream) {
  if (R <= 0 || V <= 0) return 0;
  hipLaunchKernelGGL(kl_rows_kernel, dim3(R), dim3(256), 0, (hipStream_t)stream, a, lda, b, ldb, V, out);
  return hipGetLastError();
}
