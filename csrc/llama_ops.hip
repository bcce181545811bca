// Fused elementwise kernels of the Llama family (RMSNorm, rotary position embedding, SwiGLU) for the GPU torch
// op backend: each replaces a chain of 3-8 PyTorch elementwise launches (and their [T, d] round trips) with one
// pass.  bf16 activations, fp32 statistics, fp32 parameter gradients accumulated straight into the flat arena.
//
//   RMSNorm   y = x * rsqrt(mean(x^2) + eps) * w        one wave per row, 16-B vector loads, rstd saved
//             dx = r (g - xhat mean(g xhat)),  g = dy w, xhat = x r;   dw += sum_t dy xhat  (block partials)
//   rotary    x' = x cos + rot(x) sin on the first rotary_dim features (GPT-NeoX halves or adjacent pairs);
//             the backward is the same kernel with sin negated (the rotation is orthogonal)
//   SwiGLU    post = silu(gate) * up;  dgate = dpost up silu'(gate), dup = dpost silu(gate)
#include "common.h"
#include "splice_spec.h"

namespace {

__device__ __forceinline__ void ld8(const void* p, bool f32, float* v) {
  if (f32) {
    const float4 a = ((const float4*)p)[0], b = ((const float4*)p)[1];
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
  } else {
    const bf16x8 t = *(const bf16x8*)p;
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = bf2f(t[e]);
  }
}

__device__ __forceinline__ void st8(void* p, bool f32, const float* v) {
  if (f32) {
    ((float4*)p)[0] = make_float4(v[0], v[1], v[2], v[3]);
    ((float4*)p)[1] = make_float4(v[4], v[5], v[6], v[7]);
  } else {
    bf16x8 o;
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = f2bf(v[e]);
    *(bf16x8*)p = o;
  }
}

// ------------------------------------------------------------------------------------------------ RMSNorm
template <int VB>
__global__ __launch_bounds__(256) void rms_fwd_kernel(const void* __restrict__ x, int x_f32, const float* __restrict__ w,
                                                      __bf16* __restrict__ y, float* __restrict__ rstd_out, int T,
                                                      int d, float eps) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (row >= T) return;
  const int es = x_f32 ? 4 : 2;
  const char* xr = (const char*)x + (long)row * d * es;
  float v[VB][8];
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < VB; ++i) {
    const int c = lane * 8 + i * 512;
    if (c < d) {
      ld8(xr + (long)c * es, x_f32, v[i]);
#pragma unroll
      for (int e = 0; e < 8; ++e) ss += v[i][e] * v[i][e];
    }
  }
  const float r = rsqrtf(wave_sum(ss) / d + eps);
#pragma unroll
  for (int i = 0; i < VB; ++i) {
    const int c = lane * 8 + i * 512;
    if (c < d) {
      float o[8];
      if (w) {
        float ww[8];
        ld8(w + c, true, ww);
#pragma unroll
        for (int e = 0; e < 8; ++e) o[e] = v[i][e] * r * ww[e];
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) o[e] = v[i][e] * r;
      }
      st8(y + (long)row * d + c, false, o);
    }
  }
  if (lane == 0) rstd_out[row] = r;
}

template <int VB>
__global__ __launch_bounds__(256) void rms_bwd_kernel(const __bf16* __restrict__ dy, const void* __restrict__ x, int x_f32,
                                                      const float* __restrict__ rstd, const float* __restrict__ w,
                                                      void* __restrict__ dx, const void* __restrict__ dres, int T,
                                                      int d) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (row >= T) return;
  const int es = x_f32 ? 4 : 2;
  const char* xr = (const char*)x + (long)row * d * es;
  const float r = rstd[row];
  float g[VB][8], xh[VB][8];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < VB; ++i) {
    const int c = lane * 8 + i * 512;
    if (c < d) {
      ld8(dy + (long)row * d + c, false, g[i]);
      ld8(xr + (long)c * es, x_f32, xh[i]);
      float ww[8] = {1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f};
      if (w) ld8(w + c, true, ww);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        g[i][e] *= ww[e];
        xh[i][e] *= r;
        s += g[i][e] * xh[i][e];
      }
    }
  }
  s = wave_sum(s) / d;
  char* dxr = (char*)dx + (long)row * d * es;
#pragma unroll
  for (int i = 0; i < VB; ++i) {
    const int c = lane * 8 + i * 512;
    if (c < d) {
      float o[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = r * (g[i][e] - xh[i][e] * s);
      if (dres) {  // the residual stream's skip-connection gradient (x's dtype), summed here instead of by autograd
        float rr[8];
        ld8((const char*)dres + ((long)row * d + c) * es, x_f32, rr);
#pragma unroll
        for (int e = 0; e < 8; ++e) o[e] += rr[e];
      }
      st8(dxr + (long)c * es, x_f32, o);
    }
  }
}

// dw[c] += sum_t dy[t][c] * x[t][c] * rstd[t]: block = 64 columns x 64 rows (4 waves x 16), one atomic per column
// per block (short token counts -- Llama IIT batches are a few hundred tokens -- still give >= 256 blocks)
__global__ __launch_bounds__(256) void rms_dw_kernel(const __bf16* __restrict__ dy, const void* __restrict__ x, int x_f32,
                                                     const float* __restrict__ rstd, float* __restrict__ dw, int T,
                                                     int d) {
  __shared__ float part[4][64];
  const int c = blockIdx.x * 64 + (threadIdx.x & 63), wv = threadIdx.x >> 6;
  const int t0 = blockIdx.y * 64;
  float acc = 0.f;
  if (c < d)
    for (int i = 0; i < 16; ++i) {
      const int t = t0 + wv * 16 + i;
      if (t >= T) break;
      const float xv = x_f32 ? ((const float*)x)[(long)t * d + c] : bf2f(((const __bf16*)x)[(long)t * d + c]);
      acc += bf2f(dy[(long)t * d + c]) * xv * rstd[t];
    }
  part[wv][threadIdx.x & 63] = acc;
  __syncthreads();
  if (wv == 0 && c < d) {
    const int l = threadIdx.x;
    atomicAdd(dw + c, part[0][l] + part[1][l] + part[2][l] + part[3][l]);
  }
}

// Vectorised dw: thread = 8 consecutive columns (16-B loads of dy and x) x 8 rows; block = 32 column chunks (256
// columns) x 8 row groups = 64 rows; the 8 row groups meet in LDS and each column takes one atomic per block.  The
// scalar kernel above moves 2 B per load (~2.4 TB/s on [8192][4096]); d % 8 == 0 is required (as for the row kernels).
__global__ __launch_bounds__(256) void rms_dw_vec_kernel(const __bf16* __restrict__ dy, const void* __restrict__ x,
                                                         int x_f32, const float* __restrict__ rstd,
                                                         float* __restrict__ dw, int T, int d) {
  __shared__ float part[8][257];
  const int cc = threadIdx.x & 31, rg = threadIdx.x >> 5;
  const int c = blockIdx.x * 256 + cc * 8;
  const int t0 = blockIdx.y * 64 + rg * 8;
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (c < d) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int t = t0 + i;
      if (t < T) {
        float g[8], xv[8];
        ld8(dy + (long)t * d + c, false, g);
        ld8((const char*)x + ((long)t * d + c) * (x_f32 ? 4 : 2), x_f32, xv);
        const float r = rstd[t];
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[e] += g[e] * xv[e] * r;
      }
    }
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) part[rg][cc * 8 + e] = acc[e];
  __syncthreads();
  const int col = blockIdx.x * 256 + threadIdx.x;
  if (col < d) {
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < 8; ++k) s += part[k][threadIdx.x];
    atomicAdd(dw + col, s);
  }
}

// ------------------------------------------------------------------------------------------------ rotary
// x [B, S, H, D] with element strides (sb, ss, sh), unit stride on D; out contiguous [B, S, H, D].  cos/sin
// [n_ctx, rd] fp32 (TL tables: angle repeated per pair layout).  One thread per (row, pair).
__global__ __launch_bounds__(256) void rotary_kernel(const __bf16* __restrict__ x, long sb, long ss, long sh,
                                                     __bf16* __restrict__ out, const float* __restrict__ cosT,
                                                     const float* __restrict__ sinT, float sin_sign, int B, int S,
                                                     int H, int D, int rd, int offset, int adjacent) {
  const long rows = (long)B * S * H;
  const int half = rd / 2, npair = half + (D - rd);  // rotated pairs, then pass-through features
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= rows * npair) return;
  const long row = idx / npair;
  const int j = idx % npair;
  const int h = row % H, s = (row / H) % S, b = row / ((long)H * S);
  const __bf16* xr = x + b * sb + (long)s * ss + (long)h * sh;
  __bf16* orow = out + row * D;
  if (j >= half) {  // features past rotary_dim pass through
    const int e = rd + (j - half);
    orow[e] = xr[e];
    return;
  }
  const int i0 = adjacent ? 2 * j : j, i1 = adjacent ? 2 * j + 1 : j + half;
  const float* ct = cosT + (long)(offset + s) * rd;
  const float* st = sinT + (long)(offset + s) * rd;
  const float a = bf2f(xr[i0]), bb = bf2f(xr[i1]);
  // rot(x)[i0] = -x[i1], rot(x)[i1] = x[i0]
  orow[i0] = f2bf(a * ct[i0] - bb * st[i0] * sin_sign);
  orow[i1] = f2bf(bb * ct[i1] + a * st[i1] * sin_sign);
}

// Vectorised form: one thread per 8 consecutive features (one 16-B load of x, plus the 16-B partner chunk half a
// rotary span away for GPT-NeoX halves); every access of a row is a full 16-B chunk.  Needs D % 8 == 0, the rotary
// span a multiple of 16 (halves) or 8 (adjacent pairs) and 16-B aligned rows -- the Llama shapes (D = rd = 128);
// anything else takes the per-pair kernel above.  Work per row: rd/16 (halves; each thread rotates its chunk and
// the partner chunk) or rd/8 (adjacent) rotating threads, then (D - rd)/8 pass-through threads.
__global__ __launch_bounds__(256) void rotary_vec_kernel(const __bf16* __restrict__ x, long sb, long ss, long sh,
                                                         __bf16* __restrict__ out, const float* __restrict__ cosT,
                                                         const float* __restrict__ sinT, float sin_sign, int B, int S,
                                                         int H, int D, int rd, int offset, int adjacent) {
  const int rot = adjacent ? rd / 8 : rd / 16, per_row = rot + (D - rd) / 8;
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long rows = (long)B * S * H;
  if (idx >= rows * per_row) return;
  const long row = idx / per_row;
  const int j = idx % per_row;
  const int h = row % H, s = (row / H) % S, b = row / ((long)H * S);
  const __bf16* xr = x + b * sb + (long)s * ss + (long)h * sh;
  __bf16* orow = out + row * D;
  if (j >= rot) {  // pass-through chunk
    const int c = rd + (j - rot) * 8;
    *(bf16x8*)(orow + c) = *(const bf16x8*)(xr + c);
    return;
  }
  const float* ct = cosT + (long)(offset + s) * rd;
  const float* st = sinT + (long)(offset + s) * rd;
  if (adjacent) {  // pairs (2i, 2i+1) inside the chunk: rot(x)[2i] = -x[2i+1], rot(x)[2i+1] = x[2i]
    const int c = j * 8;
    float v[8], cs[8], sn[8], o[8];
    ld8(xr + c, false, v);
    ld8(ct + c, true, cs);
    ld8(st + c, true, sn);
#pragma unroll
    for (int e = 0; e < 8; e += 2) {
      o[e] = v[e] * cs[e] - v[e + 1] * sn[e] * sin_sign;
      o[e + 1] = v[e + 1] * cs[e + 1] + v[e] * sn[e + 1] * sin_sign;
    }
    st8(orow + c, false, o);
  } else {  // halves: element c + e pairs with c + half + e
    const int half = rd / 2, c0 = j * 8, c1 = c0 + half;
    float a[8], bb[8], c0s[8], c0n[8], c1s[8], c1n[8], o0[8], o1[8];
    ld8(xr + c0, false, a);
    ld8(xr + c1, false, bb);
    ld8(ct + c0, true, c0s);
    ld8(st + c0, true, c0n);
    ld8(ct + c1, true, c1s);
    ld8(st + c1, true, c1n);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      o0[e] = a[e] * c0s[e] - bb[e] * c0n[e] * sin_sign;
      o1[e] = bb[e] * c1s[e] + a[e] * c1n[e] * sin_sign;
    }
    st8(orow + c0, false, o0);
    st8(orow + c1, false, o1);
  }
}

// ------------------------------------------------------------------------------------------------ SwiGLU
__device__ __forceinline__ float silu_f(float g) { return g * __builtin_amdgcn_rcpf(1.f + __expf(-g)); }

// SW_U 16-B chunks per thread, all loads issued before any math (more bytes in flight per wave: the one-chunk form
// measured ~3 TB/s on the Llama MLP shapes); chunk u of block b is b * 256 * SW_U + u * 256 + tid (coalesced per u)
constexpr int SW_U = 4;

__global__ __launch_bounds__(256) void swiglu_fwd_kernel(const __bf16* __restrict__ gate, const __bf16* __restrict__ up,
                                                         __bf16* __restrict__ post, long n8) {
  const long base = (long)blockIdx.x * 256 * SW_U + threadIdx.x;
  bf16x8 g[SW_U], u[SW_U];
#pragma unroll
  for (int k = 0; k < SW_U; ++k) {
    const long i = base + k * 256;
    if (i < n8) {
      g[k] = __builtin_nontemporal_load((const bf16x8*)gate + i);
      u[k] = __builtin_nontemporal_load((const bf16x8*)up + i);
    }
  }
#pragma unroll
  for (int k = 0; k < SW_U; ++k) {
    const long i = base + k * 256;
    if (i < n8) {
      bf16x8 o;
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = f2bf(silu_f(bf2f(g[k][e])) * bf2f(u[k][e]));
      *((bf16x8*)post + i) = o;
    }
  }
}

__global__ __launch_bounds__(256) void swiglu_bwd_kernel(const __bf16* __restrict__ dpost, const __bf16* __restrict__ gate,
                                                         const __bf16* __restrict__ up, __bf16* __restrict__ dgate,
                                                         __bf16* __restrict__ dup, long n8) {
  const long base = (long)blockIdx.x * 256 * SW_U + threadIdx.x;
  bf16x8 dp[SW_U], g[SW_U], u[SW_U];
#pragma unroll
  for (int k = 0; k < SW_U; ++k) {
    const long i = base + k * 256;
    if (i < n8) {
      dp[k] = __builtin_nontemporal_load((const bf16x8*)dpost + i);
      g[k] = __builtin_nontemporal_load((const bf16x8*)gate + i);
      u[k] = __builtin_nontemporal_load((const bf16x8*)up + i);
    }
  }
#pragma unroll
  for (int k = 0; k < SW_U; ++k) {
    const long i = base + k * 256;
    if (i < n8) {
      bf16x8 dg, du;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float gv = bf2f(g[k][e]), dv = bf2f(dp[k][e]);
        const float sg = __builtin_amdgcn_rcpf(1.f + __expf(-gv));
        du[e] = f2bf(dv * gv * sg);
        dg[e] = f2bf(dv * bf2f(u[k][e]) * sg * (1.f + gv * (1.f - sg)));
      }
      *((bf16x8*)dgate + i) = dg;
      *((bf16x8*)dup + i) = du;
    }
  }
}

// SwiGLU with an interchange splice of its output (``mlp.hook_post``) applied in the producer: the elements the patch
// spec selects take the source's value instead of silu(gate) * up, and their gate / up gradients are zero (the spliced
// value is a constant) -- the reference's hook ``out[idx] = src[idx]`` (base_model_pair.py:151-163) without the
// separate read + write pass of the standalone splice kernel and its gradient mask.  One thread per 8 consecutive
// features (the spec's innermost dimension a multiple of 8).
__global__ __launch_bounds__(256) void swiglu_splice_fwd_kernel(const __bf16* __restrict__ gate,
                                                                const __bf16* __restrict__ up,
                                                                __bf16* __restrict__ post,
                                                                const __bf16* __restrict__ src, long n8,
                                                                SpliceSpec sp) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= n8) return;
  int c0, c1, c2, c3;
  spec_coords(sp, i * 8, c0, c1, c2, c3);
  const bool row = in_ranges(sp, 0, c0) && in_ranges(sp, 1, c1) && in_ranges(sp, 2, c2);
  const bf16x8 g = *((const bf16x8*)gate + i), u = *((const bf16x8*)up + i);
  bf16x8 o;
#pragma unroll
  for (int e = 0; e < 8; ++e) o[e] = f2bf(silu_f(bf2f(g[e])) * bf2f(u[e]));
  if (row) {
    const long sb = (long)c0 * sp.sstride[0] + (long)c1 * sp.sstride[1] + (long)c2 * sp.sstride[2];
#pragma unroll
    for (int e = 0; e < 8; ++e)
      if (in_ranges(sp, 3, c3 + e)) o[e] = src[sb + (long)(c3 + e) * sp.sstride[3]];
  }
  *((bf16x8*)post + i) = o;
}

__global__ __launch_bounds__(256) void swiglu_splice_bwd_kernel(const __bf16* __restrict__ dpost,
                                                                const __bf16* __restrict__ gate,
                                                                const __bf16* __restrict__ up,
                                                                __bf16* __restrict__ dgate, __bf16* __restrict__ dup,
                                                                long n8, SpliceSpec sp) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= n8) return;
  int c0, c1, c2, c3;
  spec_coords(sp, i * 8, c0, c1, c2, c3);
  const bool row = in_ranges(sp, 0, c0) && in_ranges(sp, 1, c1) && in_ranges(sp, 2, c2);
  const bf16x8 dp = *((const bf16x8*)dpost + i), g = *((const bf16x8*)gate + i), u = *((const bf16x8*)up + i);
  bf16x8 dg, du;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const float gv = bf2f(g[e]);
    const float dv = (row && in_ranges(sp, 3, c3 + e)) ? 0.f : bf2f(dp[e]);
    const float sg = __builtin_amdgcn_rcpf(1.f + __expf(-gv));
    du[e] = f2bf(dv * gv * sg);
    dg[e] = f2bf(dv * bf2f(u[e]) * sg * (1.f + gv * (1.f - sg)));
  }
  *((bf16x8*)dgate + i) = dg;
  *((bf16x8*)dup + i) = du;
}

// Token embedding gather with an interchange splice of its output (``hook_embed``) applied in the producer: out[t, :] =
// W[tokens[t], :] (bf16 mirror rows, row stride ``ld``) except the elements the patch spec selects, which take the
// source's value -- W_E[tokens] followed by ``out[idx] = src[idx]`` (base_model_pair.py:151-163) in one pass.  One
// thread per 8 consecutive features (d a multiple of 8).
__global__ __launch_bounds__(256) void embed_splice_fwd_kernel(const long* __restrict__ tokens,
                                                               const __bf16* __restrict__ W, long ld,
                                                               __bf16* __restrict__ out,
                                                               const __bf16* __restrict__ src, long n8, int d,
                                                               SpliceSpec sp) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= n8) return;
  const long t = i * 8 / d;
  const int c = (int)(i * 8 - t * d);
  bf16x8 o = *(const bf16x8*)(W + tokens[t] * ld + c);
  int c0, c1, c2, c3;
  spec_coords(sp, i * 8, c0, c1, c2, c3);
  if (in_ranges(sp, 0, c0) && in_ranges(sp, 1, c1) && in_ranges(sp, 2, c2)) {
    const long sb = (long)c0 * sp.sstride[0] + (long)c1 * sp.sstride[1] + (long)c2 * sp.sstride[2];
#pragma unroll
    for (int e = 0; e < 8; ++e)
      if (in_ranges(sp, 3, c3 + e)) o[e] = src[sb + (long)(c3 + e) * sp.sstride[3]];
  }
  *((bf16x8*)out + i) = o;
}

// The embedding gradient of the spliced gather: grad[tokens[t], :] += dout[t, :] (fp32 grad rows, memory-side fp32
// atomics as torch's index_add), skipping the spliced elements (a constant from the source run: no gradient).
template <typename G>
__global__ __launch_bounds__(256) void embed_splice_bwd_kernel(const long* __restrict__ tokens,
                                                               const G* __restrict__ dout,
                                                               float* __restrict__ grad, long ldg, long n8, int d,
                                                               SpliceSpec sp) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= n8) return;
  const long t = i * 8 / d;
  const int c = (int)(i * 8 - t * d);
  int c0, c1, c2, c3;
  spec_coords(sp, i * 8, c0, c1, c2, c3);
  const bool row = in_ranges(sp, 0, c0) && in_ranges(sp, 1, c1) && in_ranges(sp, 2, c2);
  float* g = grad + tokens[t] * ldg + c;
  const G* dp = dout + i * 8;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    if (row && in_ranges(sp, 3, c3 + e)) continue;
    atomicAdd(g + e, (float)dp[e]);
  }
}

bool al16(const void* p) { return (((uintptr_t)p) & 15) == 0; }

// IIT_LLAMA_VEC=0 selects the scalar rotary / RMSNorm-dw kernels (A/B and fallback), read once per process
bool llama_vec_on() {
  static const bool on = [] {
    const char* e = getenv("IIT_LLAMA_VEC");
    return !(e && e[0] == '0');
  }();
  return on;
}

}  // namespace

IIT_EXPORT int iit_rms_fwd(const void* x, int x_f32, const float* w, void* y, float* rstd, int T, int d, float eps,
                           void* stream) {
  if (d % 8 || d > 8192 || !al16(x) || !al16(y) || (w && !al16(w))) return (int)hipErrorInvalidValue;
  dim3 grid((T + 3) / 4), block(256);
  hipStream_t s = (hipStream_t)stream;
  const int vb = (d + 511) / 512;
#define RF(V) hipLaunchKernelGGL(rms_fwd_kernel<V>, grid, block, 0, s, x, x_f32, w, (__bf16*)y, rstd, T, d, eps)
  if (vb <= 1) RF(1); else if (vb <= 2) RF(2); else if (vb <= 4) RF(4); else if (vb <= 8) RF(8); else RF(16);
#undef RF
  return (int)hipGetLastError();
}

IIT_EXPORT int iit_rms_bwd_res(const void* dy, const void* x, int x_f32, const float* rstd, const float* w, void* dx,
                               const void* dres, float* dw, int T, int d, void* stream);

// dx has x's dtype; dw (nullable) accumulates in fp32
IIT_EXPORT int iit_rms_bwd(const void* dy, const void* x, int x_f32, const float* rstd, const float* w, void* dx,
                           float* dw, int T, int d, void* stream) {
  return iit_rms_bwd_res(dy, x, x_f32, rstd, w, dx, nullptr, dw, T, d, stream);
}

// ``dres`` (nullable, x's dtype): added to dx -- the fork form (RMSNorm output + residual passthrough) of the
// pre-norm block, one pass instead of the norm backward plus autograd's gradient sum over [T, d]
IIT_EXPORT int iit_rms_bwd_res(const void* dy, const void* x, int x_f32, const float* rstd, const float* w, void* dx,
                               const void* dres, float* dw, int T, int d, void* stream) {
  if (d % 8 || d > 8192 || !al16(x) || !al16(dy) || !al16(dx) || (w && !al16(w)) || (dres && !al16(dres)))
    return (int)hipErrorInvalidValue;
  dim3 grid((T + 3) / 4), block(256);
  hipStream_t s = (hipStream_t)stream;
  const int vb = (d + 511) / 512;
#define RB(V) hipLaunchKernelGGL(rms_bwd_kernel<V>, grid, block, 0, s, (const __bf16*)dy, x, x_f32, rstd, w, dx, dres, T, d)
  if (vb <= 1) RB(1); else if (vb <= 2) RB(2); else if (vb <= 4) RB(4); else if (vb <= 8) RB(8); else RB(16);
#undef RB
  if (dw) {
    if (llama_vec_on()) {
      dim3 g2((d + 255) / 256, (T + 63) / 64);
      hipLaunchKernelGGL(rms_dw_vec_kernel, g2, block, 0, s, (const __bf16*)dy, x, x_f32, rstd, dw, T, d);
    } else {
      dim3 g2((d + 63) / 64, (T + 63) / 64);
      hipLaunchKernelGGL(rms_dw_kernel, g2, block, 0, s, (const __bf16*)dy, x, x_f32, rstd, dw, T, d);
    }
  }
  return (int)hipGetLastError();
}

IIT_EXPORT int iit_rotary(const void* x, long sb, long ss, long sh, void* out, const float* cosT, const float* sinT,
                          int inverse, int B, int S, int H, int D, int rd, int offset, int adjacent, void* stream) {
  if (rd % 2 || rd > D) return (int)hipErrorInvalidValue;
  const bool vec = llama_vec_on() && D % 8 == 0 && (adjacent ? rd % 8 == 0 : rd % 16 == 0) && sb % 8 == 0 &&
                   ss % 8 == 0 && sh % 8 == 0 && al16(x) && al16(out);
  if (vec) {
    const long work = (long)B * S * H * ((adjacent ? rd / 8 : rd / 16) + (D - rd) / 8);
    hipLaunchKernelGGL(rotary_vec_kernel, dim3((work + 255) / 256), dim3(256), 0, (hipStream_t)stream,
                       (const __bf16*)x, sb, ss, sh, (__bf16*)out, cosT, sinT, inverse ? -1.f : 1.f, B, S, H, D, rd,
                       offset, adjacent);
    return (int)hipGetLastError();
  }
  const long work = (long)B * S * H * (rd / 2 + (D - rd));
  hipLaunchKernelGGL(rotary_kernel, dim3((work + 255) / 256), dim3(256), 0, (hipStream_t)stream, (const __bf16*)x,
                     sb, ss, sh, (__bf16*)out, cosT, sinT, inverse ? -1.f : 1.f, B, S, H, D, rd, offset, adjacent);
  return (int)hipGetLastError();
}

IIT_EXPORT int iit_swiglu_fwd(const void* gate, const void* up, void* post, long n, void* stream) {
  if (n % 8 || !al16(gate) || !al16(up) || !al16(post)) return (int)hipErrorInvalidValue;
  const long n8 = n / 8;
  hipLaunchKernelGGL(swiglu_fwd_kernel, dim3((n8 + 256 * SW_U - 1) / (256 * SW_U)), dim3(256), 0, (hipStream_t)stream,
                     (const __bf16*)gate, (const __bf16*)up, (__bf16*)post, n8);
  return (int)hipGetLastError();
}

IIT_EXPORT int iit_swiglu_bwd(const void* dpost, const void* gate, const void* up, void* dgate, void* dup, long n,
                              void* stream) {
  if (n % 8 || !al16(dpost) || !al16(gate) || !al16(up) || !al16(dgate) || !al16(dup)) return (int)hipErrorInvalidValue;
  const long n8 = n / 8;
  hipLaunchKernelGGL(swiglu_bwd_kernel, dim3((n8 + 256 * SW_U - 1) / (256 * SW_U)), dim3(256), 0, (hipStream_t)stream,
                     (const __bf16*)dpost, (const __bf16*)gate, (const __bf16*)up, (__bf16*)dgate, (__bf16*)dup, n8);
  return (int)hipGetLastError();
}

// ``spec``: host pointer to one SpliceSpec over the [.., d_mlp] activation (innermost dimension a multiple of 8)
IIT_EXPORT int iit_swiglu_splice_fwd(const void* gate, const void* up, void* post, const void* src, long n,
                                     const void* spec, void* stream) {
  const SpliceSpec sp = *(const SpliceSpec*)spec;
  if (n % 8 || sp.shape[3] % 8 || !al16(gate) || !al16(up) || !al16(post)) return (int)hipErrorInvalidValue;
  const long n8 = n / 8;
  hipLaunchKernelGGL(swiglu_splice_fwd_kernel, dim3((n8 + 255) / 256), dim3(256), 0, (hipStream_t)stream,
                     (const __bf16*)gate, (const __bf16*)up, (__bf16*)post, (const __bf16*)src, n8, sp);
  return (int)hipGetLastError();
}

IIT_EXPORT int iit_swiglu_splice_bwd(const void* dpost, const void* gate, const void* up, void* dgate, void* dup,
                                     long n, const void* spec, void* stream) {
  const SpliceSpec sp = *(const SpliceSpec*)spec;
  if (n % 8 || sp.shape[3] % 8 || !al16(dpost) || !al16(gate) || !al16(up) || !al16(dgate) || !al16(dup))
    return (int)hipErrorInvalidValue;
  const long n8 = n / 8;
  hipLaunchKernelGGL(swiglu_splice_bwd_kernel, dim3((n8 + 255) / 256), dim3(256), 0, (hipStream_t)stream,
                     (const __bf16*)dpost, (const __bf16*)gate, (const __bf16*)up, (__bf16*)dgate, (__bf16*)dup, n8,
                     sp);
  return (int)hipGetLastError();
}

// ``tokens`` int64 [T]; ``W`` the bf16 mirror of W_E (row stride ``ld``); ``out`` / ``src`` bf16 over the spec's shape
// (T * d elements; the spec's innermost dimension a multiple of 8, so 8 consecutive features share its outer coordinates)
IIT_EXPORT int iit_embed_splice_fwd(const void* tokens, const void* W, long ld, void* out, const void* src, long T,
                                    int d, const void* spec, void* stream) {
  const SpliceSpec sp = *(const SpliceSpec*)spec;
  if (d % 8 || ld % 8 || sp.shape[3] % 8 || !al16(W) || !al16(out)) return (int)hipErrorInvalidValue;
  const long n8 = T * d / 8;
  hipLaunchKernelGGL(embed_splice_fwd_kernel, dim3((n8 + 255) / 256), dim3(256), 0, (hipStream_t)stream,
                     (const long*)tokens, (const __bf16*)W, ld, (__bf16*)out, (const __bf16*)src, n8, d, sp);
  return (int)hipGetLastError();
}

// ``dout`` bf16 (dout_f32 = 0) or fp32 [T, d]; ``grad`` fp32 rows of stride ``ldg``
IIT_EXPORT int iit_embed_splice_bwd(const void* tokens, const void* dout, int dout_f32, float* grad, long ldg, long T,
                                    int d, const void* spec, void* stream) {
  const SpliceSpec sp = *(const SpliceSpec*)spec;
  if (d % 8 || sp.shape[3] % 8) return (int)hipErrorInvalidValue;
  const long n8 = T * d / 8;
  if (dout_f32)
    hipLaunchKernelGGL(embed_splice_bwd_kernel<float>, dim3((n8 + 255) / 256), dim3(256), 0, (hipStream_t)stream,
                       (const long*)tokens, (const float*)dout, grad, ldg, n8, d, sp);
  else
    hipLaunchKernelGGL(embed_splice_bwd_kernel<__bf16>, dim3((n8 + 255) / 256), dim3(256), 0, (hipStream_t)stream,
                       (const long*)tokens, (const __bf16*)dout, grad, ldg, n8, d, sp);
  return (int)hipGetLastError();
}
