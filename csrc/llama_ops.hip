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

// ------------------------------------------------------------------------------------------------ SwiGLU
__device__ __forceinline__ float silu_f(float g) { return g * __builtin_amdgcn_rcpf(1.f + __expf(-g)); }

__global__ __launch_bounds__(256) void swiglu_fwd_kernel(const __bf16* __restrict__ gate, const __bf16* __restrict__ up,
                                                         __bf16* __restrict__ post, long n8) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n8) return;
  float g[8], u[8], o[8];
  ld8(gate + i * 8, false, g);
  ld8(up + i * 8, false, u);
#pragma unroll
  for (int e = 0; e < 8; ++e) o[e] = silu_f(g[e]) * u[e];
  st8(post + i * 8, false, o);
}

__global__ __launch_bounds__(256) void swiglu_bwd_kernel(const __bf16* __restrict__ dpost, const __bf16* __restrict__ gate,
                                                         const __bf16* __restrict__ up, __bf16* __restrict__ dgate,
                                                         __bf16* __restrict__ dup, long n8) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n8) return;
  float dp[8], g[8], u[8], dg[8], du[8];
  ld8(dpost + i * 8, false, dp);
  ld8(gate + i * 8, false, g);
  ld8(up + i * 8, false, u);
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const float sg = __builtin_amdgcn_rcpf(1.f + __expf(-g[e]));
    du[e] = dp[e] * g[e] * sg;
    dg[e] = dp[e] * u[e] * sg * (1.f + g[e] * (1.f - sg));
  }
  st8(dgate + i * 8, false, dg);
  st8(dup + i * 8, false, du);
}

bool al16(const void* p) { return (((uintptr_t)p) & 15) == 0; }

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
    dim3 g2((d + 63) / 64, (T + 63) / 64);
    hipLaunchKernelGGL(rms_dw_kernel, g2, block, 0, s, (const __bf16*)dy, x, x_f32, rstd, dw, T, d);
  }
  return (int)hipGetLastError();
}

IIT_EXPORT int iit_rotary(const void* x, long sb, long ss, long sh, void* out, const float* cosT, const float* sinT,
                          int inverse, int B, int S, int H, int D, int rd, int offset, int adjacent, void* stream) {
  if (rd % 2 || rd > D) return (int)hipErrorInvalidValue;
  const long work = (long)B * S * H * (rd / 2 + (D - rd));
  hipLaunchKernelGGL(rotary_kernel, dim3((work + 255) / 256), dim3(256), 0, (hipStream_t)stream, (const __bf16*)x,
                     sb, ss, sh, (__bf16*)out, cosT, sinT, inverse ? -1.f : 1.f, B, S, H, D, rd, offset, adjacent);
  return (int)hipGetLastError();
}

IIT_EXPORT int iit_swiglu_fwd(const void* gate, const void* up, void* post, long n, void* stream) {
  if (n % 8 || !al16(gate) || !al16(up) || !al16(post)) return (int)hipErrorInvalidValue;
  const long n8 = n / 8;
  hipLaunchKernelGGL(swiglu_fwd_kernel, dim3((n8 + 255) / 256), dim3(256), 0, (hipStream_t)stream,
                     (const __bf16*)gate, (const __bf16*)up, (__bf16*)post, n8);
  return (int)hipGetLastError();
}

IIT_EXPORT int iit_swiglu_bwd(const void* dpost, const void* gate, const void* up, void* dgate, void* dup, long n,
                              void* stream) {
  if (n % 8 || !al16(dpost) || !al16(gate) || !al16(up) || !al16(dgate) || !al16(dup)) return (int)hipErrorInvalidValue;
  const long n8 = n / 8;
  hipLaunchKernelGGL(swiglu_bwd_kernel, dim3((n8 + 255) / 256), dim3(256), 0, (hipStream_t)stream,
                     (const __bf16*)dpost, (const __bf16*)gate, (const __bf16*)up, (__bf16*)dgate, (__bf16*)dup, n8);
  return (int)hipGetLastError();
}
