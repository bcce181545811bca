// Fused BatchNorm (+ residual add) (+ ReLU) for NHWC (channels-last) bf16 or fp32 activations -- the PVR ResNet-18's
// normalisation, forward and backward, in place of MIOpenBatchNormFwdTrainSpatial / MIOpenBatchNormBwdSpatial plus
// the separate ReLU, residual-add and running-statistics kernels (profiles/bench_family_pvr_resnet18_r4.txt: 5.0 ms
// of norm and ~3 ms of elementwise per bf16 step).
//
// Layout: x [M][C] (M = N * H * W rows, C channels contiguous, C % 8 == 0); one thread owns 8 consecutive channels
// of a row (one 16-B load / store), a wave covers 64 / (C / 8) rows at once.
//
// Forward (training): a stats pass over row chunks -- every workgroup owns a contiguous chunk of rows, sums x - p and
// (x - p)^2 per channel in fp32 around a per-chunk pivot p (the chunk's first row: |mean - p| is O(std), so the
// variance does not cancel the way E[x^2] - mean^2 does when |mean| >> std) and stores its chunk's (mean, M2) with plain
// stores -- no atomics, no ticket, no serial last-workgroup tail.  The apply pass then combines the R chunk partials
// of its channels in a fixed order with Chan's parallel update (deterministic, identical in every workgroup), writes
// y = relu(x * scale + shift (+ res)) and, in workgroup 0, mean / rstd for the backward, the running mean / unbiased
// variance with the momentum and num_batches_tracked (torch.nn.BatchNorm2d's buffer semantics).  Eval mode: the apply
// pass alone, from the running statistics.
//
// Backward: dz = dy * (y > 0) (the ReLU mask from the saved output); a stats pass stores per-chunk partial sums of dz
// and dz * xhat; the apply pass combines them (fixed order), writes dx = w rstd (dz - sum(dz) / M - xhat
// sum(dz xhat) / M) (training; eval: w rstd dz) and the residual's gradient dz, and workgroup 0 ADDS the weight / bias
// gradients sum(dz xhat) / sum(dz) into the parameters' gradient buffers (no autograd accumulation launch).
//
// The kernel boundary between the two passes is the only synchronisation: the partials are written by one launch and
// read by the next (round 6: the round-5 fp32 memory-side atomics on 8 slots per channel + a ticketed last workgroup
// cost 10-17 us per call on 0.5-3 us of HBM traffic, profiles/pvr_step_r5.txt).
#include "common.h"
#include "splice_spec.h"
#include <stdlib.h>

namespace {

constexpr int TPB = 256;
// partial bytes the apply pass combines per workgroup: R chunks x 2C floats <= RC_MAX x 2 floats
constexpr int RC_MAX = 8192;
constexpr int C_MAX = 2048;  // C / 8 <= TPB

// Interchange splice of the BN input (the preceding conv's hook, ``hook_point`` of mode-"q" PVR sites): the
// activation the kernels read is x' = where(spec, src, x), spec over the logical [N][C][H][W] with src's element
// strides; the backward zeroes the spliced elements' input gradient (SpliceFn's semantics).  ``hw`` = H * W, ``W``.
struct XSplice {
  const void* src;  // the activation's dtype (bf16 or fp32)
  int hw, W;
  SpliceSpec sp;
};

// row (n, h, w) of a spliced x: whether the row is inside the spec's batch / spatial ranges, and the source row base
__device__ __forceinline__ bool xs_row(const XSplice& xs, long row, long& sbase) {
  const int n = (int)(row / xs.hw), r = (int)(row - (long)n * xs.hw), h = r / xs.W, w = r - h * xs.W;
  sbase = n * xs.sp.sstride[0] + h * xs.sp.sstride[2] + w * xs.sp.sstride[3];
  return in_ranges(xs.sp, 0, n) && in_ranges(xs.sp, 2, h) && in_ranges(xs.sp, 3, w);
}

struct Row8 {
  float v[8];
};

__device__ __forceinline__ Row8 load8(const __bf16* p) {
  const bf16x8 t = *(const bf16x8*)p;
  Row8 r;
#pragma unroll
  for (int e = 0; e < 8; ++e) r.v[e] = bf2f(t[e]);
  return r;
}

__device__ __forceinline__ Row8 load8(const float* p) {  // fp32 activations (the reference-precision PVR step)
  const float4 a = ((const float4*)p)[0], b = ((const float4*)p)[1];
  Row8 r;
  r.v[0] = a.x; r.v[1] = a.y; r.v[2] = a.z; r.v[3] = a.w;
  r.v[4] = b.x; r.v[5] = b.y; r.v[6] = b.z; r.v[7] = b.w;
  return r;
}

// x' row segment [c0, c0 + 8) of row ``row`` (the spliced input when xs.src is set); ``hit`` = which of the 8
// elements came from the source (their input gradient is zero)
template <bool SP, typename T>
__device__ __forceinline__ Row8 load_x(const T* x, long row, int C, int c0, const XSplice& xs, unsigned& hit) {
  Row8 v = load8(x + row * C + c0);
  hit = 0u;
  if (SP) {
    long sb;
    if (xs_row(xs, row, sb)) {
#pragma unroll
      for (int e = 0; e < 8; ++e)
        if (in_ranges(xs.sp, 1, c0 + e)) {
          v.v[e] = (float)((const T*)xs.src)[sb + (long)(c0 + e) * xs.sp.sstride[1]];
          hit |= 1u << e;
        }
    }
  }
  return v;
}

__device__ __forceinline__ void store8(__bf16* p, const Row8& r) {
  bf16x8 t;
#pragma unroll
  for (int e = 0; e < 8; ++e) t[e] = f2bf(r.v[e]);
  *(bf16x8*)p = t;
}

__device__ __forceinline__ void store8(float* p, const Row8& r) {
  ((float4*)p)[0] = make_float4(r.v[0], r.v[1], r.v[2], r.v[3]);
  ((float4*)p)[1] = make_float4(r.v[4], r.v[5], r.v[6], r.v[7]);
}

// per-channel totals of this workgroup's per-thread [8] pairs (a, b) (threads sharing a channel group, rows r < rpi):
// thread c (c < C, strided) gets (sum a, sum b) of channel c; ``red`` is TPB * 16 floats of LDS
__device__ __forceinline__ void block_channel_sums(const float* a, const float* b, int C, int G, int rpi, int tid,
                                                   float* red) {
  const int g = tid % G, r = tid / G;
  if (r < rpi) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      red[(r * G + g) * 16 + e] = a[e];
      red[(r * G + g) * 16 + 8 + e] = b[e];
    }
  }
  __syncthreads();
}

__device__ __forceinline__ void channel_total(const float* red, int c, int G, int rpi, float& sa, float& sb) {
  const int gg = c / 8, e = c % 8;
  float x = 0.f, y = 0.f;
  for (int rr = 0; rr < rpi; ++rr) {
    x += red[(rr * G + gg) * 16 + e];
    y += red[(rr * G + gg) * 16 + 8 + e];
  }
  sa = x;
  sb = y;
}

// rows of chunk w of R chunks of ``chunk`` rows over M rows
__device__ __forceinline__ long chunk_rows(int w, long chunk, long M) {
  const long r0 = (long)w * chunk;
  const long r1 = r0 + chunk < M ? r0 + chunk : M;
  return r1 - r0;
}

// part[w][0, C) = mean, part[w][C, 2C) = M2 of chunk w = blockIdx.x (rows [w chunk, (w + 1) chunk))
template <bool SP, typename T>
__global__ __launch_bounds__(TPB) void bn_stats_kernel(const T* __restrict__ x, long M, int C, long chunk,
                                                       float* __restrict__ part, XSplice xs) {
  __shared__ float red[TPB * 16];
  __shared__ float piv[C_MAX];
  const int G = C / 8, rpi = TPB / G, tid = threadIdx.x;
  const int g = tid % G, r = tid / G;
  const long r0 = (long)blockIdx.x * chunk;
  const long r1 = r0 + chunk < M ? r0 + chunk : M;
  float s[8], q[8], p[8];
  {
    unsigned hit;
    const Row8 pv = load_x<SP>(x, r0, C, g * 8, xs, hit);  // the pivot: this chunk's first row (x' when spliced)
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      p[e] = pv.v[e];
      s[e] = q[e] = 0.f;
    }
    if (r == 0) {
#pragma unroll
      for (int e = 0; e < 8; ++e) piv[g * 8 + e] = p[e];
    }
  }
  if (r < rpi) {
#pragma unroll 4  // several rows' loads in flight per thread (the loop is latency-bound)
    for (long row = r0 + r; row < r1; row += rpi) {
      unsigned hit;
      const Row8 v = load_x<SP>(x, row, C, g * 8, xs, hit);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float d = v.v[e] - p[e];
        s[e] += d;
        q[e] = __builtin_fmaf(d, d, q[e]);
      }
    }
  }
  block_channel_sums(s, q, C, G, rpi, tid, red);
  const float n = (float)(r1 - r0);
  float* dst = part + (long)blockIdx.x * 2 * C;
  for (int c = tid; c < C; c += TPB) {
    float S, Q;
    channel_total(red, c, G, rpi, S, Q);
    dst[c] = piv[c] + S / n;                  // chunk mean
    dst[C + c] = fmaxf(Q - S * (S / n), 0.f);  // chunk M2 = sum (x - mean)^2
  }
}

// mean[c], var[c] (biased) of all M rows from the R chunk partials, combined in chunk order (Chan et al.'s pairwise
// update); TPC threads per channel each fold a contiguous range of chunks, then their results are folded in order
__device__ __forceinline__ void combine_stats(const float* __restrict__ part, int R, long chunk, long M, int C,
                                              float* mean_out, float* var_out, float* lds3 /* [3][TPB] */) {
  const int tid = threadIdx.x;
  const int TPC = C >= TPB ? 1 : TPB / C;  // threads per channel (C divides TPB or TPB divides C)
  const int per = (R + TPC - 1) / TPC;
  for (int base = 0; base < C; base += TPB / TPC) {
    const int c = base + tid / TPC, j = tid % TPC;
    float na = 0.f, ma = 0.f, m2a = 0.f;
    if (c < C) {
      const int w0 = j * per, w1 = min(R, w0 + per);
      for (int w = w0; w < w1; ++w) {
        const float nb = (float)chunk_rows(w, chunk, M);
        const float mb = part[(long)w * 2 * C + c], m2b = part[(long)w * 2 * C + C + c];
        const float nn = na + nb;
        const float d = mb - ma;
        ma += d * (nb / nn);
        m2a += m2b + d * d * (na * nb / nn);
        na = nn;
      }
    }
    lds3[tid] = na;
    lds3[TPB + tid] = ma;
    lds3[2 * TPB + tid] = m2a;
    __syncthreads();
    if (c < C && j == 0) {
      for (int k = 1; k < TPC; ++k) {
        const float nb = lds3[tid + k], mb = lds3[TPB + tid + k], m2b = lds3[2 * TPB + tid + k];
        if (nb == 0.f) continue;
        const float nn = na + nb;
        const float d = mb - ma;
        ma += d * (nb / nn);
        m2a += m2b + d * d * (na * nb / nn);
        na = nn;
      }
      mean_out[c] = ma;
      var_out[c] = m2a / (float)M;
    }
    __syncthreads();
  }
}

// (sum a, sum b)[c] over the R chunk partials, in chunk order (TPC threads per channel, then folded in order)
__device__ __forceinline__ void combine_sums(const float* __restrict__ part, int R, int C, float* a_out, float* b_out,
                                             float* lds2 /* [2][TPB] */) {
  const int tid = threadIdx.x;
  const int TPC = C >= TPB ? 1 : TPB / C;
  const int per = (R + TPC - 1) / TPC;
  for (int base = 0; base < C; base += TPB / TPC) {
    const int c = base + tid / TPC, j = tid % TPC;
    float sa = 0.f, sb = 0.f;
    if (c < C) {
      const int w0 = j * per, w1 = min(R, w0 + per);
      for (int w = w0; w < w1; ++w) {
        sa += part[(long)w * 2 * C + c];
        sb += part[(long)w * 2 * C + C + c];
      }
    }
    lds2[tid] = sa;
    lds2[TPB + tid] = sb;
    __syncthreads();
    if (c < C && j == 0) {
      for (int k = 1; k < TPC; ++k) {
        sa += lds2[tid + k];
        sb += lds2[TPB + tid + k];
      }
      a_out[c] = sa;
      b_out[c] = sb;
    }
    __syncthreads();
  }
}

// y = relu?(x * scale + shift (+ res)); training: the statistics from the R chunk partials (workgroup 0 also writes
// save = (mean, rstd), the running statistics and num_batches_tracked); eval: from the running statistics, and
// workgroup 0 writes them to ``save`` for the backward
template <bool SP, typename T>
__global__ __launch_bounds__(TPB) void bn_apply_kernel(const T* __restrict__ x, const T* __restrict__ res,
                                                       T* __restrict__ y, float* __restrict__ save,
                                                       float* __restrict__ rmean, float* __restrict__ rvar,
                                                       const float* __restrict__ w, const float* __restrict__ b, long M,
                                                       int C, float eps, int relu, int batch, const float* part, int R,
                                                       long chunk, float momentum, long long* nbt, XSplice xs) {
  __shared__ float st_mean[C_MAX], st_var[C_MAX];
  __shared__ float lds3[3 * TPB];
  const int G = C / 8, rpi = TPB / G, tid = threadIdx.x;
  const int g = tid % G, r = tid / G;
  if (batch) {
    combine_stats(part, R, chunk, M, C, st_mean, st_var, lds3);
    if (blockIdx.x == 0) {
      for (int c = tid; c < C; c += TPB) {
        const float mean = st_mean[c], var = st_var[c];
        save[c] = mean;
        save[C + c] = rsqrtf(var + eps);
        const float unb = M > 1 ? var * (float)M / (float)(M - 1) : var;
        rmean[c] = (1.f - momentum) * rmean[c] + momentum * mean;
        rvar[c] = (1.f - momentum) * rvar[c] + momentum * unb;
      }
      if (tid == 0 && nbt) nbt[0] += 1;
    }
  } else if (blockIdx.x == 0) {
    for (int c = tid; c < C; c += TPB) {
      save[c] = rmean[c];
      save[C + c] = rsqrtf(rvar[c] + eps);
    }
  }
  if (r >= rpi) return;
  float sc[8], sh[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const int c = g * 8 + e;
    const float mean = batch ? st_mean[c] : rmean[c];
    const float rstd = batch ? rsqrtf(st_var[c] + eps) : rsqrtf(rvar[c] + eps);
    sc[e] = w[c] * rstd;
    sh[e] = b[c] - mean * sc[e];
  }
#pragma unroll 4
  for (long row = (long)blockIdx.x * rpi + r; row < M; row += (long)gridDim.x * rpi) {
    unsigned hit;
    Row8 v = load_x<SP>(x, row, C, g * 8, xs, hit);
    if (res) {
      const Row8 rv = load8(res + row * C + g * 8);
#pragma unroll
      for (int e = 0; e < 8; ++e) v.v[e] = __builtin_fmaf(v.v[e], sc[e], sh[e]) + rv.v[e];
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) v.v[e] = __builtin_fmaf(v.v[e], sc[e], sh[e]);
    }
    if (relu) {
#pragma unroll
      for (int e = 0; e < 8; ++e) v.v[e] = fmaxf(v.v[e], 0.f);
    }
    store8(y + row * C + g * 8, v);
  }
}

// part[w][0, C) = sum dz, part[w][C, 2C) = sum dz * xhat over chunk w   (dz = dy masked by y > 0 when y is given)
template <bool SP, typename T>
__global__ __launch_bounds__(TPB) void bn_bwd_stats_kernel(const T* __restrict__ dy, const T* __restrict__ y,
                                                           const T* __restrict__ x, const float* __restrict__ save,
                                                           long M, int C, long chunk, float* __restrict__ part,
                                                           XSplice xs) {
  __shared__ float red[TPB * 16];
  const int G = C / 8, rpi = TPB / G, tid = threadIdx.x;
  const int g = tid % G, r = tid / G;
  const long r0 = (long)blockIdx.x * chunk;
  const long r1 = r0 + chunk < M ? r0 + chunk : M;
  float s[8], q[8], mean[8], rstd[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    s[e] = q[e] = 0.f;
    mean[e] = save[g * 8 + e];
    rstd[e] = save[C + g * 8 + e];
  }
  if (r < rpi) {
#pragma unroll 4
    for (long row = r0 + r; row < r1; row += rpi) {
      const long o = row * C + g * 8;
      Row8 d = load8(dy + o);
      unsigned hit;
      const Row8 xv = load_x<SP>(x, row, C, g * 8, xs, hit);
      if (y) {
        const Row8 yv = load8(y + o);
#pragma unroll
        for (int e = 0; e < 8; ++e) d.v[e] = yv.v[e] > 0.f ? d.v[e] : 0.f;
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        s[e] += d.v[e];
        q[e] = __builtin_fmaf(d.v[e], (xv.v[e] - mean[e]) * rstd[e], q[e]);
      }
    }
  }
  block_channel_sums(s, q, C, G, rpi, tid, red);
  float* dst = part + (long)blockIdx.x * 2 * C;
  for (int c = tid; c < C; c += TPB) {
    float S, Q;
    channel_total(red, c, G, rpi, S, Q);
    dst[c] = S;
    dst[C + c] = Q;
  }
}

template <bool SP, typename T>
__global__ __launch_bounds__(TPB) void bn_bwd_apply_kernel(const T* __restrict__ dy, const T* __restrict__ y,
                                                           const T* __restrict__ x, const float* __restrict__ save,
                                                           const float* __restrict__ w, const float* __restrict__ part,
                                                           int R, long M, int C, int batch, T* __restrict__ dx,
                                                           T* __restrict__ dres, float* coef, float* dw, float* db,
                                                           XSplice xs) {
  __shared__ float st_a[C_MAX], st_b[C_MAX];
  __shared__ float lds2[2 * TPB];
  const int G = C / 8, rpi = TPB / G, tid = threadIdx.x;
  const int g = tid % G, r = tid / G;
  if (batch || dw || db) {
    combine_sums(part, R, C, st_a, st_b, lds2);
    if (blockIdx.x == 0) {  // coef = (sum dz, sum dz xhat); parameter gradients accumulated
      for (int c = tid; c < C; c += TPB) {
        coef[c] = st_a[c];
        coef[C + c] = st_b[c];
        if (dw) dw[c] += st_b[c];
        if (db) db[c] += st_a[c];
      }
    }
  }
  if (r >= rpi) return;
  float k1[8], k2[8], k3[8], mean[8], rstd[8];
  const float inv_m = 1.f / (float)M;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const int c = g * 8 + e;
    mean[e] = save[c];
    rstd[e] = save[C + c];
    k1[e] = w[c] * rstd[e];                          // dx = k1 (dz - k2 - xhat k3)
    k2[e] = batch ? st_a[c] * inv_m : 0.f;
    k3[e] = batch ? st_b[c] * inv_m : 0.f;
  }
#pragma unroll 4
  for (long row = (long)blockIdx.x * rpi + r; row < M; row += (long)gridDim.x * rpi) {
    const long o = row * C + g * 8;
    Row8 d = load8(dy + o);
    if (y) {
      const Row8 yv = load8(y + o);
#pragma unroll
      for (int e = 0; e < 8; ++e) d.v[e] = yv.v[e] > 0.f ? d.v[e] : 0.f;
    }
    if (dres) store8(dres + o, d);
    Row8 out;
    unsigned hit = 0u;
    if (batch) {
      const Row8 xv = load_x<SP>(x, row, C, g * 8, xs, hit);
#pragma unroll
      for (int e = 0; e < 8; ++e) out.v[e] = k1[e] * (d.v[e] - k2[e] - (xv.v[e] - mean[e]) * rstd[e] * k3[e]);
    } else {
      if (SP) {
        long sb;
        if (xs_row(xs, row, sb)) {
#pragma unroll
          for (int e = 0; e < 8; ++e) hit |= (in_ranges(xs.sp, 1, g * 8 + e) ? 1u : 0u) << e;
        }
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) out.v[e] = k1[e] * d.v[e];
    }
    if (SP && hit) {  // spliced input elements: a constant, no gradient
#pragma unroll
      for (int e = 0; e < 8; ++e)
        if ((hit >> e) & 1u) out.v[e] = 0.f;
    }
    store8(dx + o, out);
  }
}

int bn_rows_per_group() {  // IIT_BN_ROWS (A/B of the grid size; default 8), read once per process
  static const int v = [] {
    const char* e = getenv("IIT_BN_ROWS");
    const int r = e ? atoi(e) : 8;
    return r >= 1 && r <= 256 ? r : 8;
  }();
  return v;
}

int grid_for(long M, int C) {
  const int rpi = TPB / (C / 8);
  const long want = (M + rpi - 1) / rpi;
  // ~8 rows per thread group: enough work per workgroup to amortise the per-channel atomics, >= 4 workgroups per CU
  const int rows = bn_rows_per_group();
  long g = (want + rows - 1) / rows;
  if (g < 1) g = 1;
  if (g > 2048) g = 2048;
  return (int)g;
}

// the stats passes' row chunks: R workgroups of ``chunk`` rows (R * C <= RC_MAX so the apply pass's fixed-order
// combine reads <= 64 KiB of partials per workgroup; >= 4 row iterations per thread group); IIT_BN_RC overrides the cap
int bn_rc_max() {
  static const int v = [] {
    const char* e = getenv("IIT_BN_RC");
    const int r = e ? atoi(e) : RC_MAX;
    return r >= 64 && r <= 65536 ? r : RC_MAX;
  }();
  return v;
}

void chunks_for(long M, int C, int& R, long& chunk) {
  const int rpi = TPB / (C / 8);
  int cap = bn_rc_max() / C;
  if (cap < 1) cap = 1;
  const long min_rows = 4L * rpi;
  long want = (M + min_rows - 1) / min_rows;
  if (want < 1) want = 1;
  R = (int)(want < cap ? want : cap);
  chunk = (M + R - 1) / R;
  R = (int)((M + chunk - 1) / chunk);  // no empty chunk
}

bool shape_ok(long M, int C, const void* p) {
  return M > 0 && C >= 8 && C % 8 == 0 && C / 8 <= TPB && (TPB % (C / 8)) == 0 && ((uintptr_t)p & 15) == 0;
}

// ---------------------------------------------------------------------------------------------------------------
// 3x3 / stride 2 / padding 1 max pooling on channels-last bf16 (the PVR ResNet's stem pool), forward storing the
// argmax tap (0..8, row-major in the window) as one byte per output element instead of torch's int64 flat index
// (8x fewer index bytes), and a gather-form backward: each input element sums the gradients of the (up to 4)
// windows that hold it and chose it -- no scatter, no atomics, no zero-fill of the input gradient.  Ties and NaN
// follow torch's kernel: the first tap in scan order wins, a NaN is taken.  One thread per 8 channels.
template <typename T>
__global__ __launch_bounds__(256) void maxpool3s2_fwd_kernel(const T* __restrict__ x, T* __restrict__ y,
                                                             unsigned char* __restrict__ idx, int N, int H, int W,
                                                             int C, int OH, int OW) {
  const int c8n = C / 8;
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  const long total = (long)N * OH * OW * c8n;
  if (i >= total) return;
  const int c8 = (int)(i % c8n);
  long r = i / c8n;
  const int ow = (int)(r % OW);
  r /= OW;
  const int oh = (int)(r % OH);
  const int n = (int)(r / OH);
  float best[8];
  unsigned char arg[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    best[e] = -INFINITY;
    arg[e] = 0;
  }
  bool first = true;
#pragma unroll
  for (int kh = 0; kh < 3; ++kh) {
    const int ih = 2 * oh - 1 + kh;
    if (ih < 0 || ih >= H) continue;
#pragma unroll
    for (int kw = 0; kw < 3; ++kw) {
      const int iw = 2 * ow - 1 + kw;
      if (iw < 0 || iw >= W) continue;
      const Row8 v = load8(x + (((long)n * H + ih) * W + iw) * C + c8 * 8);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float f = v.v[e];
        if (first || f > best[e] || f != f) {
          best[e] = f;
          arg[e] = (unsigned char)(kh * 3 + kw);
        }
      }
      first = false;
    }
  }
  Row8 o;
#pragma unroll
  for (int e = 0; e < 8; ++e) o.v[e] = best[e];
  const long oi = (((long)n * OH + oh) * OW + ow) * C + c8 * 8;
  store8(y + oi, o);
  unsigned long long packed = 0;
#pragma unroll
  for (int e = 0; e < 8; ++e) packed |= (unsigned long long)arg[e] << (8 * e);
  *(unsigned long long*)(idx + oi) = packed;
}

template <typename T>
__global__ __launch_bounds__(256) void maxpool3s2_bwd_kernel(const T* __restrict__ dy,
                                                             const unsigned char* __restrict__ idx,
                                                             T* __restrict__ dx, int N, int H, int W, int C,
                                                             int OH, int OW) {
  const int c8n = C / 8;
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  const long total = (long)N * H * W * c8n;
  if (i >= total) return;
  const int c8 = (int)(i % c8n);
  long r = i / c8n;
  const int iw = (int)(r % W);
  r /= W;
  const int ih = (int)(r % H);
  const int n = (int)(r / H);
  float acc[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) acc[e] = 0.f;
#pragma unroll
  for (int kh = 0; kh < 3; ++kh) {
    const int th = ih + 1 - kh;  // = 2 oh
    if (th < 0 || (th & 1) || (th >> 1) >= OH) continue;
    const int oh = th >> 1;
#pragma unroll
    for (int kw = 0; kw < 3; ++kw) {
      const int tw = iw + 1 - kw;
      if (tw < 0 || (tw & 1) || (tw >> 1) >= OW) continue;
      const int ow = tw >> 1;
      const long oi = (((long)n * OH + oh) * OW + ow) * C + c8 * 8;
      const unsigned long long packed = *(const unsigned long long*)(idx + oi);
      const Row8 g = load8(dy + oi);
      const unsigned tap = (unsigned)(kh * 3 + kw);
#pragma unroll
      for (int e = 0; e < 8; ++e)
        if (((packed >> (8 * e)) & 0xffull) == tap) acc[e] += g.v[e];
    }
  }
  Row8 o;
#pragma unroll
  for (int e = 0; e < 8; ++e) o.v[e] = acc[e];
  store8(dx + (((long)n * H + ih) * W + iw) * C + c8 * 8, o);
}

}  // namespace

// channels-last bf16 [N][H][W][C] -> [N][OH][OW][C] (OH = (H - 1) / 2 + 1, OW likewise), idx one byte per output
// ``f32``: fp32 activations instead of bf16
IIT_EXPORT int iit_maxpool3s2_fwd(const void* x, void* y, void* idx, int N, int H, int W, int C, int f32,
                                  void* stream) {
  const int OH = (H - 1) / 2 + 1, OW = (W - 1) / 2 + 1;
  if (C % 8 || (((uintptr_t)x) & 15) || (((uintptr_t)y) & 15) || (((uintptr_t)idx) & 7)) return (int)hipErrorInvalidValue;
  const long total = (long)N * OH * OW * (C / 8);
  if (f32)
    hipLaunchKernelGGL(maxpool3s2_fwd_kernel<float>, dim3((total + 255) / 256), dim3(256), 0, (hipStream_t)stream,
                       (const float*)x, (float*)y, (unsigned char*)idx, N, H, W, C, OH, OW);
  else
    hipLaunchKernelGGL(maxpool3s2_fwd_kernel<__bf16>, dim3((total + 255) / 256), dim3(256), 0, (hipStream_t)stream,
                       (const __bf16*)x, (__bf16*)y, (unsigned char*)idx, N, H, W, C, OH, OW);
  return (int)hipGetLastError();
}

IIT_EXPORT int iit_maxpool3s2_bwd(const void* dy, const void* idx, void* dx, int N, int H, int W, int C, int f32,
                                  void* stream) {
  const int OH = (H - 1) / 2 + 1, OW = (W - 1) / 2 + 1;
  if (C % 8 || (((uintptr_t)dy) & 15) || (((uintptr_t)dx) & 15) || (((uintptr_t)idx) & 7)) return (int)hipErrorInvalidValue;
  const long total = (long)N * H * W * (C / 8);
  if (f32)
    hipLaunchKernelGGL(maxpool3s2_bwd_kernel<float>, dim3((total + 255) / 256), dim3(256), 0, (hipStream_t)stream,
                       (const float*)dy, (const unsigned char*)idx, (float*)dx, N, H, W, C, OH, OW);
  else
    hipLaunchKernelGGL(maxpool3s2_bwd_kernel<__bf16>, dim3((total + 255) / 256), dim3(256), 0, (hipStream_t)stream,
                       (const __bf16*)dy, (const unsigned char*)idx, (__bf16*)dx, N, H, W, C, OH, OW);
  return (int)hipGetLastError();
}

// forward: ws = per-module partials buffer (iit_bn_ws_floats, fully rewritten by every call that reads it);
// y = relu?(bn(x) (+ res)); save [2C] = mean, rstd (the batch's in training, the running ones in eval)
static bool make_xsplice(XSplice& xs, const void* src, const void* spec, long M, int C, int H, int W) {
  xs = XSplice{};
  if (!src || !spec) return true;
  xs.src = src;
  xs.sp = *(const SpliceSpec*)spec;
  xs.hw = H * W;
  xs.W = W;
  return H > 0 && W > 0 && (long)xs.sp.shape[0] * H * W == M && xs.sp.shape[1] == C && xs.sp.shape[2] == H &&
         xs.sp.shape[3] == W;
}

template <typename T>
int bn_fwd_impl(const void* x, const void* res, void* y, float* ws, float* rmean, float* rvar, const float* w,
                const float* b, long M, int C, float eps, int relu, int training, float* save, float momentum,
                long long* nbt, const XSplice& xs, hipStream_t s) {
  const int grid = grid_for(M, C);
  int R = 0;
  long chunk = M;
  if (training) chunks_for(M, C, R, chunk);
  // the splice-reading instantiations only where a splice is given (the others keep the lean inner loop)
  if (xs.src) {
    if (training)
      hipLaunchKernelGGL((bn_stats_kernel<true, T>), dim3(R), dim3(TPB), 0, s, (const T*)x, M, C, chunk, ws, xs);
    hipLaunchKernelGGL((bn_apply_kernel<true, T>), dim3(grid), dim3(TPB), 0, s, (const T*)x, (const T*)res, (T*)y,
                       save, rmean, rvar, w, b, M, C, eps, relu, training, (const float*)ws, R, chunk, momentum, nbt,
                       xs);
  } else {
    if (training)
      hipLaunchKernelGGL((bn_stats_kernel<false, T>), dim3(R), dim3(TPB), 0, s, (const T*)x, M, C, chunk, ws, xs);
    hipLaunchKernelGGL((bn_apply_kernel<false, T>), dim3(grid), dim3(TPB), 0, s, (const T*)x, (const T*)res, (T*)y,
                       save, rmean, rvar, w, b, M, C, eps, relu, training, (const float*)ws, R, chunk, momentum, nbt,
                       xs);
  }
  return (int)hipGetLastError();
}

template <typename T>
int bn_bwd_impl(const void* dy, const void* y, const void* x, const float* save, const float* w, float* ws,
                float* coef, long M, int C, int training, void* dx, void* dres, float* dw, float* db,
                const XSplice& xs, hipStream_t s) {
  const int grid = grid_for(M, C);
  int R = 0;
  long chunk = M;
  const bool sums = training || dw || db;  // the eval-mode backward needs the sums only for the parameter gradients
  if (sums) chunks_for(M, C, R, chunk);
  if (xs.src) {
    if (sums)
      hipLaunchKernelGGL((bn_bwd_stats_kernel<true, T>), dim3(R), dim3(TPB), 0, s, (const T*)dy, (const T*)y,
                         (const T*)x, save, M, C, chunk, ws, xs);
    hipLaunchKernelGGL((bn_bwd_apply_kernel<true, T>), dim3(grid), dim3(TPB), 0, s, (const T*)dy, (const T*)y,
                       (const T*)x, save, w, (const float*)ws, R, M, C, training, (T*)dx, (T*)dres, coef, dw, db, xs);
  } else {
    if (sums)
      hipLaunchKernelGGL((bn_bwd_stats_kernel<false, T>), dim3(R), dim3(TPB), 0, s, (const T*)dy, (const T*)y,
                         (const T*)x, save, M, C, chunk, ws, xs);
    hipLaunchKernelGGL((bn_bwd_apply_kernel<false, T>), dim3(grid), dim3(TPB), 0, s, (const T*)dy, (const T*)y,
                       (const T*)x, save, w, (const float*)ws, R, M, C, training, (T*)dx, (T*)dres, coef, dw, db, xs);
  }
  return (int)hipGetLastError();
}

// ``f32``: the activations (x, res, y, dy, dx, dres, the splice source) are fp32 instead of bf16
IIT_EXPORT int iit_bn_fwd(const void* x, const void* res, void* y, float* ws, float* rmean, float* rvar,
                          const float* w, const float* b, long M, int C, float eps, int relu, int training,
                          float* save, float momentum, long long* nbt, const void* src, const void* spec, int H,
                          int W, int f32, void* stream) {
  if (!shape_ok(M, C, x) || ((uintptr_t)y & 15) || (res && ((uintptr_t)res & 15))) return (int)hipErrorInvalidValue;
  if (!rmean || !rvar) return (int)hipErrorInvalidValue;
  XSplice xs;
  if (!make_xsplice(xs, src, spec, M, C, H, W)) return (int)hipErrorInvalidValue;
  hipStream_t s = (hipStream_t)stream;
  return f32 ? bn_fwd_impl<float>(x, res, y, ws, rmean, rvar, w, b, M, C, eps, relu, training, save, momentum, nbt, xs, s)
             : bn_fwd_impl<__bf16>(x, res, y, ws, rmean, rvar, w, b, M, C, eps, relu, training, save, momentum, nbt, xs, s);
}

// backward: ws as in the forward; coef [2C] = (sum dz, sum dz xhat) (written when computed); dx (and dres = the residual's gradient when non-null);
// dw / db (nullable) ACCUMULATED into
IIT_EXPORT int iit_bn_bwd(const void* dy, const void* y, const void* x, const float* save, const float* w,
                          float* ws, float* coef, long M, int C, int training, void* dx, void* dres, float* dw,
                          float* db, const void* src, const void* spec, int H, int W, int f32, void* stream) {
  if (!shape_ok(M, C, dy) || ((uintptr_t)x & 15) || ((uintptr_t)dx & 15) || (y && ((uintptr_t)y & 15)) ||
      (dres && ((uintptr_t)dres & 15)))
    return (int)hipErrorInvalidValue;
  XSplice xs;
  if (!make_xsplice(xs, src, spec, M, C, H, W)) return (int)hipErrorInvalidValue;
  hipStream_t s = (hipStream_t)stream;
  return f32 ? bn_bwd_impl<float>(dy, y, x, save, w, ws, coef, M, C, training, dx, dres, dw, db, xs, s)
             : bn_bwd_impl<__bf16>(dy, y, x, save, w, ws, coef, M, C, training, dx, dres, dw, db, xs, s);
}

// floats of the per-module partials buffer ``ws`` (R chunks x 2C, R * C <= the cap; ops/bn.py allocates it)
IIT_EXPORT int iit_bn_ws_floats(int C) {
  const int cap = bn_rc_max() / C;
  return 2 * C * (cap < 1 ? 1 : cap);
}
