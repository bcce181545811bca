// Fused BatchNorm (+ residual add) (+ ReLU) for NHWC (channels-last) bf16 or fp32 activations -- the PVR ResNet-18's
// normalisation, forward and backward, in place of MIOpenBatchNormFwdTrainSpatial / MIOpenBatchNormBwdSpatial plus
// the separate ReLU, residual-add and running-statistics kernels (profiles/bench_family_pvr_resnet18_r4.txt: 5.0 ms
// of norm and ~3 ms of elementwise per bf16 step).
//
// Layout: x [M][C] (M = N * H * W rows, C channels contiguous, C % 8 == 0); one thread owns 8 consecutive channels
// of a row (one 16-B load / store), a wave covers 64 / (C / 8) rows at once.
//
// Forward (training): stats pass -- per-channel sums of x - p and (x - p)^2 in fp32 around a per-channel pivot p (the
// batch's first row: no cancellation when |mean| >> std), reduced in LDS per workgroup and
// added with one fp32 atomic per channel per workgroup into a per-module accumulator; the LAST workgroup to finish
// (a ticket) reads the totals back with atomics, writes mean / rstd for the apply pass and the backward, updates the
// running mean / unbiased variance with the momentum, increments num_batches_tracked (torch.nn.BatchNorm2d's buffer
// semantics) and re-zeroes the accumulator and the ticket for the next call (no memset launch) -- then the apply pass
// writes y = relu(x * scale + shift (+ res)) in bf16.  Eval mode: the apply pass alone, from the running statistics.
//
// Backward: dz = dy * (y > 0) (the ReLU mask from the saved bf16 output), a stats pass for sum(dz) and
// sum(dz * xhat) whose last workgroup also ADDS the weight / bias gradients sum(dz xhat) / sum(dz) into the
// parameters' gradient buffers (no autograd accumulation launch), then dx = w rstd (dz - sum(dz) / M - xhat
// sum(dz xhat) / M) (training; eval: w rstd dz) and the residual's gradient dz.
//
// Ticket protocol (MI355X_MICROARCH.md hand-off table, producer and consumer in different workgroups of one kernel):
// the fp32 adds are memory-side atomics; every thread waits vmcnt(0) for its adds before the workgroup barrier, one
// thread then takes the ticket with a relaxed agent-scope atomic, and the last workgroup reads the totals with atomic
// read-modify-writes (atomicExch to 0), which also execute at the memory side -- no L2 line of the accumulator is
// ever read with a plain load, so no acquire-side invalidate is needed either.
#include "common.h"
#include "splice_spec.h"
#include <stdlib.h>

namespace {

constexpr int TPB = 256;
// the per-channel accumulator is spread over BN_SLOTS copies (workgroup b adds into slot b % BN_SLOTS; the last
// workgroup sums them): 1/BN_SLOTS of the memory-side atomics per address -- a few thousand workgroups adding into
// the same 2C addresses serialised on them
constexpr int BN_SLOTS = 8;

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

// block reduction of per-thread [8] pairs (a, b) over the threads sharing a channel group; adds the block totals
// into acc[c] / acc[C + c] with one atomic per channel
__device__ __forceinline__ void block_channel_add(const float* a, const float* b, int C, int G, int rpi, int tid,
                                                  float* acc, float* red) {
  const int g = tid % G, r = tid / G;
  if (r < rpi) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      red[(r * G + g) * 16 + e] = a[e];
      red[(r * G + g) * 16 + 8 + e] = b[e];
    }
  }
  __syncthreads();
  for (int i = tid; i < G * 16; i += TPB) {
    const int gg = i / 16, e = i % 16;
    float s = 0.f;
    for (int rr = 0; rr < rpi; ++rr) s += red[(rr * G + gg) * 16 + e];
    const int c = gg * 8 + (e & 7);
    atomicAdd(acc + (e < 8 ? c : C + c), s);
  }
}

// block reduction as block_channel_add, but the totals are STORED (no atomics) channel-major at
// part[c * R + block] / part[(C + c) * R + block] (R = gridDim.x), for the fixed-order second level
__device__ __forceinline__ void block_channel_part(const float* a, const float* b, int C, int G, int rpi, int tid,
                                                   float* part, float* red) {
  const int g = tid % G, r = tid / G;
  if (r < rpi) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      red[(r * G + g) * 16 + e] = a[e];
      red[(r * G + g) * 16 + 8 + e] = b[e];
    }
  }
  __syncthreads();
  const long R = gridDim.x;
  for (int i = tid; i < G * 16; i += TPB) {
    const int gg = i / 16, e = i % 16;
    float s = 0.f;
    for (int rr = 0; rr < rpi; ++rr) s += red[(rr * G + gg) * 16 + e];
    const int c = gg * 8 + (e & 7);
    part[(long)(e < 8 ? c : C + c) * R + blockIdx.x] = s;
  }
}

// fixed-order sum of one channel's R partials by one wave (lane-strided, then a butterfly): bit-identical every run
__device__ __forceinline__ float wave_part_sum(const float* __restrict__ v, int R, int lane) {
  float s = 0.f;
  for (int w = lane; w < R; w += 64) s += v[w];
  return wave_sum(s);
}

// the last workgroup of a ticketed reduction: every thread waits for its memory-side atomic adds to complete
// (s_waitcnt vmcnt(0): no L2 writeback is needed, nothing here went through a cache), the workgroup barrier
// collects them, then one relaxed agent-scope ticket per workgroup -- a full __threadfence() per thread (an L2
// write-back each) made the stats pass 2.7x slower
__device__ __forceinline__ bool last_block(unsigned* ticket, int tid, int* flag) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) {
    const unsigned t = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *flag = t == gridDim.x - 1;
  }
  __syncthreads();
  return *flag;
}

// acc[0, C) += sum_rows x, acc[C, 2C) += sum_rows x^2; the last workgroup turns the totals into save = (mean, rstd),
// updates the running statistics and num_batches_tracked, and re-arms acc / ticket
template <bool SP, typename T>
__global__ __launch_bounds__(TPB) void bn_stats_kernel(const T* __restrict__ x, long M, int C, float* acc,
                                                       unsigned* ticket, float* __restrict__ save, float* rmean,
                                                       float* rvar, float eps, float momentum, long long* nbt,
                                                       XSplice xs, float* __restrict__ part) {
  __shared__ float red[TPB * 16];
  __shared__ float pivs[8 * TPB];  // the pivots, for the last workgroup's finalize (no dependent global load there)
  __shared__ int flag;
  const int G = C / 8, rpi = TPB / G, tid = threadIdx.x;
  const int g = tid % G, r = tid / G;
  float s[8], q[8];
  // sums of x - p and (x - p)^2 around a per-channel pivot p = x'[0][c] (the batch's first row, the same in every
  // workgroup): |mean - p| is O(std), so var = E[(x-p)^2] - E[x-p]^2 does not cancel the way E[x^2] - mean^2 does
  // when |mean| >> std
  unsigned hit0;
  const Row8 piv = load_x<SP>(x, 0, C, g * 8, xs, hit0);
  if (r == 0) {
#pragma unroll
    for (int e = 0; e < 8; ++e) pivs[g * 8 + e] = piv.v[e];
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) s[e] = q[e] = 0.f;
  if (r < rpi) {
#pragma unroll 4  // several rows' loads in flight per thread (the loop was latency-bound)
    for (long row = (long)blockIdx.x * rpi + r; row < M; row += (long)gridDim.x * rpi) {
      unsigned hit;
      const Row8 v = load_x<SP>(x, row, C, g * 8, xs, hit);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float d = v.v[e] - piv.v[e];
        s[e] += d;
        q[e] = __builtin_fmaf(d, d, q[e]);
      }
    }
  }
  if (part) {  // two-level reduction: this workgroup's totals, channel-major, for bn_finalize_kernel
    block_channel_part(s, q, C, G, rpi, tid, part, red);
    return;
  }
  block_channel_add(s, q, C, G, rpi, tid, acc + (blockIdx.x % BN_SLOTS) * 2 * C, red);
  if (!last_block(ticket, tid, &flag)) return;
  for (int c = tid; c < C; c += TPB) {
    float sum = 0.f, sq = 0.f;
    for (int k = 0; k < BN_SLOTS; ++k) {
      sum += atomicExch(acc + k * 2 * C + c, 0.f);
      sq += atomicExch(acc + k * 2 * C + C + c, 0.f);
    }
    const float p = pivs[c];  // the pivot of channel c (stored before block_channel_add's barrier)
    const float dm = sum / (float)M;  // mean - p
    const float mean = p + dm;
    const float var = fmaxf(sq / (float)M - dm * dm, 0.f);
    save[c] = mean;
    save[C + c] = rsqrtf(var + eps);
    if (rmean) {
      const float unb = M > 1 ? var * (float)M / (float)(M - 1) : var;
      rmean[c] = (1.f - momentum) * rmean[c] + momentum * mean;
      rvar[c] = (1.f - momentum) * rvar[c] + momentum * unb;
    }
  }
  if (tid == 0) {
    if (nbt) nbt[0] += 1;
    atomicExch(ticket, 0u);
  }
}

// second level of the two-level forward reduction: one wave per channel sums the R channel-major partials in a fixed
// order and writes save = (mean, rstd), the running statistics and (wave 0 of block 0) num_batches_tracked
template <bool SP, typename T>
__global__ __launch_bounds__(64) void bn_finalize_kernel(const T* __restrict__ x, const float* __restrict__ part,
                                                         int R, long M, int C, float* __restrict__ save, float* rmean,
                                                         float* rvar, float eps, float momentum, long long* nbt,
                                                         XSplice xs) {
  const int c = blockIdx.x, lane = threadIdx.x;
  const float sum = wave_part_sum(part + (long)c * R, R, lane);
  const float sq = wave_part_sum(part + (long)(C + c) * R, R, lane);
  if (lane != 0) return;
  unsigned hit;
  const float p = load_x<SP>(x, 0, C, (c / 8) * 8, xs, hit).v[c % 8];  // the pivot of channel c
  const float dm = sum / (float)M;
  const float mean = p + dm;
  const float var = fmaxf(sq / (float)M - dm * dm, 0.f);
  save[c] = mean;
  save[C + c] = rsqrtf(var + eps);
  if (rmean) {
    const float unb = M > 1 ? var * (float)M / (float)(M - 1) : var;
    rmean[c] = (1.f - momentum) * rmean[c] + momentum * mean;
    rvar[c] = (1.f - momentum) * rvar[c] + momentum * unb;
  }
  if (c == 0 && nbt) nbt[0] += 1;
}

// second level of the backward reduction: coef = (sum dz, sum dz xhat), the parameter gradients accumulated
__global__ __launch_bounds__(64) void bn_bwd_finalize_kernel(const float* __restrict__ part, int R, int C,
                                                             float* __restrict__ coef, float* dw, float* db) {
  const int c = blockIdx.x, lane = threadIdx.x;
  const float sdz = wave_part_sum(part + (long)c * R, R, lane);
  const float sdzx = wave_part_sum(part + (long)(C + c) * R, R, lane);
  if (lane != 0) return;
  coef[c] = sdz;
  coef[C + c] = sdzx;
  if (dw) dw[c] += sdzx;
  if (db) db[c] += sdz;
}

// y = relu?(x * scale + shift (+ res)); training: mean / rstd from ``save`` (the stats kernel); eval: from the running
// statistics, and workgroup 0 writes them to ``save`` for the backward
template <bool SP, typename T>
__global__ __launch_bounds__(TPB) void bn_apply_kernel(const T* __restrict__ x, const T* __restrict__ res,
                                                       T* __restrict__ y, float* __restrict__ save,
                                                       const float* __restrict__ rmean, const float* __restrict__ rvar,
                                                       const float* __restrict__ w, const float* __restrict__ b, long M,
                                                       int C, float eps, int relu, int batch, XSplice xs) {
  const int G = C / 8, rpi = TPB / G, tid = threadIdx.x;
  const int g = tid % G, r = tid / G;
  if (!batch && blockIdx.x == 0) {
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
    const float mean = batch ? save[c] : rmean[c];
    const float rstd = batch ? save[C + c] : rsqrtf(rvar[c] + eps);
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

// acc[0, C) += sum dz, acc[C, 2C) += sum dz * xhat   (dz = dy masked by y > 0 when y is given)
template <bool SP, typename T>
__global__ __launch_bounds__(TPB) void bn_bwd_stats_kernel(const T* __restrict__ dy, const T* __restrict__ y,
                                                           const T* __restrict__ x, const float* __restrict__ save,
                                                           long M, int C, float* acc, unsigned* ticket,
                                                           float* __restrict__ coef, float* dw, float* db, XSplice xs,
                                                           float* __restrict__ part) {
  __shared__ float red[TPB * 16];
  __shared__ int flag;
  const int G = C / 8, rpi = TPB / G, tid = threadIdx.x;
  const int g = tid % G, r = tid / G;
  float s[8], q[8], mean[8], rstd[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    s[e] = q[e] = 0.f;
    mean[e] = save[g * 8 + e];
    rstd[e] = save[C + g * 8 + e];
  }
  if (r < rpi) {
#pragma unroll 4  // several rows' loads in flight per thread (the loop was latency-bound)
    for (long row = (long)blockIdx.x * rpi + r; row < M; row += (long)gridDim.x * rpi) {
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
  if (part) {
    block_channel_part(s, q, C, G, rpi, tid, part, red);
    return;
  }
  block_channel_add(s, q, C, G, rpi, tid, acc + (blockIdx.x % BN_SLOTS) * 2 * C, red);
  if (!last_block(ticket, tid, &flag)) return;
  for (int c = tid; c < C; c += TPB) {  // coef = (sum dz, sum dz xhat); parameter gradients accumulated
    float sdz = 0.f, sdzx = 0.f;
    for (int k = 0; k < BN_SLOTS; ++k) {
      sdz += atomicExch(acc + k * 2 * C + c, 0.f);
      sdzx += atomicExch(acc + k * 2 * C + C + c, 0.f);
    }
    coef[c] = sdz;
    coef[C + c] = sdzx;
    if (dw) dw[c] += sdzx;
    if (db) db[c] += sdz;
  }
  if (tid == 0) atomicExch(ticket, 0u);
}

template <bool SP, typename T>
__global__ __launch_bounds__(TPB) void bn_bwd_apply_kernel(const T* __restrict__ dy, const T* __restrict__ y,
                                                           const T* __restrict__ x, const float* __restrict__ save,
                                                           const float* __restrict__ w, const float* __restrict__ acc,
                                                           long M, int C, int batch, T* __restrict__ dx,
                                                           T* __restrict__ dres, XSplice xs) {
  const int G = C / 8, rpi = TPB / G, tid = threadIdx.x;
  const int g = tid % G, r = tid / G;
  if (r >= rpi) return;
  float k1[8], k2[8], k3[8], mean[8], rstd[8];
  const float inv_m = 1.f / (float)M;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const int c = g * 8 + e;
    mean[e] = save[c];
    rstd[e] = save[C + c];
    k1[e] = w[c] * rstd[e];                          // dx = k1 (dz - k2 - xhat k3)
    k2[e] = batch ? acc[c] * inv_m : 0.f;
    k3[e] = batch ? acc[C + c] * inv_m : 0.f;
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

// IIT_BN_ROWS = rows per thread group (A/B of the grid size; default 8); IIT_BN_ROWS=0 sizes the grid instead:
// ceil(want / IIT_BN_GRID) rows (default target 1024 workgroups, 4 per CU), so the small layer-3 / layer-4 tensors
// spread over more CUs (fewer serial row loads per thread) and the big ones keep ~8 rows.  Read once per process.
int env_int(const char* name, int dflt, int lo, int hi) {
  const char* e = getenv(name);
  const int r = e ? atoi(e) : dflt;
  return r >= lo && r <= hi ? r : dflt;
}

int bn_rows_per_group() {
  static const int v = env_int("IIT_BN_ROWS", 8, 0, 256);
  return v;
}

int grid_for(long M, int C) {
  static const int target = env_int("IIT_BN_GRID", 1024, 64, 2048);
  const int rpi = TPB / (C / 8);
  const long want = (M + rpi - 1) / rpi;
  int rows = bn_rows_per_group();
  if (rows == 0) rows = (int)((want + target - 1) / target);
  if (rows < 1) rows = 1;
  long g = (want + rows - 1) / rows;
  if (g < 1) g = 1;
  if (g > 2048) g = 2048;
  return (int)g;
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

// forward: ws = per-module accumulator (fp32 [BN_SLOTS][2C] + a u32 ticket after it, zero at the first call, re-armed by
// every call); y = relu?(bn(x) (+ res)); save [2C] = mean, rstd (the batch's in training, the running ones in eval)
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

// the two-level reduction (per-workgroup partials stored channel-major + one wave per channel summing them in a fixed
// order): bit-identical run to run, unlike the memory-side fp32 atomics + ticketed last workgroup of the default path,
// which measured faster (forward 16-21 vs 25-31 us on layers 1-4, PVR bf16 step 8.25 vs 8.91 ms,
// profiles/bn_reduction_r6.txt) -- so it serves deterministic mode (ops/bn.py passes ``two_level``) and
// IIT_BN_REDUCE=two

constexpr int BN_PART_MAX = 2048;  // grid_for's cap: partials per channel

template <typename T>
int bn_fwd_impl(const void* x, const void* res, void* y, float* ws, float* rmean, float* rvar, const float* w,
                const float* b, long M, int C, float eps, int relu, int training, float* save, float momentum,
                long long* nbt, const XSplice& xs, int two_level, hipStream_t s) {
  const int grid = grid_for(M, C);
  unsigned* ticket = (unsigned*)(ws + BN_SLOTS * 2 * C);
  float* part = two_level ? ws + BN_SLOTS * 2 * C + 4 : nullptr;  // (16-B aligned after the ticket)
  // the splice-reading instantiations only where a splice is given (the others keep the lean inner loop)
  if (xs.src) {
    if (training) {
      hipLaunchKernelGGL((bn_stats_kernel<true, T>), dim3(grid), dim3(TPB), 0, s, (const T*)x, M, C, ws, ticket, save,
                         rmean, rvar, eps, momentum, nbt, xs, part);
      if (part)
        hipLaunchKernelGGL((bn_finalize_kernel<true, T>), dim3(C), dim3(64), 0, s, (const T*)x, (const float*)part,
                           grid, M, C, save, rmean, rvar, eps, momentum, nbt, xs);
    }
    hipLaunchKernelGGL((bn_apply_kernel<true, T>), dim3(grid), dim3(TPB), 0, s, (const T*)x, (const T*)res, (T*)y,
                       save, (const float*)rmean, (const float*)rvar, w, b, M, C, eps, relu, training, xs);
  } else {
    if (training) {
      hipLaunchKernelGGL((bn_stats_kernel<false, T>), dim3(grid), dim3(TPB), 0, s, (const T*)x, M, C, ws, ticket, save,
                         rmean, rvar, eps, momentum, nbt, xs, part);
      if (part)
        hipLaunchKernelGGL((bn_finalize_kernel<false, T>), dim3(C), dim3(64), 0, s, (const T*)x, (const float*)part,
                           grid, M, C, save, rmean, rvar, eps, momentum, nbt, xs);
    }
    hipLaunchKernelGGL((bn_apply_kernel<false, T>), dim3(grid), dim3(TPB), 0, s, (const T*)x, (const T*)res, (T*)y,
                       save, (const float*)rmean, (const float*)rvar, w, b, M, C, eps, relu, training, xs);
  }
  return (int)hipGetLastError();
}

template <typename T>
int bn_bwd_impl(const void* dy, const void* y, const void* x, const float* save, const float* w, float* ws,
                float* coef, long M, int C, int training, void* dx, void* dres, float* dw, float* db,
                const XSplice& xs, int two_level, hipStream_t s) {
  const int grid = grid_for(M, C);
  unsigned* ticket = (unsigned*)(ws + BN_SLOTS * 2 * C);
  float* part = two_level ? ws + BN_SLOTS * 2 * C + 4 : nullptr;
  if (xs.src) {
    hipLaunchKernelGGL((bn_bwd_stats_kernel<true, T>), dim3(grid), dim3(TPB), 0, s, (const T*)dy, (const T*)y,
                       (const T*)x, save, M, C, ws, ticket, coef, dw, db, xs, part);
  } else {
    hipLaunchKernelGGL((bn_bwd_stats_kernel<false, T>), dim3(grid), dim3(TPB), 0, s, (const T*)dy, (const T*)y,
                       (const T*)x, save, M, C, ws, ticket, coef, dw, db, xs, part);
  }
  if (part)
    hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3(C), dim3(64), 0, s, (const float*)part, grid, C, coef, dw, db);
  if (xs.src)
    hipLaunchKernelGGL((bn_bwd_apply_kernel<true, T>), dim3(grid), dim3(TPB), 0, s, (const T*)dy, (const T*)y,
                       (const T*)x, save, w, (const float*)coef, M, C, training, (T*)dx, (T*)dres, xs);
  else
    hipLaunchKernelGGL((bn_bwd_apply_kernel<false, T>), dim3(grid), dim3(TPB), 0, s, (const T*)dy, (const T*)y,
                       (const T*)x, save, w, (const float*)coef, M, C, training, (T*)dx, (T*)dres, xs);
  return (int)hipGetLastError();
}

// ``f32``: the activations (x, res, y, dy, dx, dres, the splice source) are fp32 instead of bf16
IIT_EXPORT int iit_bn_fwd(const void* x, const void* res, void* y, float* ws, float* rmean, float* rvar,
                          const float* w, const float* b, long M, int C, float eps, int relu, int training,
                          float* save, float momentum, long long* nbt, const void* src, const void* spec, int H,
                          int W, int f32, int two_level, void* stream) {
  if (!shape_ok(M, C, x) || ((uintptr_t)y & 15) || (res && ((uintptr_t)res & 15))) return (int)hipErrorInvalidValue;
  if (!rmean || !rvar) return (int)hipErrorInvalidValue;
  XSplice xs;
  if (!make_xsplice(xs, src, spec, M, C, H, W)) return (int)hipErrorInvalidValue;
  hipStream_t s = (hipStream_t)stream;
  return f32 ? bn_fwd_impl<float>(x, res, y, ws, rmean, rvar, w, b, M, C, eps, relu, training, save, momentum, nbt, xs,
                                   two_level, s)
             : bn_fwd_impl<__bf16>(x, res, y, ws, rmean, rvar, w, b, M, C, eps, relu, training, save, momentum, nbt, xs,
                                   two_level, s);
}

// backward: ws as in the forward; coef [2C] scratch; dx (and dres = the residual's gradient when non-null);
// dw / db (nullable) ACCUMULATED into
IIT_EXPORT int iit_bn_bwd(const void* dy, const void* y, const void* x, const float* save, const float* w,
                          float* ws, float* coef, long M, int C, int training, void* dx, void* dres, float* dw,
                          float* db, const void* src, const void* spec, int H, int W, int f32, int two_level,
                          void* stream) {
  if (!shape_ok(M, C, dy) || ((uintptr_t)x & 15) || ((uintptr_t)dx & 15) || (y && ((uintptr_t)y & 15)) ||
      (dres && ((uintptr_t)dres & 15)))
    return (int)hipErrorInvalidValue;
  XSplice xs;
  if (!make_xsplice(xs, src, spec, M, C, H, W)) return (int)hipErrorInvalidValue;
  hipStream_t s = (hipStream_t)stream;
  return f32 ? bn_bwd_impl<float>(dy, y, x, save, w, ws, coef, M, C, training, dx, dres, dw, db, xs, two_level, s)
             : bn_bwd_impl<__bf16>(dy, y, x, save, w, ws, coef, M, C, training, dx, dres, dw, db, xs, two_level, s);
}

// Training statistics from a convolution epilogue's per-tile column records (gemm_glds_body.h E_BF16_CS, written by
// csrc/conv_nhwc.hip for the conv whose output this BatchNorm reads): T row tiles of R rows each,
// cstat[(k C + c) T + t], k = 0 the tile's pivot p_t (its first row), 1 S1_t = sum (v - p_t), 2 S2_t = sum (v - p_t)^2.
// One workgroup per channel combines them around the global pivot P = p_0 (the batch's first row, as bn_stats_kernel):
// sum (v - P) = sum_t S1_t + R d_t, sum (v - P)^2 = sum_t S2_t + 2 d_t S1_t + R d_t^2 (d_t = p_t - P), in a fixed order
// (bit-identical run to run), then mean / rstd, the running statistics and num_batches_tracked as the stats kernel's
// last workgroup.  Replaces the statistics pass over the activation.
__global__ __launch_bounds__(256) void bn_tile_finalize_kernel(const float* __restrict__ cstat, int T, int R, long M,
                                                               int C, float* __restrict__ save, float* rmean,
                                                               float* rvar, float eps, float momentum, long long* nbt) {
  __shared__ float red[2][256];
  const int c = blockIdx.x, tid = threadIdx.x;
  const float* pv = cstat + (long)c * T;
  const float* s1 = cstat + (long)(C + c) * T;
  const float* s2 = cstat + (long)(2 * C + c) * T;
  const float P = pv[0], fr = (float)R;
  float a = 0.f, q = 0.f;
  for (int t = tid; t < T; t += 256) {
    const float d = pv[t] - P, u = s1[t];
    a += __builtin_fmaf(fr, d, u);
    q += s2[t] + d * __builtin_fmaf(fr, d, 2.f * u);
  }
  red[0][tid] = a;
  red[1][tid] = q;
  __syncthreads();
  for (int st = 128; st > 0; st >>= 1) {
    if (tid < st) {
      red[0][tid] += red[0][tid + st];
      red[1][tid] += red[1][tid + st];
    }
    __syncthreads();
  }
  if (tid != 0) return;
  const float dm = red[0][0] / (float)M;  // mean - P
  const float mean = P + dm;
  const float var = fmaxf(red[1][0] / (float)M - dm * dm, 0.f);
  save[c] = mean;
  save[C + c] = rsqrtf(var + eps);
  if (rmean) {
    const float unb = M > 1 ? var * (float)M / (float)(M - 1) : var;
    rmean[c] = (1.f - momentum) * rmean[c] + momentum * mean;
    rvar[c] = (1.f - momentum) * rvar[c] + momentum * unb;
  }
  if (c == 0 && nbt) nbt[0] += 1;
}

// training forward of a bf16 activation whose statistics came from its producer's epilogue (``cstat``, T tiles of R
// rows, T R = M): the tile finalize, then the apply pass (no statistics pass over x)
IIT_EXPORT int iit_bn_fwd_tiles(const void* x, const void* res, void* y, const float* cstat, int T, int R,
                                float* rmean, float* rvar, const float* w, const float* b, long M, int C, float eps,
                                int relu, float* save, float momentum, long long* nbt, void* stream) {
  if (!shape_ok(M, C, x) || ((uintptr_t)y & 15) || (res && ((uintptr_t)res & 15))) return (int)hipErrorInvalidValue;
  if (!rmean || !rvar || !cstat || T < 1 || R < 1 || (long)T * R != M) return (int)hipErrorInvalidValue;
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(bn_tile_finalize_kernel, dim3(C), dim3(256), 0, s, cstat, T, R, M, C, save, rmean, rvar, eps,
                     momentum, nbt);
  const XSplice xs{};
  hipLaunchKernelGGL((bn_apply_kernel<false, __bf16>), dim3(grid_for(M, C)), dim3(TPB), 0, s, (const __bf16*)x,
                     (const __bf16*)res, (__bf16*)y, save, (const float*)rmean, (const float*)rvar, w, b, M, C, eps,
                     relu, 1, xs);
  return (int)hipGetLastError();
}

// floats of the per-module accumulator ``ws`` (ops/bn.py allocates it zeroed)
IIT_EXPORT int iit_bn_ws_floats(int C) { return BN_SLOTS * 2 * C + 4 + 2 * C * BN_PART_MAX; }
