// Interchange-intervention splice driven by a patch-spec range table.
//
// The reference splices with a Python hook per site: ``out = act.clone(); out[idx] = src[idx]``
// (/root/reference/iit/model_pairs/base_model_pair.py:151-163), i.e. a clone, index tensors and an index_put per
// call; its gradient is the clone's gradient with the spliced slice zeroed (the source is a detached constant).
// Here a ``TorchIndex`` (None / int / slice / list atoms per dimension, /root/reference/iit/utils/index.py:28-47)
// is lowered once on the host to a range table: per dimension (up to 4) up to 8 half-open ranges [lo, hi); an
// element is selected iff every coordinate lies in one of its dimension's ranges.  One launch then produces
//   forward   out = selected ? src : act          (src may be broadcast: per-dimension strides, 0 = broadcast)
//   backward  g'  = selected ? 0   : g            (also the StopGrad zero-gradient mask, stop_grad_pair.py:62-75)
//   divide    out = selected ? act / s : act      (StopGrad's activation scaling, stop_grad_pair.py:37-44)
// with no index tensors, no host synchronisation and a single pass over the activation (graph-capturable).
// Each thread handles 8 consecutive elements of the innermost dimension (16-B bf16 / 32-B fp32 vector access).
#include "common.h"
#include "splice_spec.h"

template <typename T>
__device__ __forceinline__ float ld_f(const T* p) {
  if constexpr (sizeof(T) == 2) return bf2f(*p);
  else return *p;
}

template <typename T>
__device__ __forceinline__ T st_f(float v) {
  if constexpr (sizeof(T) == 2) return f2bf(v);
  else return v;
}

// MODE 0: out = sel ? src : act;  MODE 1: out = sel ? 0 : act;  MODE 2: out = sel ? act / scale : act, computed
// as torch does on the GPU for ``act / python_float``: a multiply by the fp32 reciprocal (bit-identical to the
// reference hook's result on a GPU).
// VEC = 8: each thread takes 8 consecutive innermost elements (innermost dimension a multiple of 8); VEC = 1: one
// element per thread (any shape, e.g. a 6 x 6 feature map's spatial quadrant).
template <typename T, int MODE, int VEC>
__global__ __launch_bounds__(256) void splice_kernel(const T* __restrict__ act, const T* __restrict__ src,
                                                     T* __restrict__ out, long nv, SpliceSpec sp, float scale) {
  const long iv = (long)blockIdx.x * 256 + threadIdx.x;
  if (iv >= nv) return;
  const int d3 = sp.shape[3];
  const long e0 = iv * VEC;  // VEC == 8: the 8 elements share coordinates 0..2
  long q = e0 / d3;
  const int c3 = (int)(e0 - q * d3);
  const int c2 = (int)(q % sp.shape[2]);
  q /= sp.shape[2];
  const int c1 = (int)(q % sp.shape[1]);
  const int c0 = (int)(q / sp.shape[1]);
  const bool row = in_ranges(sp, 0, c0) && in_ranges(sp, 1, c1) && in_ranges(sp, 2, c2);
  T v[VEC];
  if constexpr (VEC == 8 && sizeof(T) == 2) {
    *(bf16x8*)v = *(const bf16x8*)(act + e0);
  } else if constexpr (VEC == 8) {
    *(float4*)v = *(const float4*)(act + e0);
    *(float4*)(v + 4) = *(const float4*)(act + e0 + 4);
  } else {
    v[0] = act[e0];
  }
  if (row) {
    const long sb = (long)c0 * sp.sstride[0] + (long)c1 * sp.sstride[1] + (long)c2 * sp.sstride[2];
#pragma unroll
    for (int e = 0; e < VEC; ++e) {
      if (!in_ranges(sp, 3, c3 + e)) continue;
      if constexpr (MODE == 0) v[e] = src[sb + (long)(c3 + e) * sp.sstride[3]];
      else if constexpr (MODE == 1) v[e] = st_f<T>(0.f);
      else v[e] = st_f<T>(ld_f(&v[e]) * (1.f / scale));
    }
  }
  if constexpr (VEC == 8 && sizeof(T) == 2) {
    *(bf16x8*)(out + e0) = *(bf16x8*)v;
  } else if constexpr (VEC == 8) {
    *(float4*)(out + e0) = *(float4*)v;
    *(float4*)(out + e0 + 4) = *(float4*)(v + 4);
  } else {
    out[e0] = v[0];
  }
}

IIT_EXPORT int iit_splice_spec_size() { return (int)sizeof(SpliceSpec); }

// ``spec``: host pointer to one SpliceSpec (copied into the kernel arguments, so a captured graph keeps it).
// act / out contiguous with n elements (vector path: n and the innermost dimension multiples of 8, 16-B aligned);
// out may alias act (each thread reads its elements before writing them).
IIT_EXPORT int iit_splice(const void* act, const void* src, void* out, long n, const void* spec, int f32, int mode,
                          float scale, void* stream) {
  const SpliceSpec sp = *(const SpliceSpec*)spec;
  const bool vec = n % 8 == 0 && sp.shape[3] % 8 == 0 && ((uintptr_t)act % 16) == 0 && ((uintptr_t)out % 16) == 0;
  const long nv = vec ? n / 8 : n;
  const dim3 grid((unsigned)((nv + 255) / 256));
  hipStream_t s = (hipStream_t)stream;
#define SPL(T, M, V)                                                                                               \
  hipLaunchKernelGGL((splice_kernel<T, M, V>), grid, dim3(256), 0, s, (const T*)act, (const T*)src, (T*)out, nv,  \
                     sp, scale)
#define SPL_M(T, V)                 \
  if (mode == 0) SPL(T, 0, V);      \
  else if (mode == 1) SPL(T, 1, V); \
  else SPL(T, 2, V);
  if (f32) {
    if (vec) { SPL_M(float, 8) } else { SPL_M(float, 1) }
  } else {
    if (vec) { SPL_M(__bf16, 8) } else { SPL_M(__bf16, 1) }
  }
#undef SPL_M
#undef SPL
  return hipGetLastError();
}

// Sparse paired splice (the paired forward's ``mlp.hook_post`` sites, iit_amd/ops/hip_ops.py MLPInPairFn): the
// activation holds T base rows followed by T source rows ([2T][ld], rows = the spec's flattened leading three
// dimensions); one thread per SELECTED element -- the work is the size of the index, not of the activation:
//   MODE 0  act[row][col] = act[row + T][col]   (forward: the source value into the base row, in place, right after
//                                                the producing GEMM wrote both halves)
//   MODE 1  act[row][col] = 0                   (backward: the spliced elements' gradient, in the producer's dpre)
// ``cnt[d]`` = number of selected coordinates of dimension d; thread i is decoded mixed-radix over them.
__device__ __forceinline__ int range_coord(const SpliceSpec& sp, int d, int k) {
#pragma unroll
  for (int r = 0; r < 8; ++r) {
    if (r >= sp.nr[d]) break;
    const int len = sp.hi[d][r] - sp.lo[d][r];
    if (k < len) return sp.lo[d][r] + k;
    k -= len;
  }
  return sp.lo[d][0];
}

template <int MODE>
__global__ __launch_bounds__(256) void sparse_pair_kernel(__bf16* __restrict__ act, long T, long ld, SpliceSpec sp,
                                                          long total, int n1, int n2, int n3) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= total) return;
  long q = i;
  const int k3 = (int)(q % n3); q /= n3;
  const int k2 = (int)(q % n2); q /= n2;
  const int k1 = (int)(q % n1);
  const int k0 = (int)(q / n1);
  const int c0 = range_coord(sp, 0, k0), c1 = range_coord(sp, 1, k1), c2 = range_coord(sp, 2, k2);
  const int c3 = range_coord(sp, 3, k3);
  const long row = ((long)c0 * sp.shape[1] + c1) * sp.shape[2] + c2;
  if (MODE == 0) act[row * ld + c3] = act[(row + T) * ld + c3];
  else act[row * ld + c3] = f2bf(0.f);
}

IIT_EXPORT int iit_sparse_pair(void* act, long T, long ld, const void* spec, int mode, void* stream) {
  const SpliceSpec sp = *(const SpliceSpec*)spec;
  long cnt[4];
  long total = 1;
  for (int d = 0; d < 4; ++d) {
    cnt[d] = 0;
    for (int r = 0; r < sp.nr[d]; ++r) cnt[d] += sp.hi[d][r] - sp.lo[d][r];
    total *= cnt[d];
  }
  if ((long)sp.shape[0] * sp.shape[1] * sp.shape[2] != T) return (int)hipErrorInvalidValue;
  if (total == 0) return 0;
  const dim3 grid((unsigned)((total + 255) / 256));
  hipStream_t s = (hipStream_t)stream;
  if (mode == 0)
    hipLaunchKernelGGL(sparse_pair_kernel<0>, grid, dim3(256), 0, s, (__bf16*)act, T, ld, sp, total, (int)cnt[1],
                       (int)cnt[2], (int)cnt[3]);
  else
    hipLaunchKernelGGL(sparse_pair_kernel<1>, grid, dim3(256), 0, s, (__bf16*)act, T, ld, sp, total, (int)cnt[1],
                       (int)cnt[2], (int)cnt[3]);
  return hipGetLastError();
}
