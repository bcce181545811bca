// MFMA GEMM for gfx950 (MI355X): C[M,N] = A[M,K] * B[K,N] with fused epilogues.
//
// * 256-thread workgroups (4 wave64s as 2x2), output tile BM x BN, BK = 64.
// * v_mfma_f32_16x16x32_bf16: each wave owns a (BM/2) x (BN/2) sub-tile of
//   16x16 accumulators (fp32 in the unified VGPR/AGPR file).
// * Operands may be "k-contiguous" (A stored [M][K], B stored [N][K]) or
//   "k-major" (A stored [K][M], B stored [K][N]); k-major tiles are staged as
//   loaded and read with the gfx950 transpose read ds_read_b64_tr_b16, so the
//   weight-gradient GEMMs (X^T dY) need no transpose pass.  fp32 operands (the
//   fp32 residual-stream gradient) are converted to bf16 while staging.
// * Register-staged double-buffered LDS: global loads of tile k+1 are issued
//   before the MFMAs of tile k and written to the other LDS buffer after them;
//   one barrier per K tile.
// * XCD-aware bijective workgroup remap so the tiles one XCD works on share
//   A row panels in that XCD's L2.
// * Epilogues: bf16 (+bias, +3-way bias for packed QKV), fp32 residual add,
//   bias+gelu_new (writes pre and post), dgelu, fp32 accumulate (plain or
//   atomic for split-K) incl. a head-blocked scatter for the packed QKV weight
//   gradient into TL-layout W_Q/W_K/W_V gradients.
#include "common.h"

enum Epi : int {
  EPI_BF16 = 0,       // C(bf16) = acc (+bias[n])
  EPI_BF16_BIAS3 = 1, // C(bf16) = acc + bias[n / bias_cols][n % bias_cols]
  EPI_F32_RESID = 2,  // C(f32)  = resid + acc (+bias)
  EPI_GELU = 3,       // pre = acc + bias -> C2(bf16); C(bf16) = gelu_new(pre)
  EPI_DGELU = 4,      // C(bf16) = acc * gelu_new'(aux_pre)
  EPI_F32_ACC = 5,    // C(f32) += acc   (atomic when p.atomic)
  EPI_F32_ACC_QKV = 6,// head-blocked scatter-accumulate into 3 TL-layout grads
  EPI_F32_STORE = 7,  // C(f32) = acc (+bias)
  EPI_GELU_ERF = 8,   // as EPI_GELU with the exact (erf) GELU (BERT)
  EPI_DGELU_ERF = 9,  // as EPI_DGELU with the exact (erf) GELU's derivative
};

struct GemmArgs {
  const void* A;
  const void* B;
  void* C;
  void* C2;
  void* C3;
  const float* bias0;
  const float* bias1;
  const float* bias2;
  const float* resid;
  const void* aux;
  long lda, ldb, ldc, ldc2, ldr;
  int M, N, K;
  int k_per_split;
  int bias_cols;
  int qkv_dh, qkv_H, qkv_d;
  int atomic;
};

template <bool KMAJ, bool F32, int ROWS>
struct TileLoader {
  // chunk = 8 consecutive elements along the contiguous global dimension
  static constexpr int BK = 64;
  static constexpr int CHUNKS = ROWS * BK / 8;
  static constexpr int PER_THREAD = CHUNKS / 256;
  static constexpr int LDS_ROW = KMAJ ? (ROWS + 16) : (BK + 8);
  static constexpr int LDS_ELEMS = KMAJ ? BK * LDS_ROW : ROWS * LDS_ROW;
  uint4 r[PER_THREAD];

  __device__ __forceinline__ void load(const void* base, long ld, int row0, int nrows, int k0, int kend, int tid) {
#pragma unroll
    for (int i = 0; i < PER_THREAD; ++i) {
      const int c = tid + i * 256;
      int row, k;
      if (KMAJ) {
        k = k0 + c / (ROWS / 8);
        row = row0 + (c % (ROWS / 8)) * 8;
      } else {
        row = row0 + c / (BK / 8);
        k = k0 + (c % (BK / 8)) * 8;
      }
      uint4 v = make_uint4(0, 0, 0, 0);
      if (KMAJ) {
        if (k < kend) {
          if (row + 8 <= nrows) {
            v = fetch8<F32>(base, (long)k * ld + row);
          } else if (row < nrows) {
            v = fetch_partial<F32>(base, (long)k * ld + row, nrows - row);
          }
        }
      } else {
        if (row < nrows && k < kend) {
          if (k + 8 <= kend) v = fetch8<F32>(base, (long)row * ld + k);
          else v = fetch_partial<F32>(base, (long)row * ld + k, kend - k);
        }
      }
      r[i] = v;
    }
  }

  template <bool F>
  static __device__ __forceinline__ uint4 fetch8(const void* base, long off) {
    if (!F) {
      return *(const uint4*)((const __bf16*)base + off);
    } else {
      const float4* p = (const float4*)((const float*)base + off);
      float4 a = p[0], b = p[1];
      bf16x8 o = {f2bf(a.x), f2bf(a.y), f2bf(a.z), f2bf(a.w), f2bf(b.x), f2bf(b.y), f2bf(b.z), f2bf(b.w)};
      return __builtin_bit_cast(uint4, o);
    }
  }
  template <bool F>
  static __device__ __forceinline__ uint4 fetch_partial(const void* base, long off, int n) {
    bf16x8 o;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      float x = 0.f;
      if (e < n) x = F ? ((const float*)base)[off + e] : bf2f(((const __bf16*)base)[off + e]);
      o[e] = f2bf(x);
    }
    return __builtin_bit_cast(uint4, o);
  }

  __device__ __forceinline__ void store(__bf16* lds, int tid) const {
#pragma unroll
    for (int i = 0; i < PER_THREAD; ++i) {
      const int c = tid + i * 256;
      int off;
      if (KMAJ) off = (c / (ROWS / 8)) * LDS_ROW + (c % (ROWS / 8)) * 8;
      else off = (c / (BK / 8)) * LDS_ROW + (c % (BK / 8)) * 8;
      *(uint4*)(lds + off) = r[i];
    }
  }

  // MFMA 16x16x32 operand fragment: lane l gets X[row0 + (l&15)][kbase + 8*(l>>4) + j], j = 0..7
  static __device__ __forceinline__ bf16x8 frag(const __bf16* lds, int row0, int kbase, int lane) {
    if (!KMAJ) {
      return *(const bf16x8*)(lds + (row0 + (lane & 15)) * LDS_ROW + kbase + 8 * (lane >> 4));
    } else {
      const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
      const __bf16* a0 = lds + (kbase + 8 * g + q) * LDS_ROW + row0 + 4 * p;
      typedef __attribute__((address_space(3))) i16x4 lds_i16x4;
      const i16x4 v0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_i16x4*)(a0));
      const i16x4 v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_i16x4*)(a0 + 4 * LDS_ROW));
      // whole-vector reinterpretation: element-wise bit_casts of the tr16 results are
      // miscompiled by hipcc (ROCm 7.2) into duplicated halves
      const i16x8 w = __builtin_shufflevector(v0, v1, 0, 1, 2, 3, 4, 5, 6, 7);
      return __builtin_bit_cast(bf16x8, w);
    }
  }
};

__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int xcd = bid % 8;
  const int q = nwg / 8, r = nwg % 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + bid / 8;
}

template <int BM, int BN, bool AKM, bool BKM, bool AF32, bool BF32, int EPI>
__global__ __launch_bounds__(256) void gemm_kernel(GemmArgs p) {
  constexpr int BK = 64;
  constexpr int WM = BM / 2, WN = BN / 2;
  constexpr int TM = WM / 16, TN = WN / 16;
  using LA = TileLoader<AKM, AF32, BM>;
  using LB = TileLoader<BKM, BF32, BN>;
  __shared__ __attribute__((aligned(16))) __bf16 smem[2 * (LA::LDS_ELEMS + LB::LDS_ELEMS)];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int tiles_n = (p.N + BN - 1) / BN, tiles_m = (p.M + BM - 1) / BM;
  const int nwg = tiles_n * tiles_m;
  const int t = xcd_remap(blockIdx.x, nwg);
  const int m0 = (t / tiles_n) * BM, n0 = (t % tiles_n) * BN;
  const int kbeg = blockIdx.y * p.k_per_split;
  const int kend = min(p.K, kbeg + p.k_per_split);
  const int ntiles = (kend - kbeg + BK - 1) / BK;

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  LA la;
  LB lb;
  constexpr int STAGE = LA::LDS_ELEMS + LB::LDS_ELEMS;
#define SA(buf) (smem + (buf) * STAGE)
#define SB(buf) (smem + (buf) * STAGE + LA::LDS_ELEMS)

  if (ntiles > 0) {
    la.load(p.A, p.lda, m0, p.M, kbeg, kend, tid);
    lb.load(p.B, p.ldb, n0, p.N, kbeg, kend, tid);
    la.store(SA(0), tid);
    lb.store(SB(0), tid);
  }
  __syncthreads();
  int cur = 0;
  for (int kt = 0; kt < ntiles; ++kt) {
    const bool more = kt + 1 < ntiles;
    if (more) {
      la.load(p.A, p.lda, m0, p.M, kbeg + (kt + 1) * BK, kend, tid);
      lb.load(p.B, p.ldb, n0, p.N, kbeg + (kt + 1) * BK, kend, tid);
    }
#pragma unroll
    for (int s = 0; s < BK / 32; ++s) {
      bf16x8 a[TM], b[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) a[i] = LA::frag(SA(cur), wm * WM + i * 16, s * 32, lane);
#pragma unroll
      for (int j = 0; j < TN; ++j) b[j] = LB::frag(SB(cur), wn * WN + j * 16, s * 32, lane);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
    }
    if (more) {
      la.store(SA(cur ^ 1), tid);
      lb.store(SB(cur ^ 1), tid);
    }
    __syncthreads();
    cur ^= 1;
  }

#undef SA
#undef SB
  // ---------------------------------------------------------------- epilogue
#pragma unroll
  for (int i = 0; i < TM; ++i) {
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int col = n0 + wn * WN + j * 16 + (lane & 15);
      if (col >= p.N) continue;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = m0 + wm * WM + i * 16 + 4 * (lane >> 4) + r;
        if (row >= p.M) continue;
        float v = acc[i][j][r];
        if (EPI == EPI_BF16) {
          if (p.bias0) v += p.bias0[col];
          ((__bf16*)p.C)[(long)row * p.ldc + col] = f2bf(v);
        } else if (EPI == EPI_BF16_BIAS3) {
          const int w = col / p.bias_cols, o = col - w * p.bias_cols;
          const float* bb = w == 0 ? p.bias0 : (w == 1 ? p.bias1 : p.bias2);
          if (bb) v += bb[o];
          ((__bf16*)p.C)[(long)row * p.ldc + col] = f2bf(v);
        } else if (EPI == EPI_F32_RESID) {
          if (p.bias0) v += p.bias0[col];
          ((float*)p.C)[(long)row * p.ldc + col] = p.resid[(long)row * p.ldr + col] + v;
        } else if (EPI == EPI_GELU || EPI == EPI_GELU_ERF) {
          if (p.bias0) v += p.bias0[col];
          if (p.C2) ((__bf16*)p.C2)[(long)row * p.ldc2 + col] = f2bf(v);  // null: an inference forward
          ((__bf16*)p.C)[(long)row * p.ldc + col] = f2bf(EPI == EPI_GELU ? gelu_new_f(v) : gelu_erf_f(v));
        } else if (EPI == EPI_DGELU || EPI == EPI_DGELU_ERF) {
          const float pre = bf2f(((const __bf16*)p.aux)[(long)row * p.ldc2 + col]);
          const float gp = EPI == EPI_DGELU ? gelu_new_grad_f(pre) : gelu_erf_grad_f(pre);
          ((__bf16*)p.C)[(long)row * p.ldc + col] = f2bf(v * gp);
        } else if (EPI == EPI_F32_ACC) {
          float* dst = (float*)p.C + (long)row * p.ldc + col;
          if (p.atomic) atomicAdd(dst, v);
          else *dst += v;
        } else if (EPI == EPI_F32_ACC_QKV) {
          const int hd = p.qkv_H * p.qkv_dh;
          const int w = col / hd, rem = col - w * hd;
          const int h = rem / p.qkv_dh, jj = rem - h * p.qkv_dh;
          float* base = (float*)(w == 0 ? p.C : (w == 1 ? p.C2 : p.C3));
          float* dst = base + ((long)h * p.qkv_d + row) * p.qkv_dh + jj;
          if (p.atomic) atomicAdd(dst, v);
          else *dst += v;
        } else if (EPI == EPI_F32_STORE) {
          if (p.bias0) v += p.bias0[col];
          ((float*)p.C)[(long)row * p.ldc + col] = v;
        }
      }
    }
  }
}

// ---------------------------------------------------------------------------- dispatch
template <int BM, int BN, bool AKM, bool BKM, bool AF32, bool BF32, int EPI>
static hipError_t launch_t(const GemmArgs& a, int splits, hipStream_t s) {
  const int tiles = cdiv(a.M, BM) * cdiv(a.N, BN);
  dim3 grid(tiles, splits);
  hipLaunchKernelGGL((gemm_kernel<BM, BN, AKM, BKM, AF32, BF32, EPI>), grid, dim3(256), 0, s, a);
  return hipGetLastError();
}

template <bool AKM, bool BKM, bool AF32, bool BF32, int EPI>
static hipError_t launch_tiles(const GemmArgs& a, int splits, int big, hipStream_t s) {
  if (big) return launch_t<128, 128, AKM, BKM, AF32, BF32, EPI>(a, splits, s);
  return launch_t<64, 64, AKM, BKM, AF32, BF32, EPI>(a, splits, s);
}

// mode bits: 1 = A k-major, 2 = B k-major, 4 = A fp32, 8 = B fp32
#define IIT_GEMM_CASE(MODE, AKM, BKM, AF, BF, EPI) \
  if (mode == (MODE) && epi == (EPI)) return launch_tiles<AKM, BKM, AF, BF, EPI>(a, splits, big, s);

IIT_EXPORT int iit_gemm(const void* A, const void* B, void* C, void* C2, void* C3, const float* bias0,
                        const float* bias1, const float* bias2, const float* resid, const void* aux, long lda,
                        long ldb, long ldc, long ldc2, long ldr, int M, int N, int K, int mode, int epi, int splits,
                        int big, int bias_cols, int qkv_dh, int qkv_H, int qkv_d, int atomic, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  if (M <= 0 || N <= 0) return 0;
  GemmArgs a;
  a.A = A; a.B = B; a.C = C; a.C2 = C2; a.C3 = C3;
  a.bias0 = bias0; a.bias1 = bias1; a.bias2 = bias2; a.resid = resid; a.aux = aux;
  a.lda = lda; a.ldb = ldb; a.ldc = ldc; a.ldc2 = ldc2; a.ldr = ldr;
  a.M = M; a.N = N; a.K = K;
  if (splits < 1) splits = 1;
  int kps = (K + splits - 1) / splits;
  kps = (kps + 63) / 64 * 64;
  splits = (K + kps - 1) / kps;
  if (splits < 1) splits = 1;
  a.k_per_split = kps;
  a.bias_cols = bias_cols; a.qkv_dh = qkv_dh; a.qkv_H = qkv_H; a.qkv_d = qkv_d;
  a.atomic = atomic || splits > 1;
  // forward / dX GEMMs: both operands k-contiguous
  IIT_GEMM_CASE(0, false, false, false, false, EPI_BF16)
  IIT_GEMM_CASE(0, false, false, false, false, EPI_BF16_BIAS3)
  IIT_GEMM_CASE(0, false, false, false, false, EPI_F32_RESID)
  IIT_GEMM_CASE(0, false, false, false, false, EPI_GELU)
  IIT_GEMM_CASE(0, false, false, false, false, EPI_GELU_ERF)
  IIT_GEMM_CASE(0, false, false, false, false, EPI_DGELU)
  IIT_GEMM_CASE(0, false, false, false, false, EPI_DGELU_ERF)
  IIT_GEMM_CASE(0, false, false, false, false, EPI_F32_STORE)
  IIT_GEMM_CASE(0, false, false, false, false, EPI_F32_ACC)
  // forward GEMMs straight from TL-layout ([K][N]) bf16 weights: B k-major (tr16 reads)
  IIT_GEMM_CASE(2, false, true, false, false, EPI_BF16)
  IIT_GEMM_CASE(2, false, true, false, false, EPI_BF16_BIAS3)
  IIT_GEMM_CASE(2, false, true, false, false, EPI_F32_RESID)
  IIT_GEMM_CASE(2, false, true, false, false, EPI_GELU)
  IIT_GEMM_CASE(2, false, true, false, false, EPI_GELU_ERF)
  IIT_GEMM_CASE(2, false, true, false, false, EPI_F32_STORE)
  // dX from the fp32 residual-stream gradient
  IIT_GEMM_CASE(4, false, false, true, false, EPI_BF16)
  IIT_GEMM_CASE(4, false, false, true, false, EPI_DGELU)
  IIT_GEMM_CASE(4, false, false, true, false, EPI_F32_ACC)
  IIT_GEMM_CASE(4, false, false, true, false, EPI_F32_STORE)
  // weight gradients: both operands k-major (reduction over tokens)
  IIT_GEMM_CASE(1, true, false, false, false, EPI_F32_ACC)
  IIT_GEMM_CASE(2, false, true, false, false, EPI_F32_ACC)
  IIT_GEMM_CASE(3, true, true, false, false, EPI_F32_ACC)
  IIT_GEMM_CASE(3, true, true, false, false, EPI_F32_ACC_QKV)
  IIT_GEMM_CASE(11, true, true, false, true, EPI_F32_ACC)
  IIT_GEMM_CASE(3, true, true, false, false, EPI_F32_STORE)
  return (int)hipErrorInvalidValue;
}
