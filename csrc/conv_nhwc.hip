// NHWC bf16 3 x 3 / stride-1 / pad-1 convolution as an implicit GEMM on the LDS-DMA MFMA body (gemm_glds_body.h):
// the ResNet-18 BasicBlock convolutions of the PVR task's low-level model (/root/reference/iit/tasks/mnist_pvr/
// get_alignment.py:9-15, torchvision's resnet18) in place of MIOpen / CK.
//
//   y[n][h][w][co] = sum_{kh, kw, ci} x[n][h + kh - 1][w + kw - 1][ci] * W[co][kh][kw][ci]
//
// is the GEMM  Y [M = N H W][Cout] = A [M][K = 9 Cin] x B^T, with B = the channels-last weight [Cout][3][3][Cin] read
// as [Cout][9 Cin] (mode 0: both operands k-contiguous) and A the implicit im2col matrix: row m = output pixel
// (n, h, w), K index = tap * Cin + ci with the 9 taps outermost.  With Cin % 64 == 0 a 64-deep K-tile is 64 channels
// of ONE tap, i.e. for every row one 128-B segment of one input pixel: ConvRowStager gives each lane of the LDS-DMA
// (global_load_lds) the source address of its row's pixel shifted by the tile's tap -- or the zero page when the
// shifted pixel is outside the image (the padding) -- into exactly the swizzled LDS image the strided stager builds,
// so the main loop, the MFMA fragments and the epilogue are the GEMM's, unchanged.  No im2col buffer, no padding copy.
//
// The input gradient is the same kernel with the tap offsets negated (conv_flip) on A = dY and B = the weight
// re-laid [Cin][3][3][Cout]:  dx[n][h][w][ci] = sum_{kh, kw, co} dy[n][h - kh + 1][w - kw + 1][co] W[co][kh][kw][ci].
#include "gemm_glds_body.h"

namespace {

template <int R, int NW>
struct ConvRowStager {
  static constexpr int RPI = 8;  // rows per LDS-DMA instruction: 8 rows x 128 B (the k-contiguous BK = 64 image)
  static constexpr int N = R / (RPI * NW);
  static_assert(N >= 1, "tile too narrow for the workgroup's waves");
  const __bf16* x;
  const __bf16* zero;
  long pix[N];  // element offset of the lane's row pixel (n, h, w) in x
  int ph[N], pw[N];
  int cc[N];    // the lane's 16-B chunk of its row (source-side swizzle, as Stager<false, R, NW, 64>)
  int off[N];   // wave-uniform LDS offset of instruction i
  int H, W, C, flip, kbeg;

  __device__ __forceinline__ void init(const G2Args& p, int r0g, int kbeg_, int wave, int lane) {
    x = p.A;
    zero = p.zero;
    H = p.conv_h;
    W = p.conv_w;
    C = p.conv_c;
    flip = p.conv_flip;
    kbeg = kbeg_;
    const int hw = H * W;
#pragma unroll
    for (int i = 0; i < N; ++i) {
      const int r0 = i * RPI * NW + wave * RPI;
      const int row = r0 + lane / 8;
      const long m = (long)r0g + row;
      const int n = (int)(m / hw);
      const int rem = (int)(m - (long)n * hw);
      const int h = rem / W;
      ph[i] = h;
      pw[i] = rem - h * W;
      pix[i] = m * C;
      cc[i] = ((lane & 7) ^ kcont_swz<64>(row)) * 8;
      off[i] = r0 * 128;
    }
  }

  __device__ __forceinline__ void stage(int kt, char* img) const {
    const int k0 = kbeg + kt * 64;
    const int tap = k0 / C, ci0 = k0 - tap * C;
    const int th = tap / 3;
    int dh = th - 1, dw = tap - 3 * th - 1;
    if (flip) {
      dh = -dh;
      dw = -dw;
    }
    const long shift = (long)(dh * W + dw) * C + ci0;
#pragma unroll
    for (int i = 0; i < N; ++i) {
      const int hh = ph[i] + dh, ww = pw[i] + dw;
      const bool in = (unsigned)hh < (unsigned)H && (unsigned)ww < (unsigned)W;
      glds16(in ? x + pix[i] + shift + cc[i] : zero + cc[i], img + off[i]);
    }
  }
};

// q = a / d for 0 <= a < 2^24 by a float reciprocal and one correction step (the weight-gradient stager's per-K-tile
// pixel -> (h, w) split; an integer division by a run-time divisor is ~40 instructions)
__device__ __forceinline__ int fdiv(int a, int d, float inv) {
  int q = (int)((float)a * inv);
  if (q * d > a) --q;
  else if ((q + 1) * d <= a) ++q;
  return q;
}

// The weight gradient's B operand: dW [Cout][9 Cin] = dY^T [Cout][K = N H W] x im2col(x) [K][9 Cin], staged k-major
// ([64 pixels][R columns], the image of Stager<true, R, NW, 64>): an N-tile of R columns is R channels [ci0, ci0 + R)
// of ONE tap (Cin % R == 0), so k-row ``pix`` of the tile is one contiguous 2R-byte segment of input pixel ``pix``
// shifted by the tap -- or the zero page outside the image.  The tap is fixed per workgroup; each K-tile recomputes
// the lanes' pixels' (h, w) (the K range advances 64 pixels per K-tile).  Reads the activation from ``p.B``.
template <int R, int NW>
struct ConvColStager {
  static constexpr int CH = R / 8;      // 16-B chunks per k-row
  static constexpr int KRI = 64 / CH;   // k-rows per LDS-DMA instruction
  static constexpr int N = 64 / (NW * KRI);
  static_assert(N >= 1 && (R == 64 || R == 128), "64- or 128-column tiles");
  const __bf16* x;
  const __bf16* zero;
  int kr[N], col[N], off[N];
  int H, W, C, dh, dw, ci0, kbeg;
  float invW, invH;

  __device__ __forceinline__ void init(const G2Args& p, int r0g, int kbeg_, int wave, int lane) {
    x = p.B;
    zero = p.zero;
    H = p.conv_h;
    W = p.conv_w;
    C = p.conv_c;
    kbeg = kbeg_;
    invW = 1.f / (float)W;
    invH = 1.f / (float)H;
    const int tap = r0g / C;
    ci0 = r0g - tap * C;
    const int th = tap / 3;
    dh = th - 1;
    dw = tap - 3 * th - 1;
#pragma unroll
    for (int i = 0; i < N; ++i) {
      const int kr0 = (i * NW + wave) * KRI;
      const int k = kr0 + lane / CH;
      const int ch = lane % CH;
      kr[i] = k;
      col[i] = (((ch >> 1) ^ kmaj_swz<R>(k)) << 4) + ((ch & 1) << 3);
      off[i] = kr0 * R * 2;
    }
  }

  __device__ __forceinline__ void stage(int kt, char* img) const {
#pragma unroll
    for (int i = 0; i < N; ++i) {
      const int pix = kbeg + kt * 64 + kr[i];
      const int q = fdiv(pix, W, invW);
      const int w = pix - q * W;
      const int h = q - fdiv(q, H, invH) * H;
      const int hh = h + dh, ww = w + dw;
      const bool in = (unsigned)hh < (unsigned)H && (unsigned)ww < (unsigned)W;
      glds16(in ? x + (long)(pix + dh * W + dw) * C + ci0 + col[i] : zero + col[i], img + off[i]);
    }
  }
};

template <int BM, int BN, int NS, int NW, int OCC, int EPI>
__global__ __launch_bounds__(NW * 64, OCC) void conv3x3_wgrad_kernel(G2Args p) {
  __shared__ __attribute__((aligned(16))) char smem[GldsSmem<BM, BN, NS, NW, 64, OCC>::BYTES];
  gemm_glds_body<BM, BN, NS, true, true, EPI, NW, 64, OCC, false, void, ConvColStager<BN, NW>>(
      p, blockIdx.x, gridDim.x, blockIdx.y, gridDim.y, smem);
}

// blockIdx.y = K-split (reduction split over the 9 Cin taps-x-channels: every split publishes its fp32 partial tile,
// the last arriver sums them in split order and runs the bf16 epilogue -- deterministic); gridDim.y = 1: no split
// EPI = E_BF16_CS: the epilogue also writes per-tile column statistics of the output (a.cstat) for the BatchNorm that
// reads it (ops/bn.py: the statistics pass over the activation is skipped)
template <int BM, int BN, int NS, int NW, int OCC, int EPI>
__global__ __launch_bounds__(NW * 64, OCC) void conv3x3_kernel(G2Args p) {
  __shared__ __attribute__((aligned(16))) char smem[GldsSmem<BM, BN, NS, NW, 64, OCC>::BYTES];
  gemm_glds_body<BM, BN, NS, false, false, EPI, NW, 64, OCC, false, ConvRowStager<BM, NW>>(p, blockIdx.x, gridDim.x,
                                                                                           blockIdx.y, gridDim.y, smem);
}

template <int BM, int BN, int NS, int NW = 4, int OCC = 1>
hipError_t launch_conv(const G2Args& a, int splits, hipStream_t s) {
  const int tiles = (a.M / BM) * (a.N / BN);
  if (a.cstat)
    hipLaunchKernelGGL((conv3x3_kernel<BM, BN, NS, NW, OCC, E_BF16_CS>), dim3(tiles, splits), dim3(NW * 64), 0, s, a);
  else
    hipLaunchKernelGGL((conv3x3_kernel<BM, BN, NS, NW, OCC, E_BF16>), dim3(tiles, splits), dim3(NW * 64), 0, s, a);
  return hipGetLastError();
}

// tiles (BM, BN, ring depth, waves, workgroups per CU): the output is [N H W][Cout] with Cout 64..512
constexpr int kConvTiles = 6;
const int kConvBM[kConvTiles] = {128, 128, 64, 128, 64, 128};
const int kConvBN[kConvTiles] = {64, 128, 64, 128, 128, 64};

hipError_t launch_conv_tile(const G2Args& a, int tile, int splits, hipStream_t s) {
  switch (tile) {
    case 0: return launch_conv<128, 64, 4>(a, splits, s);
    case 1: return launch_conv<128, 128, 3>(a, splits, s);
    case 2: return launch_conv<64, 64, 4, 4, 2>(a, splits, s);
    case 3: return launch_conv<128, 128, 2, 4, 2>(a, splits, s);
    case 4: return launch_conv<64, 128, 2, 4, 3>(a, splits, s);
    case 5: return launch_conv<128, 64, 2, 4, 2>(a, splits, s);
    default: return hipErrorInvalidValue;
  }
}

// weight-gradient tiles (BM = Cout rows, BN = channels of one tap, ring depth)
constexpr int kWgTiles = 4;
const int kWgBM[kWgTiles] = {64, 128, 128, 64};
const int kWgBN[kWgTiles] = {64, 64, 128, 128};

template <int EPI>
hipError_t launch_wgrad(const G2Args& a, int tile, int splits, hipStream_t s) {
  const dim3 block(256);
#define WG(T, BM_, BN_, NS_)                                                                                 \
  case T:                                                                                                   \
    hipLaunchKernelGGL((conv3x3_wgrad_kernel<BM_, BN_, NS_, 4, 1, EPI>), dim3((a.M / BM_) * (a.N / BN_), splits), \
                       block, 0, s, a);                                                                     \
    break;
  switch (tile) {
    WG(0, 64, 64, 4)
    WG(1, 128, 64, 4)
    WG(2, 128, 128, 3)
    WG(3, 64, 128, 4)
    default: return hipErrorInvalidValue;
  }
#undef WG
  return hipGetLastError();
}

}  // namespace

IIT_EXPORT int iit_conv3x3_tiles() { return kConvTiles; }
IIT_EXPORT int iit_conv3x3_wgrad_tiles() { return kWgTiles; }

// 1 when the weight-gradient kernel covers the convolution on ``tile`` with ``splits`` K-splits (reduction split:
// deterministic, the last-arriving split sums the partials): Cout % BM, Cin % BN, N H W % (64 splits) == 0
IIT_EXPORT int iit_conv3x3_wgrad_ok(long N, int H, int W, int Cin, int Cout, int tile, int splits) {
  if (tile < 0 || tile >= kWgTiles || N <= 0 || splits < 1 || Cin % 64) return 0;
  const long K = N * H * W;
  if (Cout % kWgBM[tile] || Cin % kWgBN[tile] || K % (64L * splits) || K >= (1L << 24)) return 0;
  return 1;
}

// dw [Cout][3][3][Cin] fp32 (+)= sum over pixels of dy[pix][co] x[pix shifted by the tap][ci] (``acc``: accumulate into
// dw, else store); ``splits`` > 1 needs ``ws`` (>= splits Cout 9 Cin floats) and ``counters`` (>= the tile count,
// zero when idle)
IIT_EXPORT int iit_conv3x3_wgrad(const void* dy, const void* x, float* dw, const void* zero, long N, int H, int W,
                                 int Cin, int Cout, int acc, int tile, int splits, float* ws, int* counters,
                                 void* stream) {
  if (!iit_conv3x3_wgrad_ok(N, H, W, Cin, Cout, tile, splits)) return (int)hipErrorInvalidValue;
  if (((uintptr_t)dy | (uintptr_t)x | (uintptr_t)dw | (uintptr_t)zero) & 15) return (int)hipErrorInvalidValue;
  if (splits > 1 && (!ws || !counters)) return (int)hipErrorInvalidValue;
  G2Args a{};
  a.A = (const __bf16*)dy;
  a.B = (const __bf16*)x;
  a.C = dw;
  a.lda = Cout;
  a.ldb = 9L * Cin;
  a.ldc = 9L * Cin;
  a.M = Cout;
  a.N = 9 * Cin;
  a.K = (int)(N * H * W);
  a.k_per_split = a.K / splits;
  a.ws = splits > 1 ? ws : nullptr;
  a.counters = splits > 1 ? counters : nullptr;
  a.zero = (const __bf16*)zero;
  a.conv_h = H;
  a.conv_w = W;
  a.conv_c = Cin;
  hipStream_t s = (hipStream_t)stream;
  return (int)(acc ? launch_wgrad<E_F32_ACC>(a, tile, splits, s) : launch_wgrad<E_F32_STORE>(a, tile, splits, s));
}

// 1 when the implicit-GEMM kernel covers a 3x3 / stride-1 / pad-1 convolution of [N][H][W][Cin] into Cout channels on
// ``tile`` with ``splits`` K-splits: Cin % 64 == 0 (a K-tile is one tap), Cout % BN == 0, N H W % BM == 0 (no partial
// row tiles), 9 Cin % (64 splits) == 0 (equal K ranges)
IIT_EXPORT int iit_conv3x3_ok(long N, int H, int W, int Cin, int Cout, int tile, int splits) {
  if (tile < 0 || tile >= kConvTiles || N <= 0 || H <= 0 || W <= 0 || Cin <= 0 || Cout <= 0 || splits < 1) return 0;
  const long M = N * H * W;
  if (Cin % 64 || Cout % kConvBN[tile] || M % kConvBM[tile] || M >= (1L << 31)) return 0;
  if ((9 * Cin) % (64 * splits)) return 0;
  return 1;
}

// y [N][H][W][Cout] = conv3x3(x [N][H][W][Cin], w [Cout][3][3][Cin]) (bf16, NHWC, stride 1, pad 1, no bias);
// ``flip``: the tap offsets negated (the input gradient: x = dY, w = the weight re-laid [Cin][3][3][Cout]).
// ``zero``: >= 128 zero bytes, 16-B aligned (the padding rows' LDS-DMA source).  ``splits`` > 1 needs ``ws`` (>= splits
// N H W Cout floats) and ``counters`` (>= the tile count, zero when idle; re-armed by every launch).
IIT_EXPORT int iit_conv3x3_rows(int tile) { return tile >= 0 && tile < kConvTiles ? kConvBM[tile] : 0; }

// ``cstat`` (nullable): per-tile column statistics of y for its BatchNorm, [3][Cout][N H W / BM] floats
// (gemm_glds_body.h E_BF16_CS; BM = iit_conv3x3_rows(tile))
IIT_EXPORT int iit_conv3x3(const void* x, const void* w, void* y, const void* zero, long N, int H, int W, int Cin,
                           int Cout, int flip, int tile, int splits, float* ws, int* counters, float* cstat,
                           void* stream) {
  if (!iit_conv3x3_ok(N, H, W, Cin, Cout, tile, splits)) return (int)hipErrorInvalidValue;
  if (((uintptr_t)x | (uintptr_t)w | (uintptr_t)y | (uintptr_t)zero) & 15) return (int)hipErrorInvalidValue;
  if (splits > 1 && (!ws || !counters)) return (int)hipErrorInvalidValue;
  G2Args a{};
  a.A = (const __bf16*)x;
  a.B = (const __bf16*)w;
  a.C = y;
  a.lda = 9L * Cin;
  a.ldb = 9L * Cin;
  a.ldc = Cout;
  a.M = (int)(N * H * W);
  a.N = Cout;
  a.K = 9 * Cin;
  a.k_per_split = a.K / splits;
  a.ws = splits > 1 ? ws : nullptr;
  a.counters = splits > 1 ? counters : nullptr;
  a.zero = (const __bf16*)zero;
  a.conv_h = H;
  a.conv_w = W;
  a.conv_c = Cin;
  a.conv_flip = flip;
  a.cstat = cstat;
  return (int)launch_conv_tile(a, tile, splits, (hipStream_t)stream);
}
