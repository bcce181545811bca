// NHWC bf16 convolutions (kernel 1 x 1 or 3 x 3, stride 1 or 2) as implicit GEMMs on the LDS-DMA MFMA body
// (gemm_glds_body.h): the ResNet-18 BasicBlock convolutions of the PVR task's low-level model (/root/reference/iit/
// tasks/mnist_pvr/get_alignment.py:9-15, torchvision's resnet18) -- the 3 x 3 stride-1 and stride-2 convolutions and
// the 1 x 1 stride-2 downsample -- in place of MIOpen / CK.
//
//   y[n][h][w][co] = sum_{kh, kw, ci} x[n][s h + kh - pad][s w + kw - pad][ci] * W[co][kh][kw][ci]
//
// is the GEMM  Y [M = N Ho Wo][Cout] = A [M][K = k k Cin] x B^T, with B = the channels-last weight [Cout][k][k][Cin]
// read as [Cout][k k Cin] (mode 0: both operands k-contiguous) and A the implicit im2col matrix: row m = output pixel
// (n, h, w), K index = tap * Cin + ci with the taps outermost.  With Cin % 64 == 0 a 64-deep K-tile is 64 channels
// of ONE tap, i.e. for every row one 128-B segment of one source pixel: ConvRowStager gives each lane of the LDS-DMA
// (global_load_lds) the source address of its row's pixel for the tile's tap -- or the zero page when that pixel is
// outside the image (the padding) -- into exactly the swizzled LDS image the strided stager builds, so the main loop,
// the MFMA fragments and the epilogue are the GEMM's, unchanged.  No im2col buffer, no padding copy.
//
// The input gradient is the same GEMM body in transposed mode (conv_flip) on A = dY and B = the forward weight read
// k-major in place (ConvWTStager):  dx[n][h][w][ci] = sum_{kh, kw, co} dy[n][(h + pad - kh) / s][(w + pad - kw) / s][co]
// W[co][kh][kw][ci] over the taps where the division is exact (stride 2: the other taps read the zero page).
#include "gemm_glds_body.h"

namespace {

template <int R, int NW>
struct ConvRowStager {
  static constexpr int RPI = 8;  // rows per LDS-DMA instruction: 8 rows x 128 B (the k-contiguous BK = 64 image)
  static constexpr int N = R / (RPI * NW);
  static_assert(N >= 1, "tile too narrow for the workgroup's waves");
  const __bf16* x;
  const __bf16* zero;
  long nb[N];   // element offset of the lane's row's image n in the source: n * SH * SW * C
  int ph[N], pw[N];
  int cc[N];    // the lane's 16-B chunk of its row (source-side swizzle, as Stager<false, R, NW, 64>)
  int off[N];   // wave-uniform LDS offset of instruction i
  int SH, SW, C, flip, kbeg, KS, S, PAD;

  __device__ __forceinline__ void init(const G2Args& p, int r0g, int kbeg_, int wave, int lane) {
    x = p.A;
    zero = p.zero;
    SH = p.conv_sh;
    SW = p.conv_sw;
    C = p.conv_c;
    flip = p.conv_flip;
    KS = p.conv_k;
    S = p.conv_s;
    PAD = p.conv_pad;
    kbeg = kbeg_;
    const int hw = p.conv_h * p.conv_w;
#pragma unroll
    for (int i = 0; i < N; ++i) {
      const int r0 = i * RPI * NW + wave * RPI;
      const int row = r0 + lane / 8;
      const long m = (long)r0g + row;
      const int n = (int)(m / hw);
      const int rem = (int)(m - (long)n * hw);
      const int h = rem / p.conv_w;
      ph[i] = h;
      pw[i] = rem - h * p.conv_w;
      nb[i] = (long)n * SH * SW * C;
      cc[i] = ((lane & 7) ^ kcont_swz<64>(row)) * 8;
      off[i] = r0 * 128;
    }
  }

  __device__ __forceinline__ void stage(int kt, char* img) const {
    const int k0 = kbeg + kt * 64;
    const int tap = k0 / C, ci0 = k0 - tap * C;
    const int kh = KS == 1 ? 0 : tap / 3;
    const int kw = tap - kh * KS;
#pragma unroll
    for (int i = 0; i < N; ++i) {
      int hs, ws;
      bool in;
      if (!flip) {  // forward: source (s h + kh - pad, s w + kw - pad)
        hs = S * ph[i] + kh - PAD;
        ws = S * pw[i] + kw - PAD;
        in = (unsigned)hs < (unsigned)SH && (unsigned)ws < (unsigned)SW;
      } else {  // transposed (input gradient): source ((h + pad - kh) / s, (w + pad - kw) / s) where exact
        const int a = ph[i] + PAD - kh, b = pw[i] + PAD - kw;
        hs = S == 2 ? a >> 1 : a;
        ws = S == 2 ? b >> 1 : b;
        in = a >= 0 && b >= 0 && (S == 1 || ((a | b) & 1) == 0) && hs < SH && ws < SW;
      }
      glds16(in ? x + nb[i] + ((long)hs * SW + ws) * C + ci0 + cc[i] : zero + cc[i], img + off[i]);
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

// The weight gradient's B operand: dW [Cout][k k Cin] = dY^T [Cout][K = N OH OW] x im2col(x) [K][k k Cin], staged
// k-major ([64 output pixels][R columns], the image of Stager<true, R, NW, 64>): an N-tile of R columns is R channels
// [ci0, ci0 + R) of ONE tap (Cin % R == 0), so k-row ``pix`` of the tile is one contiguous 2R-byte segment of the
// source pixel (s h + kh - pad, s w + kw - pad) of output pixel ``pix`` -- or the zero page outside the image.  The tap
// is fixed per workgroup; each K-tile recomputes the lanes' pixels' (n, h, w) (the K range advances 64 pixels per
// K-tile).  Reads the activation from ``p.B``.
template <int R, int NW>
struct ConvColStager {
  static constexpr int CH = R / 8;      // 16-B chunks per k-row
  static constexpr int KRI = 64 / CH;   // k-rows per LDS-DMA instruction
  static constexpr int N = 64 / (NW * KRI);
  static_assert(N >= 1 && (R == 64 || R == 128), "64- or 128-column tiles");
  const __bf16* x;
  const __bf16* zero;
  int kr[N], col[N], off[N];
  int H, W, SH, SW, C, kh, kw, S, PAD, ci0, kbeg;
  float invW, invH;

  __device__ __forceinline__ void init(const G2Args& p, int r0g, int kbeg_, int wave, int lane) {
    x = p.B;
    zero = p.zero;
    H = p.conv_h;
    W = p.conv_w;
    SH = p.conv_sh;
    SW = p.conv_sw;
    C = p.conv_c;
    S = p.conv_s;
    PAD = p.conv_pad;
    kbeg = kbeg_;
    invW = 1.f / (float)W;
    invH = 1.f / (float)H;
    const int tap = r0g / C;
    ci0 = r0g - tap * C;
    kh = p.conv_k == 1 ? 0 : tap / 3;
    kw = tap - kh * p.conv_k;
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
      const int pix = kbeg + kt * 64 + kr[i];  // output pixel (n, h, w) = the dy row
      const int q = fdiv(pix, W, invW);
      const int w = pix - q * W;
      const int n = fdiv(q, H, invH);
      const int h = q - n * H;
      const int hs = S * h + kh - PAD, ws = S * w + kw - PAD;
      const bool in = (unsigned)hs < (unsigned)SH && (unsigned)ws < (unsigned)SW;
      glds16(in ? x + (((long)n * SH + hs) * SW + ws) * C + ci0 + col[i] : zero + col[i], img + off[i]);
    }
  }
};

// The transposed convolution's (input gradient's) B operand read straight from the FORWARD weight
// [Cout][k][k][Cin] -- no re-laid copy of the weight per backward: B [n = ci][K = tap * Cout + co] = W[co][tap][ci],
// staged k-major ([64 K rows][R columns], the image of Stager<true, R, NW, 64>): a K-tile is 64 output channels co of
// one tap (Cout % 64 == 0), so k-row r of the tile is the contiguous 2R-byte run W[co0 + r][tap][n0 .. n0 + R).
template <int R, int NW>
struct ConvWTStager {
  static constexpr int CH = R / 8;      // 16-B chunks per k-row
  static constexpr int KRI = 64 / CH;   // k-rows per LDS-DMA instruction
  static constexpr int N = 64 / (NW * KRI);
  static_assert(N >= 1 && (R == 64 || R == 128), "64- or 128-column tiles");
  const __bf16* w;
  long kkC;  // row stride of W: k k Cin
  int kr[N], col[N], off[N];
  int C, CS, n0, kbeg;

  __device__ __forceinline__ void init(const G2Args& p, int r0g, int kbeg_, int wave, int lane) {
    w = p.B;
    C = p.N;        // GEMM columns = the conv's input channels
    CS = p.conv_c;  // the source (dy) channels = the conv's output channels
    kkC = (long)p.conv_k * p.conv_k * C;
    n0 = r0g;
    kbeg = kbeg_;
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
    const int k0 = kbeg + kt * 64;
    const int tap = k0 / CS, co0 = k0 - tap * CS;
#pragma unroll
    for (int i = 0; i < N; ++i)
      glds16(w + (long)(co0 + kr[i]) * kkC + (long)tap * C + n0 + col[i], img + off[i]);
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

// the transposed convolution (input gradient): B k-major from the forward weight (ConvWTStager)
template <int BM, int BN, int NS, int NW, int OCC>
__global__ __launch_bounds__(NW * 64, OCC) void conv_t_kernel(G2Args p) {
  __shared__ __attribute__((aligned(16))) char smem[GldsSmem<BM, BN, NS, NW, 64, OCC>::BYTES];
  gemm_glds_body<BM, BN, NS, false, true, E_BF16, NW, 64, OCC, false, ConvRowStager<BM, NW>, ConvWTStager<BN, NW>>(
      p, blockIdx.x, gridDim.x, blockIdx.y, gridDim.y, smem);
}

template <int BM, int BN, int NS, int NW = 4, int OCC = 1>
hipError_t launch_conv(const G2Args& a, int splits, hipStream_t s) {
  const int tiles = (a.M / BM) * (a.N / BN);
  if (a.conv_flip == 1)  // transposed, forward weight in place; 2 = transposed on a re-laid [Cin][k][k][Cout] copy
    hipLaunchKernelGGL((conv_t_kernel<BM, BN, NS, NW, OCC>), dim3(tiles, splits), dim3(NW * 64), 0, s, a);
  else if (a.cstat)
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
IIT_EXPORT int iit_conv3x3_rows(int tile) { return tile >= 0 && tile < kConvTiles ? kConvBM[tile] : 0; }

// the forward convolution (kernel k, stride s, padding pad) maps an SH x SW image to OH x OW
static bool conv_geom_ok(long N, int SH, int SW, int OH, int OW, int k, int s, int pad) {
  if (N <= 0 || SH <= 0 || SW <= 0 || OH <= 0 || OW <= 0) return false;
  if (!(k == 1 || k == 3) || !(s == 1 || s == 2) || pad < 0 || pad > 1) return false;
  return OH == (SH + 2 * pad - k) / s + 1 && OW == (SW + 2 * pad - k) / s + 1;
}

// 1 when the implicit-GEMM kernel covers the convolution on ``tile`` with ``splits`` K-splits.  Forward: source x
// [N][SH][SW][Cs] -> y [N][OH][OW][Co]; transposed (the input gradient of a forward conv from [OH][OW][Co] to
// [SH][SW][Cs]): source dy [N][SH][SW][Cs] -> dx [N][OH][OW][Co].  Cs % 64 == 0 (a K-tile is one tap), Co % BN == 0,
// N OH OW % BM == 0 (no partial row tiles), k k Cs % (64 splits) == 0 (equal K ranges)
IIT_EXPORT int iit_conv2d_ok(long N, int SH, int SW, int Cs, int OH, int OW, int Co, int k, int s, int pad,
                             int transposed, int tile, int splits) {
  if (tile < 0 || tile >= kConvTiles || Cs <= 0 || Co <= 0 || splits < 1) return 0;
  if (transposed ? !conv_geom_ok(N, OH, OW, SH, SW, k, s, pad) : !conv_geom_ok(N, SH, SW, OH, OW, k, s, pad)) return 0;
  const long M = N * OH * OW;
  if (Cs % 64 || Co % kConvBN[tile] || M % kConvBM[tile] || M >= (1L << 31)) return 0;
  if ((k * k * Cs) % (64 * splits)) return 0;
  return 1;
}

// y = conv(x, w) (forward: w [Co][k][k][Cs]) or the transposed convolution: ``transposed`` 1 = w is the FORWARD
// weight [Cs = Cout][k][k][Co = Cin], read k-major in place; 2 = w re-laid [Co = Cin][k][k][Cs = Cout] (k-contiguous:
// faster per call, but the caller pays a copy);
// bf16 NHWC, no bias.  ``zero``: >= 128 zero bytes, 16-B aligned.  ``splits`` > 1 needs ``ws`` (>= splits N OH OW Co
// floats) and ``counters`` (>= the tile count, zero when idle; re-armed by every launch).  ``cstat`` (nullable):
// per-tile column statistics of y for its BatchNorm, [3][Co][N OH OW / BM] floats (gemm_glds_body.h E_BF16_CS).
IIT_EXPORT int iit_conv2d(const void* x, const void* w, void* y, const void* zero, long N, int SH, int SW, int Cs,
                          int OH, int OW, int Co, int k, int s, int pad, int transposed, int tile, int splits,
                          float* ws, int* counters, float* cstat, void* stream) {
  if (transposed < 0 || transposed > 2 || !iit_conv2d_ok(N, SH, SW, Cs, OH, OW, Co, k, s, pad, transposed, tile, splits))
    return (int)hipErrorInvalidValue;
  if (((uintptr_t)x | (uintptr_t)w | (uintptr_t)y | (uintptr_t)zero) & 15) return (int)hipErrorInvalidValue;
  if (splits > 1 && (!ws || !counters)) return (int)hipErrorInvalidValue;
  G2Args a{};
  a.A = (const __bf16*)x;
  a.B = (const __bf16*)w;
  a.C = y;
  a.lda = (long)k * k * Cs;
  a.ldb = (long)k * k * Cs;
  a.ldc = Co;
  a.M = (int)(N * OH * OW);
  a.N = Co;
  a.K = k * k * Cs;
  a.k_per_split = a.K / splits;
  a.ws = splits > 1 ? ws : nullptr;
  a.counters = splits > 1 ? counters : nullptr;
  a.zero = (const __bf16*)zero;
  a.conv_h = OH;
  a.conv_w = OW;
  a.conv_sh = SH;
  a.conv_sw = SW;
  a.conv_c = Cs;
  a.conv_k = k;
  a.conv_s = s;
  a.conv_pad = pad;
  a.conv_flip = transposed;
  a.cstat = cstat;
  return (int)launch_conv_tile(a, tile, splits, (hipStream_t)stream);
}

// 1 when the weight-gradient kernel covers the convolution x [N][SH][SW][Cin] -> dy [N][OH][OW][Cout] on ``tile``
// with ``splits`` K-splits (reduction split: deterministic, the last-arriving split sums the partials): Cout % BM,
// Cin % BN, N OH OW % (64 splits) == 0
IIT_EXPORT int iit_conv2d_wgrad_ok(long N, int SH, int SW, int Cin, int OH, int OW, int Cout, int k, int s, int pad,
                                   int tile, int splits) {
  if (tile < 0 || tile >= kWgTiles || splits < 1 || Cin % 64 || !conv_geom_ok(N, SH, SW, OH, OW, k, s, pad)) return 0;
  const long K = N * OH * OW;
  if (Cout % kWgBM[tile] || Cin % kWgBN[tile] || K % (64L * splits) || K >= (1L << 24)) return 0;
  return 1;
}

// dw [Cout][k][k][Cin] fp32 (+)= sum over output pixels of dy[pix][co] x[source of pix for the tap][ci] (``acc``:
// accumulate into dw, else store); ``splits`` > 1 needs ``ws`` (>= splits Cout k k Cin floats) and ``counters``
IIT_EXPORT int iit_conv2d_wgrad(const void* dy, const void* x, float* dw, const void* zero, long N, int SH, int SW,
                                int Cin, int OH, int OW, int Cout, int k, int s, int pad, int acc, int tile,
                                int splits, float* ws, int* counters, void* stream) {
  if (!iit_conv2d_wgrad_ok(N, SH, SW, Cin, OH, OW, Cout, k, s, pad, tile, splits)) return (int)hipErrorInvalidValue;
  if (((uintptr_t)dy | (uintptr_t)x | (uintptr_t)dw | (uintptr_t)zero) & 15) return (int)hipErrorInvalidValue;
  if (splits > 1 && (!ws || !counters)) return (int)hipErrorInvalidValue;
  G2Args a{};
  a.A = (const __bf16*)dy;
  a.B = (const __bf16*)x;
  a.C = dw;
  a.lda = Cout;
  a.ldb = (long)k * k * Cin;
  a.ldc = (long)k * k * Cin;
  a.M = Cout;
  a.N = k * k * Cin;
  a.K = (int)(N * OH * OW);
  a.k_per_split = a.K / splits;
  a.ws = splits > 1 ? ws : nullptr;
  a.counters = splits > 1 ? counters : nullptr;
  a.zero = (const __bf16*)zero;
  a.conv_h = OH;
  a.conv_w = OW;
  a.conv_sh = SH;
  a.conv_sw = SW;
  a.conv_c = Cin;
  a.conv_k = k;
  a.conv_s = s;
  a.conv_pad = pad;
  hipStream_t st = (hipStream_t)stream;
  return (int)(acc ? launch_wgrad<E_F32_ACC>(a, tile, splits, st) : launch_wgrad<E_F32_STORE>(a, tile, splits, st));
}

// the 3 x 3 / stride-1 / pad-1 entry points (same image size in and out)
IIT_EXPORT int iit_conv3x3_ok(long N, int H, int W, int Cin, int Cout, int tile, int splits) {
  return iit_conv2d_ok(N, H, W, Cin, H, W, Cout, 3, 1, 1, 0, tile, splits);
}

IIT_EXPORT int iit_conv3x3(const void* x, const void* w, void* y, const void* zero, long N, int H, int W, int Cin,
                           int Cout, int flip, int tile, int splits, float* ws, int* counters, float* cstat,
                           void* stream) {
  return iit_conv2d(x, w, y, zero, N, H, W, Cin, H, W, Cout, 3, 1, 1, flip, tile, splits, ws, counters, cstat, stream);
}

IIT_EXPORT int iit_conv3x3_wgrad_ok(long N, int H, int W, int Cin, int Cout, int tile, int splits) {
  return iit_conv2d_wgrad_ok(N, H, W, Cin, H, W, Cout, 3, 1, 1, tile, splits);
}

IIT_EXPORT int iit_conv3x3_wgrad(const void* dy, const void* x, float* dw, const void* zero, long N, int H, int W,
                                 int Cin, int Cout, int acc, int tile, int splits, float* ws, int* counters,
                                 void* stream) {
  return iit_conv2d_wgrad(dy, x, dw, zero, N, H, W, Cin, H, W, Cout, 3, 1, 1, acc, tile, splits, ws, counters, stream);
}
