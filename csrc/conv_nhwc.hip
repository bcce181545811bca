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

template <int BM, int BN, int NS, int NW, int OCC>
__global__ __launch_bounds__(NW * 64, OCC) void conv3x3_kernel(G2Args p) {
  __shared__ __attribute__((aligned(16))) char smem[GldsSmem<BM, BN, NS, NW, 64, OCC>::BYTES];
  gemm_glds_body<BM, BN, NS, false, false, E_BF16, NW, 64, OCC, false, ConvRowStager<BM, NW>>(p, blockIdx.x, gridDim.x,
                                                                                              0, 1, smem);
}

template <int BM, int BN, int NS, int NW = 4, int OCC = 1>
hipError_t launch_conv(const G2Args& a, hipStream_t s) {
  const int tiles = (a.M / BM) * (a.N / BN);
  hipLaunchKernelGGL((conv3x3_kernel<BM, BN, NS, NW, OCC>), dim3(tiles), dim3(NW * 64), 0, s, a);
  return hipGetLastError();
}

// tiles (BM, BN, ring depth, waves, workgroups per CU): the output is [N H W][Cout] with Cout 64..512
constexpr int kConvTiles = 6;
const int kConvBM[kConvTiles] = {128, 128, 64, 128, 64, 128};
const int kConvBN[kConvTiles] = {64, 128, 64, 128, 128, 64};

hipError_t launch_conv_tile(const G2Args& a, int tile, hipStream_t s) {
  switch (tile) {
    case 0: return launch_conv<128, 64, 4>(a, s);
    case 1: return launch_conv<128, 128, 3>(a, s);
    case 2: return launch_conv<64, 64, 4, 4, 2>(a, s);
    case 3: return launch_conv<128, 128, 2, 4, 2>(a, s);
    case 4: return launch_conv<64, 128, 2, 4, 3>(a, s);
    case 5: return launch_conv<128, 64, 2, 4, 2>(a, s);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace

IIT_EXPORT int iit_conv3x3_tiles() { return kConvTiles; }

// 1 when the implicit-GEMM kernel covers a 3x3 / stride-1 / pad-1 convolution of [N][H][W][Cin] into Cout channels on
// ``tile``: Cin % 64 == 0 (a K-tile is one tap), Cout % BN == 0, N H W % BM == 0 (no partial row tiles)
IIT_EXPORT int iit_conv3x3_ok(long N, int H, int W, int Cin, int Cout, int tile) {
  if (tile < 0 || tile >= kConvTiles || N <= 0 || H <= 0 || W <= 0 || Cin <= 0 || Cout <= 0) return 0;
  const long M = N * H * W;
  if (Cin % 64 || Cout % kConvBN[tile] || M % kConvBM[tile] || M >= (1L << 31)) return 0;
  return 1;
}

// y [N][H][W][Cout] = conv3x3(x [N][H][W][Cin], w [Cout][3][3][Cin]) (bf16, NHWC, stride 1, pad 1, no bias);
// ``flip``: the tap offsets negated (the input gradient: x = dY, w = the weight re-laid [Cin][3][3][Cout]).
// ``zero``: >= 128 zero bytes, 16-B aligned (the padding rows' LDS-DMA source).
IIT_EXPORT int iit_conv3x3(const void* x, const void* w, void* y, const void* zero, long N, int H, int W, int Cin,
                           int Cout, int flip, int tile, void* stream) {
  if (!iit_conv3x3_ok(N, H, W, Cin, Cout, tile)) return (int)hipErrorInvalidValue;
  if (((uintptr_t)x | (uintptr_t)w | (uintptr_t)y | (uintptr_t)zero) & 15) return (int)hipErrorInvalidValue;
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
  a.k_per_split = a.K;
  a.zero = (const __bf16*)zero;
  a.conv_h = H;
  a.conv_w = W;
  a.conv_c = Cin;
  a.conv_flip = flip;
  return (int)launch_conv_tile(a, tile, (hipStream_t)stream);
}
