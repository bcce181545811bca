// 256 x 256 x 64 LDS-DMA GEMM with FOUR waves (2 x 2, a 128 x 128 output block each) on v_mfma_f32_32x32x16_bf16,
// one workgroup per CU -- the large-problem GEMM (Llama-3-8B projections, 8192-row paired forwards), served as
// LDS-DMA tile 41 by gemm_glds.hip.  Same operand layouts / epilogues / C ABI as the other LDS-DMA kernels:
//   mode 0  A [M][K], B [N][K];  mode 2  A [M][K], B [K][N];  mode 3  A [K][M], B [K][N]
//
// Why four waves with 128 x 128 each (cdna_hip_programming.md §3, §5): per K-tile a wave reads 32 KiB of operand
// fragments for 128 x 128 x 64 of MFMA work -- half the LDS bytes per flop of the 8-wave 128 x 64 wave tiles
// (gemm_8ph.hip) -- and one wave per SIMD owns the matrix pipe, so no partner wave competes for it.  The 16 x 256
// fp32 accumulators per lane live in the AGPR half of the unified register file (this file is built WITHOUT
// -amdgpu-mfma-vgpr-form); the 32x32x16 shape keeps the operand double buffer at 2 x 8 fragments = 64 VGPRs.
//
// Pipeline per K-tile t (four 16-deep k-steps): the fragments of k-step s + 1 are read while the 16 MFMAs of
// k-step s run (register double buffer; an explicit lgkmcnt(0) before each k-step: hipcc does not track the
// inline-asm LDS reads, and by then the reads have had 16 MFMAs = 512 cycles to land); at the
// K-tile boundary every wave retires its reads, waits for K-tile t + 1's LDS-DMA (vmcnt), one raw s_barrier, then
// re-stages the slot t just released with K-tile t + 2 (two-slot LDS-DMA ring, 128 KiB).
//
// LDS images (lane-linear per wave, XOR-swizzled through the source address: gemm_glds_body.h Stager / kcont_swz /
// kmaj_swz, unchanged): k-contiguous operands [256][64] with 16-B chunk c of row r at slot c ^ ((r >> 1) & 7) --
// a 32x32x16 fragment (32 rows, 2 chunks) then touches 16 distinct 16-B slots per ds_read_b128 lane group
// (conflict-free); k-major operands [64][256] as four 64-column panels read with ds_read_b64_tr_b16.
#include "gemm_w4.h"

namespace {

template <bool AKM, bool BKM, int EPI, int BK>
__global__ __launch_bounds__(W4_NT, 1) void gemm_4w_kernel(G2Args p) {
  __shared__ __attribute__((aligned(16))) char smem[W4_BYTES];  // ONE LDS object (see gemm_glds.hip)
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const int tiles_n = p.N / W4_BN;
  const int t = xcd_remap(blockIdx.x, gridDim.x);
  int tm, tn;
  grouped_tile(t, p.M / W4_BM, tiles_n, tm, tn, p.group_m > 0 ? p.group_m : 8);
  const int m0 = tm * W4_BM, n0 = tn * W4_BN;

  // accumulators: 4 x 4 blocks of 32 x 32 per wave, the TRANSPOSED block (B as the MFMA's first operand): lane l
  // holds row l & 31 of the C block and columns 8 (r >> 2) + 4 (l >> 5) + (r & 3) in register r -- runs of 4
  // consecutive columns, one 16-B LDS write each in the epilogue
  f32x16 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  constexpr bool CS = AKM && BKM && (EPI == E_F32_ACC || EPI == E_F32_STORE);
  const bool do_cs = CS && p.bsum != nullptr && tm == 0 && wm == 0;
  float cs[4] = {0.f, 0.f, 0.f, 0.f};
  w4_tile_loop<AKM, BKM, EPI, BK>(p, m0, n0, 0, p.K / BK, smem, acc, do_cs, cs);
  if constexpr (CS) {
    if (do_cs) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float v = cs[j] + __shfl_xor(cs[j], 32);
        if (lane < 32) atomicAdd(p.bsum + n0 + wn * 128 + j * 32 + lane, v);
      }
    }
  }
  // epilogue: chunk ch = the 128 rows of wave row wm = ch
  glds_epilogue<W4_BM, W4_BN, EPI, W4_NT, W4_ECH, W4_EPS>(p, smem, m0, n0, blockIdx.x, [&](float* E, int ch) {
    if (wm != ch) return;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int g4 = 0; g4 < 4; ++g4) {
          const int row = i * 32 + (lane & 31);
          const int col = wn * 128 + j * 32 + 8 * g4 + 4 * (lane >> 5);
          *(f32x4*)(E + row * W4_EPS + col) =
              f32x4{acc[i][j][4 * g4], acc[i][j][4 * g4 + 1], acc[i][j][4 * g4 + 2], acc[i][j][4 * g4 + 3]};
        }
  });
}

template <bool AKM, bool BKM, int EPI>
hipError_t launch_4w(const G2Args& a, int bk, hipStream_t s) {
  const dim3 grid((a.M / W4_BM) * (a.N / W4_BN));
  if (bk == 32) hipLaunchKernelGGL((gemm_4w_kernel<AKM, BKM, EPI, 32>), grid, dim3(W4_NT), 0, s, a);
  else hipLaunchKernelGGL((gemm_4w_kernel<AKM, BKM, EPI, 64>), grid, dim3(W4_NT), 0, s, a);
  return hipGetLastError();
}

}  // namespace

// launch on a G2Args filled and validated by iit_gemm_glds_sm (gemm_glds.hip), passed as its bytes; ``bk`` = the
// K-tile depth (64: tile 41, 32: tile 42)
IIT_EXPORT int iit_gemm_4w_run(const void* args, int mode, int epi, int bk, void* stream) {
  const G2Args& a = *(const G2Args*)args;
  hipStream_t s = (hipStream_t)stream;
#define W4(MODE, AK, BK_, EPI) \
  if (mode == (MODE) && epi == (EPI)) return (int)launch_4w<AK, BK_, EPI>(a, bk, s);
  W4(0, false, false, E_BF16)
  W4(0, false, false, E_F32_ACC)
  W4(0, false, false, E_F32_STORE)
  W4(0, false, false, E_DGELU)
  W4(0, false, false, E_DGELU_ERF)
  W4(2, false, true, E_BF16)
  W4(2, false, true, E_BF16_BIAS3)
  W4(2, false, true, E_F32_RESID)
  W4(2, false, true, E_GELU)
  W4(2, false, true, E_GELU_ERF)
  W4(2, false, true, E_F32_ACC)
  W4(2, false, true, E_F32_STORE)
  W4(3, true, true, E_F32_ACC)
  W4(3, true, true, E_F32_STORE)
#undef W4
  return (int)hipErrorInvalidValue;
}
