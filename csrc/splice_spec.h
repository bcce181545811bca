// Patch-spec range table of an interchange splice (iit_amd/ops/splice.py PatchSpec): shared by the standalone
// splice kernel (csrc/splice.hip) and the producer kernels that apply a splice in their own epilogue
// (csrc/llama_ops.hip SwiGLU).  An element of a [shape0][shape1][shape2][shape3] activation is selected iff every
// coordinate lies in one of its dimension's (up to 8) half-open ranges; ``sstride`` are the source's element strides
// (0 = broadcast).
#pragma once

struct SpliceSpec {
  int shape[4];     // row-major shape (leading dims padded with 1)
  int nr[4];        // ranges per dimension (>= 1)
  int lo[4][8];
  int hi[4][8];
  long sstride[4];  // source strides in elements (0 = broadcast)
};

__device__ __forceinline__ bool in_ranges(const SpliceSpec& sp, int d, int c) {
  bool ok = false;
#pragma unroll
  for (int r = 0; r < 8; ++r)
    if (r < sp.nr[d]) ok |= (c >= sp.lo[d][r]) & (c < sp.hi[d][r]);
  return ok;
}

// coordinates (c0, c1, c2, c3) of flat element e of the spec's shape
__device__ __forceinline__ void spec_coords(const SpliceSpec& sp, long e, int& c0, int& c1, int& c2, int& c3) {
  long q = e / sp.shape[3];
  c3 = (int)(e - q * sp.shape[3]);
  c2 = (int)(q % sp.shape[2]);
  q /= sp.shape[2];
  c1 = (int)(q % sp.shape[1]);
  c0 = (int)(q / sp.shape[1]);
}
