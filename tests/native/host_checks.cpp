// Host-side checks of the kernel library's pure-host entry points, built with AddressSanitizer on the host half
// only (hipcc -Xarch_host -fsanitize=address; GPU ASan is not available on this pool) and run without a GPU
// (sanitizers for the native code).  Exercises the argument validation every launch goes through
// (tile / layout / alignment rules of the LDS-DMA GEMM), the record sizes the Python side packs (optimizer spans,
// splice range tables) and the splice launcher's reading of a packed range table.
#include <cstdio>
#include <cstdint>
#include <cstring>
#include <vector>

extern "C" {
int iit_gemm_glds_ok(const void* A, const void* B, const void* C, const void* C2, const void* resid, long lda,
                     long ldb, long ldc, long ldc2, long ldr, int M, int N, int K, int mode, int epi, int bias_cols,
                     int tile, int splits, int reduce);
int iit_adam_span_size();
int iit_splice_spec_size();
int iit_shadow_desc_size();
}

static int failures = 0;
#define CHECK(c)                                                   \
  do {                                                             \
    if (!(c)) {                                                    \
      std::fprintf(stderr, "FAILED %s:%d: %s\n", __FILE__, __LINE__, #c); \
      ++failures;                                                  \
    }                                                              \
  } while (0)

int main() {
  alignas(16) static char buf[64];
  const void* p = buf;  // 16-B aligned stand-in pointers (never dereferenced by the checks)
  // every tile accepts its own multiples and rejects ragged shapes / misaligned leading dims
  const int bm[] = {128, 128, 64, 64, 128, 256, 128, 256, 96, 128, 96, 192, 96, 128, 64, 128, 96, 64, 128, 192, 192,
                    192, 128, 128, 64, 128, 96, 128, 64, 64, 64, 64};
  const int bn[] = {128, 64, 128, 64, 128, 192, 128, 128, 96, 96, 192, 96, 96, 96, 64, 96, 96, 64, 128, 192, 192, 128,
                    192, 96, 96, 128, 96, 192, 192, 96, 64, 128};
  const int ntiles = (int)(sizeof(bm) / sizeof(bm[0]));
  for (int t = 0; t < ntiles; ++t) {
    const int M = bm[t] * 4, N = bn[t] * 2, K = 512;
    const int ok = iit_gemm_glds_ok(p, p, p, nullptr, nullptr, K, N, N, 0, 0, M, N, K, 2, 0, 0, t, 1, 0);
    CHECK(ok == (t == 19 ? 0 : 1));  // tile 19 is withdrawn
    CHECK(!iit_gemm_glds_ok(p, p, p, nullptr, nullptr, K, N, N, 0, 0, M + 1, N, K, 2, 0, 0, t, 1, 0));
    CHECK(!iit_gemm_glds_ok(p, p, p, nullptr, nullptr, K + 1, N, N, 0, 0, M, N, K, 2, 0, 0, t, 1, 0));
    CHECK(!iit_gemm_glds_ok((const char*)p + 2, p, p, nullptr, nullptr, K, N, N, 0, 0, M, N, K, 2, 0, 0, t, 1, 0));
    // split-K: only accumulate (atomic) or accumulate/store (reduction) epilogues, K divisible
    CHECK(!iit_gemm_glds_ok(p, p, p, nullptr, nullptr, K, N, N, 0, 0, M, N, K, 2, 0, 0, t, 2, 0));
  }
  CHECK(!iit_gemm_glds_ok(p, p, p, nullptr, nullptr, 64, 64, 64, 0, 0, 64, 64, 64, 2, 0, 0, -1, 1, 0));
  CHECK(!iit_gemm_glds_ok(p, p, p, nullptr, nullptr, 64, 64, 64, 0, 0, 64, 64, 64, 2, 0, 0, ntiles, 1, 0));
  // record layouts the Python packers assume (iit_amd/engine/flat.py, iit_amd/ops/splice.py, hip_kernels.py)
  CHECK(iit_adam_span_size() == 24);
  CHECK(iit_splice_spec_size() == 320);
  CHECK(iit_shadow_desc_size() > 0);
  // heap round trip under ASan: a packed range table copied the way the splice launcher reads it
  std::vector<uint8_t> spec(iit_splice_spec_size(), 0);
  uint8_t copy[512];
  std::memcpy(copy, spec.data(), spec.size());
  CHECK(copy[0] == 0);
  if (failures) return 1;
  std::printf("host checks passed (%d tiles)\n", ntiles);
  return 0;
}
