// The IOI high-level causal model's intervened label in one launch (IIT target of IOI_ModelPair).
//
// IOI_HL (/root/reference/iit/tasks/ioi/ioi_hl.py:16-130; iit_amd/tasks/ioi/ioi_hl.py) is a chain of tiny tensor ops:
//   duplicate[i]    = latest j < i with tokens[j] == tokens[i], else -1
//   s_inhibition[i] = duplicate[i] == -1 ? -1 : tokens[i]
//   logits[v]       = sum_i 10 * is_name(tokens[i]) * [v == tokens[i]]  -  15 * [s_inh[i] != -1] * [v == s_inh[i]]
// (last position only: the name mover's cumulative sum at S-1), and the IIT label is argmax_v logits (first maximal
// index).  An interchange intervention replaces one node's value by the source run's: the input tokens
// (all_nodes_hook), duplicate, s_inhibition or the name-mover output.  As torch ops that is ~25 launches per
// intervention (two HL forwards of 10-12 kernels, a [B, 50257] fp32 fill and an argmax over it); here one thread
// per sequence computes the intervened label directly from the <= 2S touched vocabulary entries:
//   max over touched values > 0  -> the smallest touched index holding it;
//   otherwise the max is 0 (an untouched index exists: V > 2S) -> the smallest index whose value is 0, i.e. the
//   smallest untouched index or a smaller touched index whose entries cancel to 0.
// All sums are of +10 / -15, exact in fp32, so the label equals torch.argmax of the dense logits bit for bit.
#include "common.h"

namespace {

constexpr int MAXS = 64;

__device__ void duplicates(const long* t, int S, int* dup) {
  for (int i = 0; i < S; ++i) {
    int d = -1;
    for (int j = 0; j < i; ++j)
      if (t[j] == t[i]) d = j;  // the latest earlier position
    dup[i] = d;
  }
}

// node: 0 = all_nodes_hook (tokens), 1 = hook_duplicate, 2 = hook_s_inhibition, 3 = hook_name_mover
__global__ __launch_bounds__(256) void ioi_hl_label_kernel(const long* __restrict__ base, const long* __restrict__ src,
                                                           const float* __restrict__ name_table, int table_n, int B,
                                                           int S, int V, int node, long* __restrict__ label) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  const long* tb = base + (long)b * S;
  const long* ts = src + (long)b * S;
  // the run whose tokens feed the downstream heads: the source for an input-token or name-mover interchange
  // (the name mover's output is the source's), the base otherwise
  const long* tok = (node == 0 || node == 3) ? ts : tb;
  int dup[MAXS];
  duplicates(node == 1 ? ts : tok, S, dup);  // hook_duplicate interchange: the source's duplicate positions
  long inh[MAXS];
  if (node == 2) {  // hook_s_inhibition interchange: the source's s_inhibition values
    int dsrc[MAXS];
    duplicates(ts, S, dsrc);
    for (int i = 0; i < S; ++i) inh[i] = dsrc[i] == -1 ? -1 : ts[i];
  } else {
    for (int i = 0; i < S; ++i) inh[i] = dup[i] == -1 ? -1 : tok[i];
  }
  // touched vocabulary entries and their summed values
  long key[2 * MAXS];
  float val[2 * MAXS];
  int n = 0;
  for (int i = 0; i < 2 * S; ++i) {
    long v;
    float d;
    if (i < S) {
      v = tok[i];
      d = (v >= 0 && v < table_n && name_table[v] != 0.f) ? 10.f : 0.f;
    } else {
      const long s = inh[i - S];
      v = s != -1 ? s : (long)(V - 1);
      d = s != -1 ? -15.f : 0.f;
    }
    int k = 0;
    while (k < n && key[k] != v) ++k;
    if (k == n) {
      key[n] = v;
      val[n] = 0.f;
      ++n;
    }
    val[k] += d;
  }
  float best = -INFINITY;
  for (int k = 0; k < n; ++k) best = fmaxf(best, val[k]);
  long out = -1;
  if (best > 0.f) {
    for (int k = 0; k < n; ++k)
      if (val[k] == best && (out < 0 || key[k] < out)) out = key[k];
  } else {
    // max is 0: the smallest untouched index, unless a smaller touched index sums to exactly 0
    long u = 0;
    for (;;) {
      bool hit = false;
      for (int k = 0; k < n; ++k) hit |= key[k] == u;
      if (!hit) break;
      ++u;
    }
    out = u;
    for (int k = 0; k < n; ++k)
      if (val[k] == 0.f && key[k] < out) out = key[k];
  }
  label[b] = out;
}

}  // namespace

IIT_EXPORT int iit_ioi_hl_label(const void* base, const void* src, const float* name_table, int table_n, int B, int S,
                                int V, int node, void* label, void* stream) {
  if (S < 1 || S > MAXS || node < 0 || node > 3 || V <= 2 * S) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(ioi_hl_label_kernel, dim3((B + 255) / 256), dim3(256), 0, (hipStream_t)stream,
                     (const long*)base, (const long*)src, name_table, table_n, B, S, V, node, (long*)label);
  return hipGetLastError();
}
