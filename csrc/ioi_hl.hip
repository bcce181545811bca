// The IOI high-level causal model's intervened label in one launch (IIT target of IOI_ModelPair).
//
// IOI_HL (/root/reference/iit/tasks/ioi/ioi_hl.py:16-130; iit_amd/tasks/ioi/ioi_hl.py) is a chain of tiny tensor ops:
//   duplicate[i]    = latest j < i with tokens[j] == tokens[i], else -1
//   s_inhibition[i] = duplicate[i] == -1 ? -1 : tokens[i]
//   logits[v]       = sum_i 10 * is_name(tokens[i]) * [v == tokens[i]]  -  15 * [s_inh[i] != -1] * [v == s_inh[i]]
// (last position only: the name mover's cumulative sum at S-1), and the IIT label is argmax_v logits (first maximal
// index).  An interchange intervention replaces one node's value by the source run's: the input tokens
// (all_nodes_hook), duplicate, s_inhibition or the name-mover output.  As torch ops that is ~25 launches per
// intervention (two HL forwards of 10-12 kernels, a [B, 50257] fp32 fill and an argmax over it); here one wave
// per sequence computes the intervened label directly from the <= 2S touched vocabulary entries:
//   max over touched values > 0  -> the smallest touched index holding it;
//   otherwise the max is 0 (an untouched index exists: V > 2S) -> the smallest index whose value is 0, i.e. the
//   smallest untouched index or a smaller touched index whose entries cancel to 0.
// All sums are of +10 / -15, exact in fp32, so the label equals torch.argmax of the dense logits bit for bit.
#include "common.h"

namespace {

constexpr int MAXS = 64;

// One wave per sequence, lane i owns position i (and touched entry i / i + S): the duplicate scan, the entry sums and
// the argmax are wave-parallel over LDS (a thread-per-sequence version kept its per-position arrays in scratch memory
// and took ~80 us for 256 sequences).
// node: 0 = all_nodes_hook (tokens), 1 = hook_duplicate, 2 = hook_s_inhibition, 3 = hook_name_mover
__global__ __launch_bounds__(64) void ioi_hl_label_kernel(const long* __restrict__ base, const long* __restrict__ src,
                                                          const float* __restrict__ name_table, int table_n, int B,
                                                          int S, int V, int node, long* __restrict__ label) {
  __shared__ long tok_s[MAXS], dtok_s[MAXS], key_s[2 * MAXS];
  __shared__ float d_s[2 * MAXS];
  const int b = blockIdx.x, lane = threadIdx.x;
  const long* tb = base + (long)b * S;
  const long* ts = src + (long)b * S;
  // the run whose tokens feed the downstream heads: the source for an input-token or name-mover interchange
  // (the name mover's output is the source's), the base otherwise; the duplicate / s-inhibition values come from
  // the source for those interchanges
  const long* tok = (node == 0 || node == 3) ? ts : tb;
  const long* dtok = (node == 1 || node == 2) ? ts : tok;
  if (lane < S) {
    tok_s[lane] = tok[lane];
    dtok_s[lane] = dtok[lane];
  }
  __syncthreads();
  if (lane < S) {
    int dup = -1;  // the latest earlier position holding the same token (of the duplicate-source run)
    for (int j = 0; j < lane; ++j)
      if (dtok_s[j] == dtok_s[lane]) dup = j;
    // s_inhibition value: the duplicated token; node 1 takes the source's duplicate positions with the base's
    // tokens, node 2 the source's s_inhibition values, others their own run's
    const long inh = dup == -1 ? -1 : (node == 1 ? tok_s[lane] : dtok_s[lane]);
    const long v = tok_s[lane];
    key_s[lane] = v;
    d_s[lane] = (v >= 0 && v < table_n && name_table[v] != 0.f) ? 10.f : 0.f;
    key_s[S + lane] = inh != -1 ? inh : (long)(V - 1);
    d_s[S + lane] = inh != -1 ? -15.f : 0.f;
  }
  __syncthreads();
  // per entry: the summed value of its key (entries sharing a key all see the same sum)
  const int n = 2 * S;
  float my_val = -INFINITY, my_zero_key = INFINITY;
  long my_key = -1;
  for (int e = lane; e < n; e += 64) {
    const long k = key_s[e];
    float sum = 0.f;
    for (int f = 0; f < n; ++f)
      if (key_s[f] == k) sum += d_s[f];
    if (sum > my_val || (sum == my_val && k < my_key)) {
      my_val = sum;
      my_key = k;
    }
    if (sum == 0.f) my_zero_key = fminf(my_zero_key, (float)k);
  }
  // the smallest untouched index: candidates 0 .. n (at most n keys, so one of the n + 1 is untouched)
  float untouched = INFINITY;
  for (int u = lane; u <= n; u += 64) {
    bool hit = false;
    for (int f = 0; f < n; ++f) hit |= key_s[f] == (long)u;
    if (!hit) untouched = fminf(untouched, (float)u);
  }
  // wave reductions: max value (ties -> smallest key), min zero-sum key, min untouched index
  for (int off = 32; off > 0; off >>= 1) {
    const float ov = __shfl_xor(my_val, off);
    const long ok = __shfl_xor(my_key, off);
    if (ov > my_val || (ov == my_val && ok >= 0 && (my_key < 0 || ok < my_key))) {
      my_val = ov;
      my_key = ok;
    }
    my_zero_key = fminf(my_zero_key, __shfl_xor(my_zero_key, off));
    untouched = fminf(untouched, __shfl_xor(untouched, off));
  }
  if (lane == 0) {
    long out;
    if (my_val > 0.f) {
      out = my_key;
    } else {  // max is 0: the smallest untouched index, unless a smaller touched index sums to exactly 0
      out = (long)untouched;
      if (my_zero_key < untouched) out = (long)my_zero_key;
    }
    label[b] = out;
  }
}

}  // namespace

IIT_EXPORT int iit_ioi_hl_label(const void* base, const void* src, const float* name_table, int table_n, int B, int S,
                                int V, int node, void* label, void* stream) {
  if (S < 1 || S > MAXS || node < 0 || node > 3 || V <= 2 * S) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(ioi_hl_label_kernel, dim3(B), dim3(64), 0, (hipStream_t)stream,
                     (const long*)base, (const long*)src, name_table, table_n, B, S, V, node, (long*)label);
  return hipGetLastError();
}
