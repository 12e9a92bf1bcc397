// topk.hip -- deterministic top-k: the k largest scores, ties broken by the
// smallest global candidate index, duplicates and NaN scores never selected.
// (= Python sorted(range(m), key=lambda i: (-s[i], i))[:k] over the valid
// candidates)
//
// Each 256-thread workgroup bitonic-sorts a 2048-entry chunk in LDS
// ((score, index) pairs, index -1 = invalid) and keeps its best k; passes
// repeat on the survivors until one chunk remains.  k <= 1024.
// A re-merge pass (mode 1) reads whole sorted lists of k from the pass before;
// for a power-of-two k it loads every odd list reversed, which makes the chunk
// the state of the network after its level-k stage, and starts at level 2k
// (k = 256: 30 compare-exchange phases instead of 66).
#include "ut_internal.h"

namespace ut {

constexpr int TK_CH = 2048;
constexpr int TK_NT = 256;

__device__ __forceinline__ bool better(double sa, int64_t ia, double sb, int64_t ib) {
  if (ia < 0) return false;
  if (ib < 0) return true;
  if (sa != sb) return sa > sb;
  return ia < ib;
}

// mode 0: input = raw scores (+ dup mask), index = cand_base + position
// mode 1: input = (score, index) pairs, sorted lists of k from a previous pass
// mode 2: input = (score, index) pairs in any order
template <int MODE>
__global__ __launch_bounds__(TK_NT) void k_topk_chunk(const double* __restrict__ in_s,
                                                      const int64_t* __restrict__ in_i,
                                                      const uint8_t* __restrict__ dup, int64_t count,
                                                      int64_t cand_base, int32_t k, double* __restrict__ out_s,
                                                      int64_t* __restrict__ out_i) {
  __shared__ double ss[TK_CH];
  __shared__ int64_t si[TK_CH];
  const int t = threadIdx.x;
  const int64_t base = (int64_t)blockIdx.x * TK_CH;
  // mode 1, k a power of two: the chunk holds 2048 / k sorted lists (best
  // first; invalid entries last, whole padding lists invalid)
  const bool runs = MODE == 1 && (k & (k - 1)) == 0 && k >= 2;
  for (int e = t; e < TK_CH; e += TK_NT) {
    // odd lists enter reversed: alternating best-first / worst-first runs are
    // exactly the network's state after its size-k level
    const int src = (runs && ((e / k) & 1)) ? (e / k) * k + (k - 1 - e % k) : e;
    const int64_t p = base + src;
    double s = 0.0;
    int64_t ix = -1;
    if (p < count) {
      s = in_s[p];
      if (MODE == 0) {
        ix = (dup && dup[p]) ? -1 : cand_base + p;
      } else {
        ix = in_i[p];
      }
      if (ix < 0) ix = -1;
      if (s != s) ix = -1;  // NaN never selected
    }
    ss[e] = s;
    si[e] = ix;
  }
  for (int size = runs ? 2 * k : 2; size <= TK_CH; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      __syncthreads();
      for (int q = t; q < TK_CH / 2; q += TK_NT) {
        const int lo = 2 * stride * (q / stride) + (q % stride);
        const int hi = lo + stride;
        const bool up = (lo & size) == 0;  // this run wants best first
        const double a = ss[lo], b = ss[hi];
        const int64_t ia = si[lo], ib = si[hi];
        const bool swap = up ? better(b, ib, a, ia) : better(a, ia, b, ib);
        if (swap) {
          ss[lo] = b; ss[hi] = a;
          si[lo] = ib; si[hi] = ia;
        }
      }
    }
  }
  __syncthreads();
  for (int e = t; e < k; e += TK_NT) {
    out_s[(int64_t)blockIdx.x * k + e] = ss[e];
    out_i[(int64_t)blockIdx.x * k + e] = si[e];
  }
}

// the top-k of explicit (score, index) pairs (index -1 = invalid), ties broken
// by the smallest index: the re-merge passes from the start
int topk_pairs_impl(ut_ctx* c, const double* score, const int64_t* idx, int64_t n, int32_t k, int64_t* out_idx,
                    double* out_score) {
  UT_CHECK(c, k >= 1 && k <= TK_CH / 2, UT_EINVAL, "topk: k must be in [1, 1024]");
  int64_t count = n < 1 ? 1 : n;
  int64_t chunks = (count + TK_CH - 1) / TK_CH;
  int rc;
  if ((rc = ensure(c, c->tk_score[0], (size_t)chunks * k))) return rc;
  if ((rc = ensure(c, c->tk_idx[0], (size_t)chunks * k))) return rc;
  if ((rc = ensure(c, c->tk_score[1], (size_t)chunks * k))) return rc;
  if ((rc = ensure(c, c->tk_idx[1], (size_t)chunks * k))) return rc;
  // first pass: whole network (the input is not made of sorted lists)
  hipLaunchKernelGGL(k_topk_chunk<2>, dim3((unsigned)chunks), dim3(TK_NT), 0, c->stream, score, idx, nullptr, n, 0, k,
                     c->tk_score[0].p, c->tk_idx[0].p);
  UT_LAUNCH_CHECK(c);
  int cur = 0;
  count = chunks * k;
  while (chunks > 1) {
    chunks = (count + TK_CH - 1) / TK_CH;
    hipLaunchKernelGGL(k_topk_chunk<1>, dim3((unsigned)chunks), dim3(TK_NT), 0, c->stream, c->tk_score[cur].p,
                       c->tk_idx[cur].p, nullptr, count, 0, k, c->tk_score[cur ^ 1].p, c->tk_idx[cur ^ 1].p);
    UT_LAUNCH_CHECK(c);
    cur ^= 1;
    count = chunks * k;
  }
  if (out_idx)
    UT_HIP(c, hipMemcpyAsync(out_idx, c->tk_idx[cur].p, sizeof(int64_t) * k, hipMemcpyDeviceToDevice, c->stream));
  if (out_score)
    UT_HIP(c, hipMemcpyAsync(out_score, c->tk_score[cur].p, sizeof(double) * k, hipMemcpyDeviceToDevice,
                             c->stream));
  return 0;
}

int topk_impl(ut_ctx* c, const double* score, const uint8_t* dup, int64_t m, int64_t cand_base, int32_t k,
              int64_t* out_idx, double* out_score) {
  UT_CHECK(c, k >= 1 && k <= TK_CH / 2, UT_EINVAL, "topk: k must be in [1, 1024]");
  UT_CHECK(c, m >= 0, UT_EINVAL, "topk: m < 0");
  int64_t chunks = (m + TK_CH - 1) / TK_CH;
  if (chunks < 1) chunks = 1;
  int rc;
  if ((rc = ensure(c, c->tk_score[0], (size_t)chunks * k))) return rc;
  if ((rc = ensure(c, c->tk_idx[0], (size_t)chunks * k))) return rc;
  if ((rc = ensure(c, c->tk_score[1], (size_t)chunks * k))) return rc;
  if ((rc = ensure(c, c->tk_idx[1], (size_t)chunks * k))) return rc;
  hipLaunchKernelGGL(k_topk_chunk<0>, dim3((unsigned)chunks), dim3(TK_NT), 0, c->stream, score, nullptr, dup, m,
                     cand_base, k, c->tk_score[0].p, c->tk_idx[0].p);
  UT_LAUNCH_CHECK(c);
  int cur = 0;
  int64_t count = chunks * k;
  while (chunks > 1) {
    chunks = (count + TK_CH - 1) / TK_CH;
    hipLaunchKernelGGL(k_topk_chunk<1>, dim3((unsigned)chunks), dim3(TK_NT), 0, c->stream, c->tk_score[cur].p,
                       c->tk_idx[cur].p, nullptr, count, 0, k, c->tk_score[cur ^ 1].p, c->tk_idx[cur ^ 1].p);
    UT_LAUNCH_CHECK(c);
    cur ^= 1;
    count = chunks * k;
  }
  if (out_idx)
    UT_HIP(c, hipMemcpyAsync(out_idx, c->tk_idx[cur].p, sizeof(int64_t) * k, hipMemcpyDeviceToDevice, c->stream));
  if (out_score)
    UT_HIP(c, hipMemcpyAsync(out_score, c->tk_score[cur].p, sizeof(double) * k, hipMemcpyDeviceToDevice,
                             c->stream));
  return 0;
}

}  // namespace ut
