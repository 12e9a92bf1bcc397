// dedup.hip -- history membership + in-batch first-occurrence dedup.
//
// Reference semantics (one SQL round trip per candidate today):
//   SearchDriver.get_configuration / has_results   driver.py:157-158,253-258
//   Configuration.get (by program, hash)           resultsdb/models.py:126-135
//   ParallelTuning.unique -> GlobalResult.get      api.py:254-280, globalmodels.py:38-45
// A candidate is a duplicate when its hash_config digest is already in the
// results history, or when an earlier candidate (smaller global index) of
// the same batch has the same digest.
//
// History: open-addressing table of 32-byte keys (linear probing, home slot
// = first digest word, which is uniformly distributed).  Batch: table of
// candidate indices; equal digests converge on one slot whose value ends as
// the minimum index (atomicMin), so the surviving index does not depend on
// scheduling.  Bound: latency/HBM (one 32-byte read per probe).
#include "ut_internal.h"

namespace ut {

__device__ __forceinline__ bool key_eq(const uint32_t* a, const uint32_t* b) {
  const uint4* x = reinterpret_cast<const uint4*>(a);
  const uint4* y = reinterpret_cast<const uint4*>(b);
  const uint4 x0 = x[0], x1 = x[1], y0 = y[0], y1 = y[1];
  return x0.x == y0.x && x0.y == y0.y && x0.z == y0.z && x0.w == y0.w && x1.x == y1.x && x1.y == y1.y &&
         x1.z == y1.z && x1.w == y1.w;
}

__global__ void k_hist_insert(uint32_t* __restrict__ keys, uint32_t* __restrict__ state, int64_t cap,
                              const uint32_t* __restrict__ dig, int64_t n) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  const uint32_t* d = dig + j * 8;
  uint64_t h = d[0] & (uint64_t)(cap - 1);
  for (int64_t probe = 0; probe < cap; ++probe) {
    if (atomicCAS(&state[h], 0u, 1u) == 0u) {
      for (int w = 0; w < 8; ++w) keys[h * 8 + w] = d[w];
      return;
    }
    h = (h + 1) & (uint64_t)(cap - 1);
  }
}

__global__ void k_batch_insert(const uint32_t* __restrict__ dig, int64_t m, int32_t* __restrict__ slots,
                               int64_t cap) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= m) return;
  const uint32_t* d = dig + i * 8;
  uint64_t h = d[0] & (uint64_t)(cap - 1);
  for (int64_t probe = 0; probe < cap; ++probe) {
    const int32_t cur = atomicCAS(&slots[h], -1, (int32_t)i);
    if (cur == -1) return;
    if (key_eq(dig + (int64_t)cur * 8, d)) {
      atomicMin(&slots[h], (int32_t)i);
      return;
    }
    h = (h + 1) & (uint64_t)(cap - 1);
  }
}

__global__ void k_dedup_mark(const uint32_t* __restrict__ dig, int64_t m, const int32_t* __restrict__ slots,
                             int64_t cap, const uint32_t* __restrict__ hkeys, const uint32_t* __restrict__ hstate,
                             int64_t hcap, uint8_t* __restrict__ dup) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= m) return;
  const uint32_t* d = dig + i * 8;
  bool is_dup = false;
  if (hcap > 0) {
    uint64_t h = d[0] & (uint64_t)(hcap - 1);
    for (int64_t probe = 0; probe < hcap; ++probe) {
      if (hstate[h] == 0u) break;
      if (key_eq(hkeys + h * 8, d)) {
        is_dup = true;
        break;
      }
      h = (h + 1) & (uint64_t)(hcap - 1);
    }
  }
  if (!is_dup) {
    uint64_t h = d[0] & (uint64_t)(cap - 1);
    for (int64_t probe = 0; probe < cap; ++probe) {
      const int32_t cur = slots[h];
      if (cur == -1) break;  // unreachable: our own insert claimed a slot on this path
      if (key_eq(dig + (int64_t)cur * 8, d)) {
        is_dup = (cur != (int32_t)i);
        break;
      }
      h = (h + 1) & (uint64_t)(cap - 1);
    }
  }
  dup[i] = is_dup ? 1 : 0;
}

// re-insert every occupied slot of an old table (capacity growth)
__global__ void k_hist_rehash(const uint32_t* __restrict__ okeys, const uint32_t* __restrict__ ostate, int64_t ocap,
                              uint32_t* __restrict__ keys, uint32_t* __restrict__ state, int64_t cap) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= ocap || ostate[j] == 0u) return;
  const uint32_t* d = okeys + j * 8;
  uint64_t h = d[0] & (uint64_t)(cap - 1);
  for (int64_t probe = 0; probe < cap; ++probe) {
    if (atomicCAS(&state[h], 0u, 1u) == 0u) {
      for (int w = 0; w < 8; ++w) keys[h * 8 + w] = d[w];
      return;
    }
    h = (h + 1) & (uint64_t)(cap - 1);
  }
}

int launch_hist_rehash(ut_ctx* c, const uint32_t* okeys, const uint32_t* ostate, int64_t ocap) {
  if (ocap <= 0) return 0;
  hipLaunchKernelGGL(k_hist_rehash, dim3(grid1(ocap, 256)), dim3(256), 0, c->stream, okeys, ostate, ocap,
                     c->hist_keys, c->hist_state, c->hist_cap);
  UT_LAUNCH_CHECK(c);
  return 0;
}

int launch_hist_insert(ut_ctx* c, const uint32_t* dig, int64_t n) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(k_hist_insert, dim3(grid1(n, 256)), dim3(256), 0, c->stream, c->hist_keys, c->hist_state,
                     c->hist_cap, dig, n);
  UT_LAUNCH_CHECK(c);
  return 0;
}

// dst[i] |= src[i] (a GA round's invalid children join its duplicates)
__global__ void k_mask_or(uint8_t* __restrict__ dst, const uint8_t* __restrict__ src, int64_t m) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < m && src[i]) dst[i] = 1;
}

int launch_mask_or(ut_ctx* c, uint8_t* dst, const uint8_t* src, int64_t m) {
  if (m <= 0) return 0;
  hipLaunchKernelGGL(k_mask_or, dim3(grid1(m, 256)), dim3(256), 0, c->stream, dst, src, m);
  UT_LAUNCH_CHECK(c);
  return 0;
}

int launch_dedup(ut_ctx* c, const uint32_t* dig, int64_t m, uint8_t* dup) {
  if (m <= 0) return 0;
  int64_t cap = 1024;
  while (cap < 2 * m) cap <<= 1;
  UT_CHECK(c, m < (int64_t)0x7FFFFFFF, UT_EINVAL, "dedup batch must be < 2^31 candidates");
  if (c->batch_cap < cap) {
    if (c->batch_slots) {
      UT_HIP(c, ut::sync_all(c));
      ut::dfree(c->batch_slots);
    }
    UT_HIP(c, ut::dmalloc((void**)&c->batch_slots, cap * sizeof(int32_t)));
    c->batch_cap = cap;
  }
  UT_HIP(c, hipMemsetAsync(c->batch_slots, 0xFF, cap * sizeof(int32_t), c->stream));
  hipLaunchKernelGGL(k_batch_insert, dim3(grid1(m, 256)), dim3(256), 0, c->stream, dig, m, c->batch_slots, cap);
  UT_LAUNCH_CHECK(c);
  hipLaunchKernelGGL(k_dedup_mark, dim3(grid1(m, 256)), dim3(256), 0, c->stream, dig, m, c->batch_slots, cap,
                     c->hist_keys, c->hist_state, c->hist_cap, dup);
  UT_LAUNCH_CHECK(c);
  return 0;
}

}  // namespace ut
