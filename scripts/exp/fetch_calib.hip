// Round 6: calibrate rocprofv3 FETCH_SIZE for k_de's access widths
// (MI355X_MICROARCH.md §HBM: FETCH_SIZE reports 1/2 of a 16-B/lane streaming
// read; "other access widths are uncalibrated").  Known byte counts:
//   k_rd8   one double per lane, lanes consecutive (k_de's target reads), 1 GiB
//   k_rd16  16 B per lane, lanes consecutive, 1 GiB
//   k_gl16  global_load_lds 16 B per lane of random 512-B rows (k_de's AOS
//           donor gathers: 8 lanes per 128-B line), 2^21 rows = 1 GiB
// Run: rocprofv3 --kernel-trace --pmc FETCH_SIZE -- ./fetch_calib ; compare
// FETCH_SIZE x 1024 with the bytes each kernel reads.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 scripts/exp/fetch_calib.hip -o scripts/exp/fetch_calib
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <vector>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      return 1;                                                                \
    }                                                                          \
  } while (0)

__global__ void k_rd8(const double* __restrict__ a, int64_t n, double* __restrict__ out) {
  double s = 0.0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    s += a[i];
  if (s == 12345.678) out[0] = s;
}

__global__ void k_rd16(const double2* __restrict__ a, int64_t n, double* __restrict__ out) {
  double s = 0.0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const double2 v = a[i];
    s += v.x + v.y;
  }
  if (s == 12345.678) out[0] = s;
}

// each wave gathers 2 random 512-B rows per instruction (lanes 0-31: row A, 32-63: row B)
__global__ __launch_bounds__(256) void k_gl16(const double* __restrict__ rows, const uint32_t* __restrict__ pick,
                                              int64_t npick, double* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) double buf[4][128];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  double s = 0.0;
  for (int64_t p = ((int64_t)blockIdx.x * 4 + w) * 2; p < npick; p += (int64_t)gridDim.x * 8) {
    const uint32_t r = pick[p + (lane >> 5)];
    const double* src = rows + (int64_t)r * 64 + (lane & 31) * 2;
    __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)buf[w], 16, 0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    s += buf[w][lane];
  }
  if (s == 12345.678) out[0] = s;
}

int main() {
  const int64_t n8 = (int64_t)1 << 27;   // 1 GiB of doubles
  double *a, *out;
  uint32_t* pick;
  CK(hipMalloc(&a, n8 * 8));
  CK(hipMalloc(&out, 64));
  CK(hipMemset(a, 0, n8 * 8));
  const int64_t nrows = n8 / 64;   // 512-B rows in the same buffer
  const int64_t npick = (int64_t)1 << 21;
  std::vector<uint32_t> hp(npick);
  uint64_t x = 88172645463325252ull;
  for (auto& v : hp) {
    x ^= x << 13; x ^= x >> 7; x ^= x << 17;
    v = (uint32_t)(x % (uint64_t)nrows);
  }
  CK(hipMalloc(&pick, npick * 4));
  CK(hipMemcpy(pick, hp.data(), npick * 4, hipMemcpyHostToDevice));
  for (int rep = 0; rep < 2; ++rep) {
    hipLaunchKernelGGL(k_rd8, dim3(4096), dim3(256), 0, 0, a, n8, out);
    hipLaunchKernelGGL(k_rd16, dim3(4096), dim3(256), 0, 0, reinterpret_cast<const double2*>(a), n8 / 2, out);
    hipLaunchKernelGGL(k_gl16, dim3(4096), dim3(256), 0, 0, a, pick, npick, out);
  }
  CK(hipDeviceSynchronize());
  printf("bytes read: k_rd8 %lld, k_rd16 %lld, k_gl16 %lld (+ %lld of row indices)\n", (long long)(n8 * 8),
         (long long)(n8 * 8), (long long)(npick * 512), (long long)(npick * 4));
  return 0;
}
