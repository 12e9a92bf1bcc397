// Experiment: can SHA-256 (VALU) waves co-issue beside the f64 MFMA
// contraction on the same SIMDs?  A = var-like MFMA kernel (512 threads/CU,
// 2 waves/SIMD, large LDS), B = SHA compress kernel capped to fit the
// remaining VGPRs.  Times A alone, B alone, A || B on two streams.
//   hipcc -O3 --offload-arch=gfx950 scripts/exp/coissue.hip -o scripts/exp/coissue
#include <hip/hip_runtime.h>
#include <cstdio>
#include "../../uptune_amd/csrc/ut_core.h"

typedef double vd4 __attribute__((ext_vector_type(4)));

__device__ double rnd(uint64_t x) {
  x = x * 0x9E3779B97F4A7C15ull + 12345;
  x ^= x >> 31; x *= 0xBF58476D1CE4E5B9ull; x ^= x >> 29;
  return (double)(x >> 11) * (1.0 / 9007199254740992.0) - 0.5;
}

constexpr int LDS_D = 18 * 1024;  // 144 KB of doubles
__global__ __launch_bounds__(512, 1) void k_mfma(double* out, int iters) {
  __shared__ double lds[LDS_D];
  for (int e = threadIdx.x; e < LDS_D; e += 512) lds[e] = rnd(e + 7919 * blockIdx.x);
  __syncthreads();
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, wm = w >> 1, wn = w & 1;
  vd4 acc[4][4];
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < 4; ++j) acc[i][j] = (vd4){0, 0, 0, 0};
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      const int kr = ks * 4 + (lane >> 4) + (it & 63) * 16;
      double af[4], bf[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) af[i] = lds[(kr * 144 + wm * 64 + i * 16 + (lane & 15)) % LDS_D];
#pragma unroll
      for (int j = 0; j < 4; ++j) bf[j] = lds[(kr * 144 + 72 + wn * 32 + j * 16 + (lane & 15)) % LDS_D];
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(af[i], bf[j], acc[i][j], 0, 0, 0);
    }
  }
  double s = 0;
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < 4; ++j) s += acc[i][j][0] + acc[i][j][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int WPE>
__global__ __launch_bounds__(128) __attribute__((amdgpu_waves_per_eu(WPE, 8))) void k_sha(uint32_t* out, int iters,
                                                                                         uint32_t seed) {
  __shared__ uint32_t scratch[2048];  // 8 KB, like the hash kernel's LDS staging
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  scratch[threadIdx.x] = t;
  uint32_t H[8], W[16];
  ut::sha256_init(H);
#pragma unroll
  for (int w = 0; w < 16; ++w) W[w] = t * 2654435761u + w * 97u + seed + scratch[(threadIdx.x + w) & 127];
  for (int it = 0; it < iters; ++it) {
    uint32_t X[16];
#pragma unroll
    for (int w = 0; w < 16; ++w) X[w] = W[w] ^ H[w & 7];
    ut::sha256_compress(H, X);
  }
  uint32_t acc = 0;
#pragma unroll
  for (int w = 0; w < 8; ++w) acc ^= H[w];
  out[t] = acc;
}

int main() {
  double* outd;
  uint32_t* outu;
  hipMalloc(&outd, sizeof(double) * 512 * 256);
  const int sha_lanes = 1 << 20;
  hipMalloc(&outu, sizeof(uint32_t) * sha_lanes);
  hipStream_t s1, s2;
  hipStreamCreateWithFlags(&s1, hipStreamNonBlocking);
  hipStreamCreateWithFlags(&s2, hipStreamNonBlocking);
  hipEvent_t a0, a1, b0, b1, t0, t1;
  for (hipEvent_t* e : {&a0, &a1, &b0, &b1, &t0, &t1}) hipEventCreate(e);
  const int mit = 3000, sit = 130;
  auto A = [&](hipStream_t s) { hipLaunchKernelGGL(k_mfma, dim3(256), dim3(512), 0, s, outd, mit); };
  auto B6 = [&](hipStream_t s) { hipLaunchKernelGGL(k_sha<6>, dim3(sha_lanes / 128), dim3(128), 0, s, outu, sit, 1u); };
  auto B3 = [&](hipStream_t s) { hipLaunchKernelGGL(k_sha<1>, dim3(sha_lanes / 128), dim3(128), 0, s, outu, sit, 1u); };
  const double mflops = 256.0 * 8 * mit * 64 * 2048;
  const double comps = (double)sha_lanes * sit;
  auto timed = [&](const char* name, auto f) {
    f();
    hipDeviceSynchronize();
    hipEventRecord(t0, s1);
    hipStreamWaitEvent(s2, t0, 0);
    for (int r = 0; r < 3; ++r) f();
    hipEventRecord(t1, s2);
    hipStreamWaitEvent(s1, t1, 0);
    hipEventRecord(t1, s1);
    hipEventSynchronize(t1);
    float ms;
    hipEventElapsedTime(&ms, t0, t1);
    printf("%-40s %8.3f ms per rep\n", name, ms / 3);
  };
  timed("mfma alone", [&] { A(s1); });
  timed("sha(cap) alone", [&] { B6(s2); });
  timed("sha(uncapped) alone", [&] { B3(s2); });
  timed("mfma || sha(cap)", [&] { A(s1); B6(s2); });
  timed("sha(cap) || mfma (sha first)", [&] { B6(s2); A(s1); });
  timed("mfma || sha(uncapped)", [&] { A(s1); B3(s2); });
  printf("mfma work %.1f TFLOP per rep; sha %.1f G compressions per rep\n", mflops * 1e-12, comps * 1e-9);
  return 0;
}
