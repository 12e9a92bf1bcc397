// Experiment: what the f64 MFMA pipe sustains on MI355X.
//  (1) register-only: 16 independent 16x16x4 accumulators, W waves per SIMD
//  (2) LDS-fed: the var GEMM inner loop (8 ds_read_b64 per 16 MFMA) over a fixed
//      LDS tile, no global traffic, 2 waves per SIMD
//   hipcc -O3 --offload-arch=gfx950 scripts/exp/mfma_f64_ceiling.hip -o scripts/exp/mfma_f64_ceiling
#include <hip/hip_runtime.h>
#include <cstdio>
#include <algorithm>
#include <vector>

typedef double vd4 __attribute__((ext_vector_type(4)));

template <int NACC>
__global__ __launch_bounds__(256) void k_reg(double* out, int iters, double seed) {
  vd4 acc[NACC];
  for (int i = 0; i < NACC; ++i) acc[i] = (vd4){0, 0, 0, 0};
  double a = seed + threadIdx.x * 1e-3, b = seed - threadIdx.x * 1e-3;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < NACC; ++i) acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[i], 0, 0, 0);
  }
  double s = 0;
  for (int i = 0; i < NACC; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__device__ double rnd(uint64_t x) {
  x = x * 0x9E3779B97F4A7C15ull + 12345;
  x ^= x >> 31; x *= 0xBF58476D1CE4E5B9ull; x ^= x >> 29;
  return (double)(x >> 11) * (1.0 / 9007199254740992.0) - 0.5;
}
__global__ __launch_bounds__(256, 2) void k_lds(double* out, int iters, int mode, unsigned long long* clk) {
  __shared__ double as[16 * 144], bs[16 * 144];
  for (int e = threadIdx.x; e < 16 * 144; e += 256) {
    if (mode == 0) {
      as[e] = 1e-3 * (e % 97);
      bs[e] = 1e-3 * (e % 89);
    } else if (mode == 1) {
      as[e] = rnd(e + 7919 * blockIdx.x);
      bs[e] = rnd(e + 104729 + 7919 * blockIdx.x);
    } else {
      as[e] = 0.0;
      bs[e] = 0.0;
    }
  }
  unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  __syncthreads();
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, wm = w >> 1, wn = w & 1;
  vd4 acc[4][4];
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < 4; ++j) acc[i][j] = (vd4){0, 0, 0, 0};
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      const int kr = ks * 4 + (lane >> 4);
      double af[4], bf[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) af[i] = as[kr * 144 + wm * 64 + i * 16 + (lane & 15)];
#pragma unroll
      for (int j = 0; j < 4; ++j) bf[j] = bs[kr * 144 + wn * 64 + j * 16 + (lane & 15)];
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(af[i], bf[j], acc[i][j], 0, 0, 0);
    }
    __syncthreads();
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0) { clk[2 * blockIdx.x] = t1 - t0; clk[2 * blockIdx.x + 1] = r1 - r0; }
  double s = 0;
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < 4; ++j) s += acc[i][j][0] + acc[i][j][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

int main() {
  double* out;
  hipMalloc(&out, sizeof(double) * 2048 * 256);
  unsigned long long* clk;
  hipMalloc(&clk, sizeof(unsigned long long) * 4096);
  auto clock_report = [&](int blocks) {
    std::vector<unsigned long long> h(2 * blocks);
    hipMemcpy(h.data(), clk, sizeof(unsigned long long) * 2 * blocks, hipMemcpyDeviceToHost);
    std::vector<double> g;
    for (int b = 0; b < blocks; ++b) g.push_back((double)h[2 * b] / (double)h[2 * b + 1] * 0.1);
    std::sort(g.begin(), g.end());
    printf("    in-kernel clock median %.2f GHz (min %.2f max %.2f)\n", g[g.size() / 2], g.front(), g.back());
  };
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  auto run = [&](const char* name, int blocks, int iters, double mfma_per_wave_iter, auto launch) {
    launch();
    hipDeviceSynchronize();
    hipEventRecord(e0);
    for (int r = 0; r < 5; ++r) launch();
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    ms /= 5;
    const double flops = (double)blocks * 4 * iters * mfma_per_wave_iter * 2048;
    printf("%-36s %8.3f ms %7.2f TF/s (%.1f%% of 78.6)\n", name, ms, flops / ms * 1e-9, flops / ms * 1e-9 / 78.6 * 100);
  };
  const int it = 20000;
  // 256 threads = 4 waves = 1 wave/SIMD per block; 256 blocks = 1/CU, 512 = 2/CU
  run("reg 16acc 1 wave/SIMD", 256, it, 16, [&] { hipLaunchKernelGGL(k_reg<16>, dim3(256), dim3(256), 0, 0, out, it, 1.0); });
  run("reg 16acc 2 waves/SIMD", 512, it, 16, [&] { hipLaunchKernelGGL(k_reg<16>, dim3(512), dim3(256), 0, 0, out, it, 1.0); });
  run("reg 4acc 2 waves/SIMD", 512, it, 4, [&] { hipLaunchKernelGGL(k_reg<4>, dim3(512), dim3(256), 0, 0, out, it, 1.0); });
  run("reg 8acc 1 wave/SIMD", 256, it, 8, [&] { hipLaunchKernelGGL(k_reg<8>, dim3(256), dim3(256), 0, 0, out, it, 1.0); });
  const int it2 = 4000;
  const char* names[3] = {"lds-fed structured 2w/SIMD", "lds-fed random 2w/SIMD", "lds-fed zeros 2w/SIMD"};
  for (int mode = 0; mode < 3; ++mode) {
    run(names[mode], 512, it2, 64, [&] { hipLaunchKernelGGL(k_lds, dim3(512), dim3(256), 0, 0, out, it2, mode, clk); });
    clock_report(512);
  }
  return 0;
}
