// Round 6: does the int8 MFMA shape change the clock the chip holds on random
// operands (MI355X_MICROARCH.md 'DVFS give-back' item 7 measured it for bf16)?
// Bare loops, operands in registers (random, per lane), independent accumulator
// chains, every CU busy; ops/s of v_mfma_i32_32x32x32_i8 vs v_mfma_i32_16x16x64_i8
// at the same K per instruction-pair and the same MACs per loop.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 scripts/exp/i8_shape_probe.hip -o scripts/exp/i8_shape_probe
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <vector>

typedef int32_t v4i __attribute__((ext_vector_type(4)));
typedef int32_t v16i __attribute__((ext_vector_type(16)));

// 32x32x32: 4 chains of 16 regs; each iteration 8 MFMAs (32768 MAC each)
__global__ __launch_bounds__(256) void k32(const v4i* __restrict__ in, int iters, int32_t* __restrict__ out) {
  const int t = blockIdx.x * 256 + threadIdx.x;
  v4i a0 = in[t & 1023], a1 = in[(t + 7) & 1023], b0 = in[(t + 13) & 1023], b1 = in[(t + 29) & 1023];
  v16i c0 = {}, c1 = {}, c2 = {}, c3 = {};
  for (int i = 0; i < iters; ++i) {
    c0 = __builtin_amdgcn_mfma_i32_32x32x32_i8(a0, b0, c0, 0, 0, 0);
    c1 = __builtin_amdgcn_mfma_i32_32x32x32_i8(a0, b1, c1, 0, 0, 0);
    c2 = __builtin_amdgcn_mfma_i32_32x32x32_i8(a1, b0, c2, 0, 0, 0);
    c3 = __builtin_amdgcn_mfma_i32_32x32x32_i8(a1, b1, c3, 0, 0, 0);
    c0 = __builtin_amdgcn_mfma_i32_32x32x32_i8(a1, b1, c0, 0, 0, 0);
    c1 = __builtin_amdgcn_mfma_i32_32x32x32_i8(a1, b0, c1, 0, 0, 0);
    c2 = __builtin_amdgcn_mfma_i32_32x32x32_i8(a0, b1, c2, 0, 0, 0);
    c3 = __builtin_amdgcn_mfma_i32_32x32x32_i8(a0, b0, c3, 0, 0, 0);
  }
  int32_t s = 0;
  for (int r = 0; r < 16; ++r) s += c0[r] ^ c1[r] ^ c2[r] ^ c3[r];
  out[t] = s;
}

// 16x16x64: 8 chains of 4 regs; each iteration 32 MFMAs (16384 MAC each) = the same MACs
__global__ __launch_bounds__(256) void k16(const v4i* __restrict__ in, int iters, int32_t* __restrict__ out) {
  const int t = blockIdx.x * 256 + threadIdx.x;
  v4i a0 = in[t & 1023], a1 = in[(t + 7) & 1023], b0 = in[(t + 13) & 1023], b1 = in[(t + 29) & 1023];
  v4i c[8] = {};
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int h = 0; h < 4; ++h) {
      c[0] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a0, b0, c[0], 0, 0, 0);
      c[1] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a0, b1, c[1], 0, 0, 0);
      c[2] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a1, b0, c[2], 0, 0, 0);
      c[3] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a1, b1, c[3], 0, 0, 0);
      c[4] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a1, b1, c[4], 0, 0, 0);
      c[5] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a1, b0, c[5], 0, 0, 0);
      c[6] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a0, b1, c[6], 0, 0, 0);
      c[7] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a0, b0, c[7], 0, 0, 0);
    }
  }
  int32_t s = 0;
  for (int h = 0; h < 8; ++h)
    for (int r = 0; r < 4; ++r) s ^= c[h][r];
  out[t] = s;
}

int main(int argc, char** argv) {
  const int zero = argc > 1 ? atoi(argv[1]) : 0;
  std::vector<int32_t> h(4096);
  srand(3);
  for (auto& x : h) x = zero ? 0 : (int32_t)(((uint32_t)rand() << 16) ^ (uint32_t)rand());
  v4i* in;
  int32_t* out;
  hipMalloc(&in, h.size() * 4);
  hipMalloc(&out, 256 * 8 * 256 * 4);
  hipMemcpy(in, h.data(), h.size() * 4, hipMemcpyHostToDevice);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int iters = 20000;
  const int grid = 256 * 2;   // two 4-wave workgroups per CU: two waves per SIMD
  std::vector<float> t32, t16;
  for (int rep = 0; rep < 7; ++rep) {
    for (int v = 0; v < 2; ++v) {
      hipEventRecord(e0);
      if (v == 0) hipLaunchKernelGGL(k32, dim3(grid), dim3(256), 0, 0, in, iters, out);
      else hipLaunchKernelGGL(k16, dim3(grid), dim3(256), 0, 0, in, iters, out);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      if (rep >= 2) (v == 0 ? t32 : t16).push_back(ms);
    }
  }
  std::sort(t32.begin(), t32.end());
  std::sort(t16.begin(), t16.end());
  const double macs = (double)grid * 4 * iters * 8 * 32768.0;   // waves * iters * 8 x 32x32x32
  printf("%s operands: 32x32x32 %.3f ms (%.0f TOPS)   16x16x64 %.3f ms (%.0f TOPS)   ratio %.3f\n",
         zero ? "zero" : "random", t32[t32.size() / 2], 2 * macs / (t32[t32.size() / 2] * 1e-3) / 1e12,
         t16[t16.size() / 2], 2 * macs / (t16[t16.size() / 2] * 1e-3) / 1e12, t32[t32.size() / 2] / t16[t16.size() / 2]);
  return 0;
}
