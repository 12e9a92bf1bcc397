// v_mfma_f32_16x16x4f32 on gfx950: (1) the A / B / D lane maps, checked against a
// host product (A[i][k] = i + 16 k + 1, B[k][j] = (k + 1) * 100 + j), with the
// assumed maps A: lane l holds A[l & 15][l >> 4], B: B[l >> 4][l & 15],
// D: register r of lane l holds D[4 (l >> 4) + r][l & 15];
// (2) does the f32 MFMA issue beside VALU streams (f32 FMA chains) on one SIMD?
//   hipcc -O3 --offload-arch=gfx950 scripts/exp/f32_mfma_probe.hip -o scripts/exp/f32_mfma_probe
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f4 __attribute__((ext_vector_type(4)));

__global__ void k_map(float* out) {
  const int l = threadIdx.x;
  const float a = (float)((l & 15) + 16 * (l >> 4) + 1);
  const float b = (float)(((l >> 4) + 1) * 100 + (l & 15));
  f4 acc = {0.f, 0.f, 0.f, 0.f};
  acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc, 0, 0, 0);
  for (int r = 0; r < 4; ++r) out[l * 4 + r] = acc[r];
}

template <int MA, int VB>
__global__ __launch_bounds__(512, 1) void k_roles(double* out, int iters_m, int iters_v) {
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  double r = 0.0;
  if (w < 4) {
    if constexpr (MA == 1) {
      f4 acc[8];
      for (int i = 0; i < 8; ++i) acc[i] = (f4){0, 0, 0, 0};
      float a = 1.0f + lane * 1e-3f, b = 0.5f - lane * 1e-4f;
      for (int it = 0; it < iters_m; ++it) {
#pragma unroll
        for (int i = 0; i < 8; ++i) acc[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[i], 0, 0, 0);
      }
      for (int i = 0; i < 8; ++i) r += acc[i][0] + acc[i][3];
    }
  } else {
    if constexpr (VB == 1) {
      float x[8];
      for (int i = 0; i < 8; ++i) x[i] = 1.0f + (lane + i) * 1e-6f;
      for (int it = 0; it < iters_v; ++it) {
#pragma unroll
        for (int i = 0; i < 8; ++i) x[i] = __builtin_fmaf(x[i], 0.9999999f, 1e-7f);
      }
      for (int i = 0; i < 8; ++i) r += x[i];
    } else if constexpr (VB == 2) {
      double x[8];
      for (int i = 0; i < 8; ++i) x[i] = 1.0 + (lane + i) * 1e-6;
      for (int it = 0; it < iters_v; ++it) {
#pragma unroll
        for (int i = 0; i < 8; ++i) x[i] = __builtin_fma(x[i], 0.9999999, 1e-7);
      }
      for (int i = 0; i < 8; ++i) r += x[i];
    }
  }
  out[blockIdx.x * 512 + t] = r;
}

template <int MA, int VB>
static float timeit(double* out, int im, int iv, int nb) {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  hipLaunchKernelGGL((k_roles<MA, VB>), dim3(nb), dim3(512), 0, 0, out, im, iv);
  (void)hipDeviceSynchronize();
  float best = 1e30f;
  for (int rep = 0; rep < 5; ++rep) {
    (void)hipEventRecord(e0, 0);
    hipLaunchKernelGGL((k_roles<MA, VB>), dim3(nb), dim3(512), 0, 0, out, im, iv);
    (void)hipEventRecord(e1, 0);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    best = ms < best ? ms : best;
  }
  return best;
}

int main() {
  float* d;
  if (hipMalloc(&d, 64 * 4 * sizeof(float)) != hipSuccess) return 1;
  hipLaunchKernelGGL(k_map, dim3(1), dim3(64), 0, 0, d);
  float h[256];
  if (hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess) return 1;
  int bad = 0;
  for (int l = 0; l < 64; ++l)
    for (int r = 0; r < 4; ++r) {
      const int i = 4 * (l >> 4) + r, j = l & 15;
      double want = 0;
      for (int k = 0; k < 4; ++k) want += (double)(i + 16 * k + 1) * (double)((k + 1) * 100 + j);
      if ((double)h[l * 4 + r] != want) ++bad;
    }
  printf("f32 16x16x4 map (D row 4 (l >> 4) + r): %s (%d mismatches)\n", bad ? "WRONG" : "ok", bad);
  if (bad) {   // print what lane 16 / 17 hold
    for (int l = 0; l < 20; ++l) printf("lane %d: %g %g %g %g\n", l, h[l * 4], h[l * 4 + 1], h[l * 4 + 2], h[l * 4 + 3]);
  }
  int ncu = 0;
  (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
  double* out;
  if (hipMalloc(&out, sizeof(double) * 512 * ncu) != hipSuccess) return 1;
  const int im = 20000, iv = 40000;
  float m = timeit<1, 0>(out, im, 0, ncu), v = timeit<0, 1>(out, 0, iv, ncu), b = timeit<1, 1>(out, im, iv, ncu);
  float v64 = timeit<0, 2>(out, 0, iv, ncu), b64 = timeit<1, 2>(out, im, iv, ncu);
  printf("f32 MFMA %.3f | f32 VALU %.3f | both %.3f (sum %.3f)\n", m, v, b, m + v);
  printf("f32 MFMA %.3f | f64 VALU %.3f | both %.3f (sum %.3f)\n", m, v64, b64, m + v64);
  return 0;
}
