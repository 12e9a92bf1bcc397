// Do MFMA waves and VALU waves of ONE workgroup overlap on a SIMD?  A 512-thread
// workgroup per CU: waves 0-3 run an MFMA loop (operands in registers), waves
// 4-7 a VALU loop; each wave records its SIMD (HW_ID).  Times MFMA alone, VALU
// alone and both, for f64 / i8 MFMAs against f64 / int VALU streams.  If "both"
// is near max(alone) the SIMD issues the VALU stream beside the MFMAs.
//   hipcc -O3 --offload-arch=gfx950 scripts/exp/coissue_roles.hip -o scripts/exp/coissue_roles
#include <hip/hip_runtime.h>
#include <cstdio>

#define CK(x)                                                                       \
  do {                                                                              \
    hipError_t e_ = (x);                                                            \
    if (e_ != hipSuccess) {                                                         \
      printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      return 1;                                                                     \
    }                                                                               \
  } while (0)

typedef double d4 __attribute__((ext_vector_type(4)));
typedef int32_t i16v __attribute__((ext_vector_type(16)));
typedef int32_t i4v __attribute__((ext_vector_type(4)));

// MA: 0 none, 1 f64 16x16x4, 2 i8 32x32x32; VB: 0 none, 1 f64 FMA chains, 2 int32 ALU chains
template <int MA, int VB>
__global__ __launch_bounds__(512, 1) void k_roles(double* out, int iters_m, int iters_v, int* simd) {
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  if (lane == 0 && blockIdx.x == 0) simd[w] = (__builtin_amdgcn_s_getreg((4) | (0 << 6) | (31 << 11)) >> 4) & 3;
  double r = 0.0;
  if (w < 4) {
    if constexpr (MA == 1) {
      d4 acc[8];
      for (int i = 0; i < 8; ++i) acc[i] = (d4){0, 0, 0, 0};
      double a = 1.0 + lane * 1e-3, b = 0.5 - lane * 1e-4;
      for (int it = 0; it < iters_m; ++it) {
#pragma unroll
        for (int i = 0; i < 8; ++i) acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[i], 0, 0, 0);
      }
      for (int i = 0; i < 8; ++i) r += acc[i][0] + acc[i][3];
    } else if constexpr (MA == 2) {
      i16v acc[4];
      for (int i = 0; i < 4; ++i)
        for (int q = 0; q < 16; ++q) acc[i][q] = 0;
      i4v a = {lane, lane * 3, lane * 5, lane * 7}, b = {lane ^ 1, lane ^ 2, lane ^ 3, lane ^ 4};
      for (int it = 0; it < iters_m; ++it) {
#pragma unroll
        for (int i = 0; i < 4; ++i) acc[i] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b, acc[i], 0, 0, 0);
      }
      for (int i = 0; i < 4; ++i) r += acc[i][0] + acc[i][15];
    }
  } else {
    if constexpr (VB == 1) {
      double x[8];
      for (int i = 0; i < 8; ++i) x[i] = 1.0 + (lane + i) * 1e-6;
      for (int it = 0; it < iters_v; ++it) {
#pragma unroll
        for (int i = 0; i < 8; ++i) x[i] = __builtin_fma(x[i], 0.9999999, 1e-7);
      }
      for (int i = 0; i < 8; ++i) r += x[i];
    } else if constexpr (VB == 2) {
      uint32_t x[8];
      for (int i = 0; i < 8; ++i) x[i] = lane * 2654435761u + i;
      for (int it = 0; it < iters_v; ++it) {
#pragma unroll
        for (int i = 0; i < 8; ++i) x[i] = ((x[i] << 7) | (x[i] >> 25)) + (x[i] ^ 0x9E3779B9u);
      }
      for (int i = 0; i < 8; ++i) r += (double)x[i];
    }
  }
  out[blockIdx.x * 512 + t] = r;
}

template <int MA, int VB>
static float timeit(double* out, int im, int iv, int* simd, int nb) {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  hipLaunchKernelGGL((k_roles<MA, VB>), dim3(nb), dim3(512), 0, 0, out, im, iv, simd);
  (void)hipDeviceSynchronize();
  float best = 1e30f;
  for (int rep = 0; rep < 5; ++rep) {
    (void)hipEventRecord(e0, 0);
    hipLaunchKernelGGL((k_roles<MA, VB>), dim3(nb), dim3(512), 0, 0, out, im, iv, simd);
    (void)hipEventRecord(e1, 0);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    best = ms < best ? ms : best;
  }
  return best;
}

int main() {
  int ncu = 0;
  CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
  double* out;
  int* simd;
  CK(hipMalloc(&out, sizeof(double) * 512 * ncu));
  CK(hipMalloc(&simd, sizeof(int) * 8));
  const int im64 = 20000, im8 = 20000, iv64 = 40000, ivi = 40000;
  float m64 = timeit<1, 0>(out, im64, 0, simd, ncu), v64 = timeit<0, 1>(out, 0, iv64, simd, ncu);
  float b64 = timeit<1, 1>(out, im64, iv64, simd, ncu);
  float vi = timeit<0, 2>(out, 0, ivi, simd, ncu), b64i = timeit<1, 2>(out, im64, ivi, simd, ncu);
  float m8 = timeit<2, 0>(out, im8, 0, simd, ncu), b8 = timeit<2, 1>(out, im8, iv64, simd, ncu);
  float b8i = timeit<2, 2>(out, im8, ivi, simd, ncu);
  int sid[8];
  CK(hipMemcpy(sid, simd, sizeof(sid), hipMemcpyDeviceToHost));
  printf("wave -> SIMD:");
  for (int i = 0; i < 8; ++i) printf(" %d", sid[i]);
  printf("\n");
  printf("f64 MFMA %.3f | f64 VALU %.3f | both %.3f (sum %.3f max %.3f)\n", m64, v64, b64, m64 + v64, m64 > v64 ? m64 : v64);
  printf("f64 MFMA %.3f | int VALU %.3f | both %.3f (sum %.3f)\n", m64, vi, b64i, m64 + vi);
  printf("i8  MFMA %.3f | f64 VALU %.3f | both %.3f (sum %.3f)\n", m8, v64, b8, m8 + v64);
  printf("i8  MFMA %.3f | int VALU %.3f | both %.3f (sum %.3f)\n", m8, vi, b8i, m8 + vi);
  return 0;
}
