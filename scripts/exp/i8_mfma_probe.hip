// Lane map check of v_mfma_i32_16x16x64_i8 on gfx950 with exact integer data
// (cdna_hip_programming.md: "check the map with exact integer data").
// Assumed: lane l holds A[row l&15][k = 16 (l>>4) + j] and B[k = 16 (l>>4) + j][col l&15]
// (j = 0..15, 16 bytes = 4 VGPRs), D[row 4 (l>>4) + q][col l&15] (q = 0..3).
// Also checks the row permutation sigma(4g + q) = g + 4q that puts the i32
// result of row r where v_mfma_f64_16x16x4 keeps row r (row (l>>4) + 4q).
// Standalone: hipcc -O3 --offload-arch=gfx950 i8_mfma_probe.hip -o i8_mfma_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>

typedef int32_t i32x4 __attribute__((ext_vector_type(4)));
typedef int32_t i32x4v __attribute__((ext_vector_type(4)));

__global__ void k_probe(const int8_t* A, const int8_t* B, int32_t* D, int32_t* Dp) {
  const int l = threadIdx.x;
  i32x4v a, b, ap;
  const int row = l & 15, kg = l >> 4;
  int8_t* pa = reinterpret_cast<int8_t*>(&a);
  int8_t* pap = reinterpret_cast<int8_t*>(&ap);
  int8_t* pb = reinterpret_cast<int8_t*>(&b);
  const int prow = (row >> 2) + 4 * (row & 3);   // sigma
  for (int j = 0; j < 16; ++j) {
    pa[j] = A[row * 64 + 16 * kg + j];
    pap[j] = A[prow * 64 + 16 * kg + j];
    pb[j] = B[(16 * kg + j) * 16 + row];
  }
  i32x4 acc = {0, 0, 0, 0}, accp = {0, 0, 0, 0};
  acc = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, acc, 0, 0, 0);
  accp = __builtin_amdgcn_mfma_i32_16x16x64_i8(ap, b, accp, 0, 0, 0);
  for (int q = 0; q < 4; ++q) {
    D[(4 * kg + q) * 16 + row] = acc[q];     // standard C/D map
    Dp[(kg + 4 * q) * 16 + row] = accp[q];   // the f64 MFMA's row map, via sigma
  }
}

int main() {
  int8_t hA[16 * 64], hB[64 * 16];
  srand(7);
  for (int i = 0; i < 16 * 64; ++i) hA[i] = (int8_t)(rand() % 255 - 127);
  for (int i = 0; i < 64 * 16; ++i) hB[i] = (int8_t)(rand() % 255 - 127);
  int8_t *dA, *dB;
  int32_t *dD, *dDp;
  hipMalloc(&dA, sizeof(hA));
  hipMalloc(&dB, sizeof(hB));
  hipMalloc(&dD, 256 * 4);
  hipMalloc(&dDp, 256 * 4);
  hipMemcpy(dA, hA, sizeof(hA), hipMemcpyHostToDevice);
  hipMemcpy(dB, hB, sizeof(hB), hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k_probe, dim3(1), dim3(64), 0, 0, dA, dB, dD, dDp);
  int32_t hD[256], hDp[256];
  hipMemcpy(hD, dD, sizeof(hD), hipMemcpyDeviceToHost);
  hipMemcpy(hDp, dDp, sizeof(hDp), hipMemcpyDeviceToHost);
  int bad = 0, badp = 0;
  for (int r = 0; r < 16; ++r)
    for (int c = 0; c < 16; ++c) {
      int32_t s = 0;
      for (int k = 0; k < 64; ++k) s += (int32_t)hA[r * 64 + k] * (int32_t)hB[k * 16 + c];
      bad += hD[r * 16 + c] != s;
      badp += hDp[r * 16 + c] != s;
    }
  printf("i8 16x16x64 map: %d / 256 wrong; with sigma rows in the f64 layout: %d / 256 wrong\n", bad, badp);
  return bad || badp;
}
