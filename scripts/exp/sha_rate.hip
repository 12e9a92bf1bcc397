// SHA-256 compression throughput on gfx950: ILP (independent messages per
// lane) x block size.  Standalone: hipcc -O3 --offload-arch=gfx950 sha_rate.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include "../../uptune_amd/csrc/ut_core.h"

template <int ILP>
__global__ void k_sha(uint32_t* out, int iters, uint32_t seed) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t H[ILP][8];
  uint32_t W[ILP][16];
#pragma unroll
  for (int j = 0; j < ILP; ++j) {
    ut::sha256_init(H[j]);
#pragma unroll
    for (int w = 0; w < 16; ++w) W[j][w] = t * 2654435761u + w * 97u + j + seed;
  }
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int j = 0; j < ILP; ++j) {
      uint32_t X[16];
#pragma unroll
      for (int w = 0; w < 16; ++w) X[w] = W[j][w] ^ H[j][w & 7];
      ut::sha256_compress(H[j], X);
    }
  }
  uint32_t acc = 0;
#pragma unroll
  for (int j = 0; j < ILP; ++j)
#pragma unroll
    for (int w = 0; w < 8; ++w) acc ^= H[j][w];
  out[t] = acc;
}

template <int ILP>
void run(int bs, int nblk, int iters) {
  uint32_t* d;
  hipMalloc(&d, sizeof(uint32_t) * bs * nblk);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  hipLaunchKernelGGL(k_sha<ILP>, dim3(nblk), dim3(bs), 0, 0, d, iters, 1u);
  hipDeviceSynchronize();
  hipEventRecord(a, 0);
  hipLaunchKernelGGL(k_sha<ILP>, dim3(nblk), dim3(bs), 0, 0, d, iters, 2u);
  hipEventRecord(b, 0);
  hipEventSynchronize(b);
  float ms = 0;
  hipEventElapsedTime(&ms, a, b);
  const double comps = (double)bs * nblk * iters * ILP;
  printf("ILP=%d bs=%d nblk=%d: %.3f ms  %.2f G compressions/s\n", ILP, bs, nblk, ms, comps / ms / 1e6);
  hipFree(d);
}

int main() {
  const int lanes = 1 << 20;
  for (int bs : {64, 128, 256}) {
    run<1>(bs, lanes / bs, 64);
    run<2>(bs, lanes / bs / 2, 64);
    run<4>(bs, lanes / bs / 4, 64);
  }
  return 0;
}
