// Experiment: HBM write bandwidth of K*-shaped stores on MI355X.
//   linear4: grid-stride dwordx4 streaming stores
//   linear2: dwordx2
//   kstar:   the k_gp_kstar epilogue's pattern: a 128 x 128 tile of a [n][ldk]
//            f64 matrix per 256-thread block, lane -> (row = (lane>>4) + 4r + 16i
//            + 64 wm, col = lane & 15 + 16 jj + 64 wn), one dwordx2 per element
//   kstar_nt: the same with nontemporal stores
//   hipcc -O3 --offload-arch=gfx950 scripts/exp/write_bw.hip -o scripts/exp/write_bw
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__global__ void k_lin4(double4* p, int64_t n4, double v) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (int64_t)gridDim.x * blockDim.x)
    p[i] = make_double4(v, v, v, v);
}
__global__ void k_lin2(double2* p, int64_t n2, double v) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n2; i += (int64_t)gridDim.x * blockDim.x)
    p[i] = make_double2(v, v);
}
template <int NT>
__global__ __launch_bounds__(256) void k_tile(double* p, int n, int64_t ldk, int RT, int CT, double v) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, wm = w >> 1, wn = w & 1;
  for (int64_t item = blockIdx.x; item < (int64_t)RT * CT; item += gridDim.x) {
    const int rt = item % RT;
    const int64_t ct = item / RT;
#pragma unroll
    for (int jj = 0; jj < 4; ++jj)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int64_t row = rt * 128 + wm * 64 + i * 16 + (lane >> 4) + 4 * r;
          const int64_t col = ct * 128 + wn * 64 + jj * 16 + (lane & 15);
          if (NT) __builtin_nontemporal_store(v + r, p + row * ldk + col);
          else p[row * ldk + col] = v + r;
        }
  }
}

int main() {
  const int n = 1024;
  const int64_t m = 1 << 20, ldk = m;
  const int64_t N = (int64_t)n * ldk;
  double* p;
  hipMalloc(&p, sizeof(double) * N);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  auto time = [&](const char* name, auto launch) {
    launch();
    hipDeviceSynchronize();
    hipEventRecord(e0);
    for (int r = 0; r < 5; ++r) launch();
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    ms /= 5;
    printf("%-12s %8.3f ms  %6.2f TB/s\n", name, ms, N * 8.0 / ms * 1e-9);
  };
  time("linear4", [&] { hipLaunchKernelGGL(k_lin4, dim3(2048), dim3(256), 0, 0, (double4*)p, N / 4, 1.0); });
  time("linear2", [&] { hipLaunchKernelGGL(k_lin2, dim3(2048), dim3(256), 0, 0, (double2*)p, N / 2, 1.0); });
  time("kstar", [&] { hipLaunchKernelGGL(k_tile<0>, dim3(512), dim3(256), 0, 0, p, n, ldk, 8, (int)(m / 128), 1.0); });
  time("kstar_nt", [&] { hipLaunchKernelGGL(k_tile<1>, dim3(512), dim3(256), 0, 0, p, n, ldk, 8, (int)(m / 128), 1.0); });
  time("kstar 2048b", [&] { hipLaunchKernelGGL(k_tile<0>, dim3(2048), dim3(256), 0, 0, p, n, ldk, 8, (int)(m / 128), 1.0); });
  return 0;
}
