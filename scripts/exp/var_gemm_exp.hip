// Standalone experiment: GP variance contraction  part[rt][col] = sum_rows (L^-1 K*^T)^2
// on the C2 shape (npad = 1024, m = 1M, fp64): a non-persistent
// global_load_lds grid (one workgroup per tile) vs the library's persistent
// k_gp_var.  The per-block stamps of the non-persistent grid are what showed
// CUs idling between tiles (in-order dispatch behind long tiles).  Not part
// of the library.
//
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off -I uptune_amd/csrc \
//     scripts/exp/var_gemm_exp.hip -L uptune_amd -luthot -Wl,-rpath,$PWD/uptune_amd -o scripts/exp/var_gemm_exp
#include "../../uptune_amd/csrc/gp_gemm.hip"

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

namespace ut {

typedef double vd4 __attribute__((ext_vector_type(4)));

// 128 rows x 256 cols per 512-thread workgroup (2 x 4 waves of 64 x 64),
// BK = 16, 3 LDS stages filled by global_load_lds_dwordx4; stage kt+1 stays
// in flight across the barrier of step kt.  A = (L^-1)^T [k][row], B = K*^T [k][col].
constexpr int X_BM = 128, X_BN = 256, X_BK = 16, X_NT = 512, X_ST = 3;
constexpr int X_SA = X_BK * X_BM, X_SB = X_BK * X_BN, X_STAGE = X_SA + X_SB;

template <int PRIO, int FIXB = 0, int FULLK = 0>
__global__ __launch_bounds__(X_NT, 1) void k_var_glds(const double* __restrict__ AT, int64_t lda,
                                                      const double* __restrict__ B, int64_t ldb, int32_t K,
                                                      int32_t RT, int32_t CT, int64_t m, double* __restrict__ part,
                                                      int64_t ldp, unsigned long long* stamps = nullptr) {
  unsigned long long ts0 = __builtin_amdgcn_s_memrealtime(), ts1 = 0, ts2 = 0;
  __shared__ __attribute__((aligned(16))) double lds[X_ST * X_STAGE];
  const int32_t b = blockIdx.x;
  const int32_t xcd = b & 7, jj = b >> 3;
  const int32_t rt = jj % RT;
  const int32_t ct = (jj / RT) * 8 + xcd;
  if (ct >= CT) return;
  const int t = threadIdx.x, lane = t & 63;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const int wm = w >> 2, wn = w & 3;
  const int64_t col0 = (int64_t)ct * X_BN;
  const int32_t row0 = rt * X_BM;
  const int32_t kmax = FULLK ? K : min(K, row0 + X_BM);
  const int32_t nk = kmax / X_BK;

  // wave w stages A rows 2w, 2w+1 and B half-rows 4w .. 4w+3 (row = h >> 1, half = h & 1)
  auto issue = [&](int32_t kt, int s) {
    double* st = lds + s * X_STAGE;
    const int32_t k0 = kt * X_BK;
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int kk = 2 * w + u;
      const double* src = AT + (int64_t)(k0 + kk) * lda + row0 + lane * 2;
      __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)(st + kk * X_BM), 16, 0, 0);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int h = 4 * w + u, kk = h >> 1, half = h & 1;
      const double* src = B + (int64_t)(k0 + kk) * ldb + (FIXB ? 0 : col0) + half * 128 + lane * 2;
      __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)(st + X_SA + kk * X_BN + half * 128),
                                       16, 0, 0);
    }
  };

  vd4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = (vd4){0.0, 0.0, 0.0, 0.0};

  issue(0, 0);
  if (nk > 1) issue(1, 1);
  for (int32_t kt = 0; kt < nk; ++kt) {
    if (kt + 1 < nk)
      asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    else
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (stamps && kt == 0) ts1 = __builtin_amdgcn_s_memrealtime();
    if (kt + 2 < nk) issue(kt + 2, (kt + 2) % X_ST);
    const double* as = lds + (kt % X_ST) * X_STAGE;
    const double* bs = as + X_SA;
    if (PRIO) __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int ks = 0; ks < X_BK / 4; ++ks) {
      const int kr = ks * 4 + (lane >> 4);
      double af[4], bf[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) af[i] = as[kr * X_BM + wm * 64 + i * 16 + (lane & 15)];
#pragma unroll
      for (int j = 0; j < 4; ++j) bf[j] = bs[kr * X_BN + wn * 64 + j * 16 + (lane & 15)];
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(af[i], bf[j], acc[i][j], 0, 0, 0);
    }
    if (PRIO) __builtin_amdgcn_s_setprio(0);
  }

  if (stamps) ts2 = __builtin_amdgcn_s_memrealtime();
  __syncthreads();
  double* red = lds;  // [2][256]
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int cl = wn * 64 + j * 16 + (lane & 15);
    double s = 0.0;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const double x = acc[i][j][r];
        s += x * x;
      }
    s += __shfl_xor(s, 16);
    s += __shfl_xor(s, 32);
    if ((lane >> 4) == 0) red[wm * X_BN + cl] = s;
  }
  __syncthreads();
  if (t < X_BN) {
    const int64_t col = col0 + t;
    if (col < m) part[(int64_t)(rt >> 0) * ldp + col] = red[t] + red[X_BN + t];
  }
  if (stamps && t == 0) {
    unsigned hw, xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    unsigned long long ts3 = __builtin_amdgcn_s_memrealtime();
    unsigned long long* o = stamps + (int64_t)b * 6;
    o[0] = ts0; o[1] = ts1; o[2] = ts2; o[3] = ts3; o[4] = ((unsigned long long)xcc << 32) | hw; o[5] = nk;
  }
}

}  // namespace ut

using namespace ut;

#define CK(x)                                                                      \
  do {                                                                             \
    hipError_t e = (x);                                                            \
    if (e != hipSuccess) {                                                         \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e)); \
      exit(1);                                                                     \
    }                                                                              \
  } while (0)

__global__ void k_fill(double* p, int64_t n, uint64_t seed, int tri_ld) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint64_t x = (uint64_t)i * 0x9E3779B97F4A7C15ull + seed;
  x ^= x >> 31; x *= 0xBF58476D1CE4E5B9ull; x ^= x >> 29;
  double v = (double)(x >> 11) * (1.0 / 9007199254740992.0) - 0.5;
  if (tri_ld > 0) {  // lower triangular row-major [r][k]
    int64_t r = i / tri_ld, k = i % tri_ld;
    if (k > r) v = 0.0;
  }
  p[i] = v;
}

__global__ void k_transpose(const double* a, double* at, int n) {
  int r = blockIdx.y, c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c < n) at[(int64_t)c * n + r] = a[(int64_t)r * n + c];
}

int main(int argc, char** argv) {
  const int npad = argc > 1 ? atoi(argv[1]) : 1024;
  const int64_t m = argc > 2 ? atoll(argv[2]) : (1 << 20);
  const int reps = argc > 3 ? atoi(argv[3]) : 5;
  const int64_t ldk = ((m + 255) / 256) * 256;
  double *L, *LT, *Kst, *p0, *p1;
  CK(hipMalloc(&L, sizeof(double) * npad * npad));
  CK(hipMalloc(&LT, sizeof(double) * npad * npad));
  CK(hipMalloc(&Kst, sizeof(double) * npad * ldk));
  const int RT = npad / 128;
  CK(hipMalloc(&p0, sizeof(double) * RT * ldk));
  CK(hipMalloc(&p1, sizeof(double) * RT * ldk));
  k_fill<<<(npad * npad + 255) / 256, 256>>>(L, (int64_t)npad * npad, 1, npad);
  k_fill<<<(unsigned)(((int64_t)npad * ldk + 255) / 256), 256>>>(Kst, (int64_t)npad * ldk, 2, 0);
  k_transpose<<<dim3((npad + 255) / 256, npad), 256>>>(L, LT, npad);
  CK(hipDeviceSynchronize());

  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const double flops = (double)m * npad * (npad + 1);
  const int CTx = (int)((m + 255) / 256), CTx8 = ((CTx + 7) / 8) * 8;

  int32_t* ticket;
  CK(hipMalloc(&ticket, sizeof(int32_t) * 8));
  auto run0 = [&]() {
    CK(hipMemsetAsync(ticket, 0, sizeof(int32_t) * 8, 0));
    hipLaunchKernelGGL(k_gp_var<double>, dim3(256), dim3(V_NT), 0, 0, (const double*)LT, (int64_t)npad,
                       (const double*)Kst, ldk, npad, RT, CTx, m, ticket, p0, ldk);
  };
  auto run1 = [&](int prio) {
    if (prio)
      hipLaunchKernelGGL(k_var_glds<1>, dim3(RT * CTx8), dim3(X_NT), 0, 0, LT, (int64_t)npad, Kst, ldk, npad, RT, CTx,
                         m, p1, ldk);
    else
      hipLaunchKernelGGL(k_var_glds<0>, dim3(RT * CTx8), dim3(X_NT), 0, 0, LT, (int64_t)npad, Kst, ldk, npad, RT, CTx,
                         m, p1, ldk);
  };
  auto timeit = [&](const char* name, auto fn) {
    fn();
    CK(hipGetLastError());
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    for (int r = 0; r < reps; ++r) fn();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    ms /= reps;
    printf("%-28s %9.3f ms  %7.2f TF/s  (%.1f%% of 78.6)\n", name, ms, flops / ms * 1e-9, flops / ms * 1e-9 / 78.6 * 100);
    fflush(stdout);
  };
  timeit("lib k_gp_var<double> (persistent)", run0);
  timeit("glds 128x256 3-stage", [&] { run1(0); });
  std::vector<double> h0((size_t)RT * ldk), h1((size_t)RT * ldk);
  CK(hipMemcpy(h0.data(), p0, sizeof(double) * h0.size(), hipMemcpyDeviceToHost));
  CK(hipMemcpy(h1.data(), p1, sizeof(double) * h1.size(), hipMemcpyDeviceToHost));
  int64_t bad = 0;
  for (int r = 0; r < RT; ++r)
    for (int64_t c = 0; c < m; ++c) {
      double a = h0[(size_t)r * ldk + c], b = h1[(size_t)r * ldk + c];
      if (a != b) ++bad;
    }
  printf("grid vs persistent: %lld mismatching partials of %lld\n", (long long)bad, (long long)(RT * m));
  timeit("glds 128x256 3-stage prio", [&] { run1(1); });
  timeit("glds fixed B tile (L2)", [&] {
    hipLaunchKernelGGL((k_var_glds<0, 1>), dim3(RT * CTx8), dim3(X_NT), 0, 0, LT, (int64_t)npad, Kst, ldk, npad, RT, CTx,
                       m, p1, ldk);
  });
  {
    // full-K tiles (square L): flops m * n * n * 2
    hipLaunchKernelGGL((k_var_glds<0, 0, 1>), dim3(RT * CTx8), dim3(X_NT), 0, 0, LT, (int64_t)npad, Kst, ldk, npad, RT,
                       CTx, m, p1, ldk);
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    for (int r = 0; r < reps; ++r)
      hipLaunchKernelGGL((k_var_glds<0, 0, 1>), dim3(RT * CTx8), dim3(X_NT), 0, 0, LT, (int64_t)npad, Kst, ldk, npad,
                         RT, CTx, m, p1, ldk);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    ms /= reps;
    const double f2 = 2.0 * m * npad * (double)npad;
    printf("%-28s %9.3f ms  %7.2f TF/s  (%.1f%% of 78.6, MFMA flops)\n", "glds full-K (square)", ms, f2 / ms * 1e-9,
           f2 / ms * 1e-9 / 78.6 * 100);
  }
  {
    unsigned long long* st;
    const int nb = RT * CTx8;
    CK(hipMalloc(&st, sizeof(unsigned long long) * 6 * nb));
    CK(hipMemset(st, 0, sizeof(unsigned long long) * 6 * nb));
    hipLaunchKernelGGL((k_var_glds<0, 0, 0>), dim3(nb), dim3(X_NT), 0, 0, LT, (int64_t)npad, Kst, ldk, npad, RT, CTx, m,
                       p1, ldk, st);
    CK(hipDeviceSynchronize());
    std::vector<unsigned long long> h((size_t)6 * nb);
    CK(hipMemcpy(h.data(), st, sizeof(unsigned long long) * h.size(), hipMemcpyDeviceToHost));
    FILE* f = fopen("gpurun_out/stamps.bin", "wb");
    if (f) {
      fwrite(h.data(), 8, h.size(), f);
      fclose(f);
    }
    printf("stamps written for %d blocks\n", nb);
  }
  CK(hipMemset(Kst, 0, sizeof(double) * npad * ldk));
  timeit("lib, K* = 0 (DVFS check)", run0);
  timeit("glds, K* = 0", [&] { run1(0); });
  return bad ? 2 : 0;
}
