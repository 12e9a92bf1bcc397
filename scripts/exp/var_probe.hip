// Experiment: where k_gp_var<double> loses MFMA time on MI355X.  (Round 2/3
// measurement aid: it includes gp_gemm.hip as of round 4 -- `git show
// b6f4ed2:uptune_amd/csrc/gp_gemm.hip` -- whose fp64 k_gp_var<T> round 5 removed.)  A copy of the
// library kernel's structure (persistent, per-XCD tickets, 128 x 256 tiles,
// 3-stage global_load_lds ring, triangular skip) with knobs:
//   MODE 0  as the library
//   MODE 1  no global loads (LDS stale): compute + barriers + item transitions
//   MODE 2  B (K*) always from strip 0: every B read hits L2
//   MODE 3  MODE 2 + A from row tile 0
//   MODE 4  prefetch across items (next ticket's first two stages issued
//           during the current item's last two steps)
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -I uptune_amd/csrc scripts/exp/var_probe.hip \
//     -L uptune_amd -luthot -Wl,-rpath,'$ORIGIN/../../uptune_amd' -o scripts/exp/var_probe
#include "../../uptune_amd/csrc/gp_gemm.hip"

#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>
#include <cmath>

namespace ut {

template <int MODE>
__global__ __launch_bounds__(V_NT, 1) void k_probe(const double* __restrict__ AT, int64_t lda,
                                                   const double* __restrict__ B, int64_t ldb, int32_t K, int32_t RT,
                                                   int32_t CT, int64_t m, int32_t* __restrict__ ticket,
                                                   double* __restrict__ part, int64_t ldp) {
  using C = VCfg<double>;
  constexpr int BK = C::BK;
  __shared__ __attribute__((aligned(16))) double lds[V_ST * C::STAGE + 2 * VAR_BN + 2];
  double* red = lds + V_ST * C::STAGE;
  int32_t* s_item = reinterpret_cast<int32_t*>(lds + V_ST * C::STAGE + 2 * VAR_BN);
  const int t = threadIdx.x, lane = t & 63;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const int wm = w >> 2, wn = w & 3;
  const int32_t xcd = blockIdx.x & 7;
  if (t == 0) s_item[0] = atomicAdd(&ticket[xcd], 1);
  __syncthreads();
  int32_t j = s_item[0];
  bool pre = false;  // MODE 4: this item's first two stages already issued
  int32_t sb = 0;    // MODE 4: ring slot of this item's stage 0
  bool stored = false;
  for (;;) {
    const int32_t ct = (j / RT) * 8 + xcd;
    if (ct >= CT) break;
    const int32_t rt = RT - 1 - (j % RT);
    const int64_t col0 = MODE >= 2 && MODE <= 3 ? 0 : (int64_t)ct * VAR_BN;
    const int32_t row0 = rt * VAR_BM;
    const int32_t arow0 = MODE == 3 ? 0 : row0;
    const int32_t nk = min(K, row0 + VAR_BM) / BK;
    int32_t jn = 0, nk_n = 0, rown = 0;
    int64_t coln = 0;
    bool nvalid = false;
    if (MODE == 4) {
      if (t == 0) s_item[1] = atomicAdd(&ticket[xcd], 1);
      __syncthreads();
      jn = s_item[1];
      const int32_t ctn = (jn / RT) * 8 + xcd;
      nvalid = ctn < CT;
      rown = (RT - 1 - (jn % RT)) * VAR_BM;
      coln = (int64_t)ctn * VAR_BN;
      nk_n = min(K, rown + VAR_BM) / BK;
    }
    vd4 acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) acc[i][jj] = (vd4){0.0, 0.0, 0.0, 0.0};
    if (MODE != 1 && !pre) {
      var_issue<double>(AT, lda, B, ldb, arow0, col0, 0, lds + (sb % V_ST) * C::STAGE, w, lane);
      if (nk > 1) var_issue<double>(AT, lda, B, ldb, arow0, col0, BK, lds + ((sb + 1) % V_ST) * C::STAGE, w, lane);
    }
    const int32_t nfull = min(nk, row0 / BK);
    for (int32_t kt = 0; kt < nk; ++kt) {
      if (MODE == 4) {
        const bool more = kt + 1 < nk || nvalid;  // a later stage is in flight behind this one
        if (kt == 0 && stored && w < 4) {         // the previous item's part store sits behind it
          if (more) asm volatile("s_waitcnt vmcnt(7)" ::: "memory");
          else asm volatile("s_waitcnt vmcnt(1)" ::: "memory");
        } else {
          if (more) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
          else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
      } else if (MODE != 1) {
        if (kt + 1 < nk)
          asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
        else
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      if (MODE != 1) {
        if (kt + 2 < nk)
          var_issue<double>(AT, lda, B, ldb, arow0, col0, (kt + 2) * BK, lds + ((sb + kt + 2) % V_ST) * C::STAGE, w,
                            lane);
        else if (MODE == 4 && nvalid && kt + 2 - nk < nk_n)
          var_issue<double>(AT, lda, B, ldb, rown, coln, (kt + 2 - nk) * BK, lds + ((sb + kt + 2) % V_ST) * C::STAGE,
                            w, lane);
      }
      const double* as = lds + ((sb + kt) % V_ST) * C::STAGE;
      int imin = 0;
      if (kt >= nfull) {
        const int kd = kt - nfull - 4 * wm;
        imin = kd < 0 ? 0 : kd;
      }
      if (imin < 4) var_step_f64(as, as + C::SA, wm, wn, lane, imin, acc);
    }
    __syncthreads();
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) {
      const int cl = wn * 64 + jj * 16 + (lane & 15);
      double s = 0.0;
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) s += acc[i][jj][r] * acc[i][jj][r];
      s += __shfl_xor(s, 16);
      s += __shfl_xor(s, 32);
      if ((lane >> 4) == 0) red[wm * VAR_BN + cl] = s;
    }
    __syncthreads();
    if (t < VAR_BN) {
      const int64_t col = (int64_t)ct * VAR_BN + t;
      if (col < m) part[(int64_t)rt * ldp + col] = red[t] + red[VAR_BN + t];
    }
    if (MODE == 4) {
      j = jn;
      pre = nvalid;
      sb = (sb + nk) % V_ST;
      stored = true;
    } else {
      if (t == 0) s_item[0] = atomicAdd(&ticket[xcd], 1);
      __syncthreads();
      j = s_item[0];
    }
  }
}

template __global__ void k_probe<0>(const double*, int64_t, const double*, int64_t, int32_t, int32_t, int32_t,
                                    int64_t, int32_t*, double*, int64_t);
template __global__ void k_probe<1>(const double*, int64_t, const double*, int64_t, int32_t, int32_t, int32_t,
                                    int64_t, int32_t*, double*, int64_t);
template __global__ void k_probe<2>(const double*, int64_t, const double*, int64_t, int32_t, int32_t, int32_t,
                                    int64_t, int32_t*, double*, int64_t);
template __global__ void k_probe<3>(const double*, int64_t, const double*, int64_t, int32_t, int32_t, int32_t,
                                    int64_t, int32_t*, double*, int64_t);
template __global__ void k_probe<4>(const double*, int64_t, const double*, int64_t, int32_t, int32_t, int32_t,
                                    int64_t, int32_t*, double*, int64_t);


// ---------------------------------------------------------------------------
// k_var2: the variance contraction as TWO 256-thread workgroups per CU
// (ping-pong): each SIMD holds one wave of each, so one workgroup's barrier
// wait and epilogue overlap the other's MFMAs.  Tile 128 rows x 128 cols
// (2 x 2 waves of 64 x 64), BK k per stage, NS-deep global_load_lds ring.
// ---------------------------------------------------------------------------
template <int NOLOAD, int BK, int NS, int FULLK = 0, int ILV = 0>
__global__ __launch_bounds__(256, 2) void k_var2(const double* __restrict__ AT, int64_t lda,
                                                 const double* __restrict__ B, int64_t ldb, int32_t K, int32_t RT,
                                                 int32_t CT, int64_t m, int32_t* __restrict__ ticket,
                                                 double* __restrict__ part, int64_t ldp,
                                                 unsigned long long* __restrict__ clk) {
  const unsigned long long c0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  constexpr int BM = 128, BN = 128, SA = BK * BM, STAGE = SA + BK * BN, PW = BK / 2;  // glds per wave per stage
  __shared__ __attribute__((aligned(16))) double lds[NS * STAGE + 2 * BN + 2];
  double* red = lds + NS * STAGE;
  int32_t& s_item = *reinterpret_cast<int32_t*>(lds + NS * STAGE + 2 * BN);
  const int t = threadIdx.x, lane = t & 63;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const int wm = w >> 1, wn = w & 1;
  const int32_t xcd = blockIdx.x & 7;
  auto issue = [&](int32_t row0, int64_t col0, int32_t k0, double* st) {
#pragma unroll
    for (int u = 0; u < PW / 2; ++u) {
      const int q = w * (PW / 2) + u;  // k row of the A tile
      __builtin_amdgcn_global_load_lds(AT + (int64_t)(k0 + q) * lda + row0 + lane * 2,
                                       (__attribute__((address_space(3))) void*)(st + q * BM), 16, 0, 0);
    }
#pragma unroll
    for (int u = 0; u < PW / 2; ++u) {
      const int q = w * (PW / 2) + u;
      __builtin_amdgcn_global_load_lds(B + (int64_t)(k0 + q) * ldb + col0 + lane * 2,
                                       (__attribute__((address_space(3))) void*)(st + SA + q * BN), 16, 0, 0);
    }
  };
  for (;;) {
    if (t == 0) s_item = atomicAdd(&ticket[xcd], 1);
    __syncthreads();
    const int32_t j = s_item;
    const int32_t ct = (j / RT) * 8 + xcd;
    if (ct >= CT) break;
    const int32_t rt = RT - 1 - (j % RT);
    const int64_t col0 = (int64_t)ct * BN;
    const int32_t row0 = rt * BM;
    const int32_t nk = FULLK ? K / BK : min(K, row0 + BM) / BK;
    vd4 acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) acc[i][jj] = (vd4){0.0, 0.0, 0.0, 0.0};
    if (!NOLOAD) {
#pragma unroll
      for (int s = 0; s < NS - 1; ++s)
        if (s < nk) issue(row0, col0, s * BK, lds + s * STAGE);
    }
    const int32_t nfull = FULLK ? nk : min(nk, row0 / BK);
    for (int32_t kt = 0; kt < nk; ++kt) {
      if (!NOLOAD) {
        const int32_t ahead = min(NS - 2, nk - 1 - kt);  // stages in flight behind stage kt
        if (ahead >= 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * PW) : "memory");
        else if (ahead == 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PW) : "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      if (!NOLOAD && kt + NS - 1 < nk) issue(row0, col0, (kt + NS - 1) * BK, lds + ((kt + NS - 1) % NS) * STAGE);
      const double* as = lds + (kt % NS) * STAGE;
      const double* bs = as + SA;
      int imin = 0;
      if (kt >= nfull) {
        const int kd = kt - nfull;
        if (ILV) {
          // sub-tile i = rows (2i + wm) * 16 ..: all zero iff BK * kd >= (2i + wm + 1) * 16
          const int z = (BK * kd) / 16 - wm;  // i < z/2 (rounded up) are zero
          imin = z <= 0 ? 0 : (z + 1) >> 1;
        } else {
          imin = BK == 16 ? kd - 4 * wm : (kd - 8 * wm) >> 1;
          imin = imin < 0 ? 0 : imin;
        }
      }
      if (imin < 4) {
#pragma unroll
        for (int ks = 0; ks < BK / 4; ++ks) {
          const int kr = ks * 4 + (lane >> 4);
          double af[4], bf[4];
#pragma unroll
          for (int jj = 0; jj < 4; ++jj) bf[jj] = bs[kr * BN + wn * 64 + jj * 16 + (lane & 15)];
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            if (i < imin) continue;
            af[i] = as[kr * BM + (ILV ? (2 * i + wm) * 16 : wm * 64 + i * 16) + (lane & 15)];
#pragma unroll
            for (int jj = 0; jj < 4; ++jj)
              acc[i][jj] = __builtin_amdgcn_mfma_f64_16x16x4f64(af[i], bf[jj], acc[i][jj], 0, 0, 0);
          }
        }
      }
    }
    // epilogue: column sums of squares over the tile's 128 rows
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) {
      const int cl = wn * 64 + jj * 16 + (lane & 15);
      double s = 0.0;
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) s += acc[i][jj][r] * acc[i][jj][r];
      s += __shfl_xor(s, 16);
      s += __shfl_xor(s, 32);
      if ((lane >> 4) == 0) red[wm * BN + cl] = s;
    }
    __syncthreads();
    if (t < BN) {
      const int64_t col = col0 + t;
      if (col < m) part[(int64_t)rt * ldp + col] = red[t] + red[BN + t];
    }
  }
  if (t == 0 && clk) {
    clk[2 * blockIdx.x] = __builtin_amdgcn_s_memtime() - c0;
    clk[2 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime() - r0;
  }
}

#define V2INST(A, B, C, D, E)                                                                                          \
  template __global__ void k_var2<A, B, C, D, E>(const double*, int64_t, const double*, int64_t, int32_t, int32_t, int32_t, \
                                           int64_t, int32_t*, double*, int64_t, unsigned long long*);
V2INST(0, 16, 2, 0, 0)
V2INST(1, 16, 2, 0, 1)
V2INST(0, 16, 2, 0, 1)
V2INST(0, 8, 4, 0, 1)
V2INST(0, 8, 3, 0, 1)

// ---------------------------------------------------------------------------
// k_var3: no LDS staging, no per-stage barriers.  Each wave loads its own MFMA
// fragments from global memory (L1/L2) into registers, double-buffered one
// 16-k stage ahead, and runs independently of the other waves; the workgroup
// (2 x 2 waves on a 128 x 128 tile, rows interleaved) meets only at the item's
// ticket and epilogue.
// ---------------------------------------------------------------------------
template <int NOLOAD, int BK = 8, int TP = 0>
__global__ __launch_bounds__(256, 2) void k_var3(const double* __restrict__ AT, int64_t lda,
                                                 const double* __restrict__ B, int64_t ldb, int32_t K, int32_t RT,
                                                 int32_t CT, int64_t m, int32_t* __restrict__ ticket,
                                                 double* __restrict__ part, int64_t ldp,
                                                 unsigned long long* __restrict__ clk) {
  const unsigned long long c0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  constexpr int BM = 128, BN = 128, KS = BK / 4;
  __shared__ double red[2 * BN];
  __shared__ int32_t s_item, s_next;
  const int t = threadIdx.x, lane = t & 63;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const int wm = w >> 1, wn = w & 1;
  const int32_t xcd = blockIdx.x & 7;
  if (TP && t == 0) s_next = atomicAdd(&ticket[xcd], 1);
  for (;;) {
    if (!TP && t == 0) s_item = atomicAdd(&ticket[xcd], 1);
    __syncthreads();
    const int32_t j = TP ? s_next : s_item;
    __syncthreads();  // everyone has j before thread 0 overwrites s_next
    // TP: the next ticket is fetched now; its latency overlaps this item
    if (TP && t == 0) s_next = atomicAdd(&ticket[xcd], 1);
    const int32_t ct = (j / RT) * 8 + xcd;
    if (ct >= CT) break;
    const int32_t rt = RT - 1 - (j % RT);
    const int64_t col0 = (int64_t)ct * BN;
    const int32_t row0 = rt * BM;
    const int32_t nk = min(K, row0 + BM) / BK;
    const int32_t nfull = min(nk, row0 / BK);
    const double* ap = AT + (int64_t)(lane >> 4) * lda + row0 + wm * 16 + (lane & 15);
    const double* bp = B + (int64_t)(lane >> 4) * ldb + col0 + wn * 64 + (lane & 15);
    vd4 acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) acc[i][jj] = (vd4){0.0, 0.0, 0.0, 0.0};
    double fa0[KS][4], fb0[KS][4], fa1[KS][4], fb1[KS][4];  // [ks][i], [ks][jj]
    auto load = [&](double (&fa)[KS][4], double (&fb)[KS][4], int32_t kt) {
      if (NOLOAD) {
#pragma unroll
        for (int ks = 0; ks < KS; ++ks)
#pragma unroll
          for (int q = 0; q < 4; ++q) { fa[ks][q] = 1e-3 * (ks + q + kt); fb[ks][q] = 2e-3 * (ks - q); }
        return;
      }
      const int64_t ka = (int64_t)kt * BK * lda, kb = (int64_t)kt * BK * ldb;
#pragma unroll
      for (int ks = 0; ks < KS; ++ks)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          fa[ks][q] = ap[ka + (int64_t)ks * 4 * lda + q * 32];
          fb[ks][q] = bp[kb + (int64_t)ks * 4 * ldb + q * 16];
        }
    };
    auto compute = [&](const double (&fa)[KS][4], const double (&fb)[KS][4], int32_t kt) {
      int imin = 0;
      if (kt >= nfull) {
        const int z = ((kt - nfull) * BK) / 16 - wm;
        imin = z <= 0 ? 0 : (z + 1) >> 1;
      }
#pragma unroll
      for (int ks = 0; ks < KS; ++ks)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          if (i < imin) continue;
#pragma unroll
          for (int jj = 0; jj < 4; ++jj)
            acc[i][jj] = __builtin_amdgcn_mfma_f64_16x16x4f64(fa[ks][i], fb[ks][jj], acc[i][jj], 0, 0, 0);
        }
    };
    load(fa0, fb0, 0);
    for (int32_t kt = 0; kt < nk; kt += 2) {   // nk is a multiple of 8
      load(fa1, fb1, kt + 1);
      compute(fa0, fb0, kt);
      if (kt + 2 < nk) load(fa0, fb0, kt + 2);
      compute(fa1, fb1, kt + 1);
    }
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) {
      const int cl = wn * 64 + jj * 16 + (lane & 15);
      double s = 0.0;
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) s += acc[i][jj][r] * acc[i][jj][r];
      s += __shfl_xor(s, 16);
      s += __shfl_xor(s, 32);
      if ((lane >> 4) == 0) red[wm * BN + cl] = s;
    }
    __syncthreads();
    if (t < BN) {
      const int64_t col = col0 + t;
      if (col < m) part[(int64_t)rt * ldp + col] = red[t] + red[BN + t];
    }
  }
  if (t == 0 && clk) {
    clk[2 * blockIdx.x] = __builtin_amdgcn_s_memtime() - c0;
    clk[2 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime() - r0;
  }
}
template __global__ void k_var3<0, 8, 0>(const double*, int64_t, const double*, int64_t, int32_t, int32_t, int32_t, int64_t,
                                   int32_t*, double*, int64_t, unsigned long long*);
template __global__ void k_var3<0, 8, 1>(const double*, int64_t, const double*, int64_t, int32_t, int32_t, int32_t, int64_t,
                                   int32_t*, double*, int64_t, unsigned long long*);
template __global__ void k_var3<1, 8, 1>(const double*, int64_t, const double*, int64_t, int32_t, int32_t, int32_t, int64_t,
                                   int32_t*, double*, int64_t, unsigned long long*);

}  // namespace ut

using namespace ut;

#define CK(x)                                                                           \
  do {                                                                                  \
    hipError_t e = (x);                                                                 \
    if (e != hipSuccess) {                                                              \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e)); \
      exit(1);                                                                          \
    }                                                                                   \
  } while (0)

__global__ void k_fillr(double* p, int64_t n, uint64_t seed, int tri_ld) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint64_t x = (uint64_t)i * 0x9E3779B97F4A7C15ull + seed;
  x ^= x >> 31;
  x *= 0xBF58476D1CE4E5B9ull;
  x ^= x >> 29;
  double v = (double)(x >> 11) * (1.0 / 9007199254740992.0) - 0.5;
  if (tri_ld > 0) {  // (L^-1)^T [k][row]: zero for k > row
    int64_t k = i / tri_ld, r = i % tri_ld;
    if (k > r) v = 0.0;
  }
  p[i] = v;
}

int main(int argc, char** argv) {
  const int npad = argc > 1 ? atoi(argv[1]) : 1024;
  const int64_t m = argc > 2 ? atoll(argv[2]) : (1 << 20);
  const int reps = argc > 3 ? atoi(argv[3]) : 5;
  const int64_t ldk = ((m + 255) / 256) * 256;
  double *LT, *Kst, *part;
  CK(hipMalloc(&LT, sizeof(double) * npad * npad));
  CK(hipMalloc(&Kst, sizeof(double) * npad * ldk));
  const int RT = npad / 128;
  CK(hipMalloc(&part, sizeof(double) * RT * ldk));
  k_fillr<<<(npad * npad + 255) / 256, 256>>>(LT, (int64_t)npad * npad, 1, npad);
  k_fillr<<<(unsigned)(((int64_t)npad * ldk + 255) / 256), 256>>>(Kst, (int64_t)npad * ldk, 2, 0);
  CK(hipDeviceSynchronize());
  int32_t* ticket;
  CK(hipMalloc(&ticket, sizeof(int32_t) * 8));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const double flops = (double)m * npad * (npad + 1);
  const int CT = (int)(ldk / 256);
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  const int ncu = prop.multiProcessorCount;
  auto timeit = [&](const char* name, auto launch) {
    auto one = [&] {
      CK(hipMemsetAsync(ticket, 0, sizeof(int32_t) * 8, 0));
      launch();
    };
    one();
    CK(hipGetLastError());
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    for (int r = 0; r < reps; ++r) one();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    ms /= reps;
    printf("%-40s %9.3f ms  %7.2f TF/s  (%.1f%% of 78.6)\n", name, ms, flops / ms * 1e-9,
           flops / ms * 1e-9 / 78.6 * 100);
    fflush(stdout);
  };
#define PROBE(MODE, NAME)                                                                                  \
  timeit(NAME, [&] {                                                                                       \
    hipLaunchKernelGGL((k_probe<MODE>), dim3(ncu), dim3(V_NT), 0, 0, (const double*)LT, (int64_t)npad,      \
                       (const double*)Kst, ldk, npad, RT, CT, m, ticket, part, ldk);                       \
  })
  unsigned long long* clk;
  CK(hipMalloc(&clk, sizeof(unsigned long long) * 2 * 2 * ncu));
  auto clock_report = [&](int blocks) {
    std::vector<unsigned long long> h(2 * blocks);
    CK(hipMemcpy(h.data(), clk, sizeof(unsigned long long) * 2 * blocks, hipMemcpyDeviceToHost));
    std::vector<double> g;
    for (int b = 0; b < blocks; ++b) g.push_back((double)h[2 * b] / (double)h[2 * b + 1] * 0.1);
    std::sort(g.begin(), g.end());
    printf("    in-kernel clock median %.3f GHz (min %.3f max %.3f)\n", g[g.size() / 2], g.front(), g.back());
  };
  PROBE(0, "probe: as library");
  const int CT2 = (int)((m + 127) / 128);
#define PROBE2(A, B, C, D, E, NAME)                                                                                \
  timeit(NAME, [&] {                                                                                         \
    hipLaunchKernelGGL((k_var2<A, B, C, D, E>), dim3(2 * ncu), dim3(256), 0, 0, (const double*)LT, (int64_t)npad, \
                       (const double*)Kst, ldk, npad, RT, CT2, m, ticket, part, ldk, clk);                        \
  });                                                                                                           \
  clock_report(2 * ncu)
  PROBE2(0, 16, 2, 0, 0, "var2 BK16 NS2");
  std::vector<double> ref((size_t)RT * ldk), got((size_t)RT * ldk);
  CK(hipMemcpy(ref.data(), part, sizeof(double) * ref.size(), hipMemcpyDeviceToHost));
  PROBE2(0, 16, 2, 0, 1, "var2 BK16 NS2 interleaved");
  CK(hipMemcpy(got.data(), part, sizeof(double) * got.size(), hipMemcpyDeviceToHost));
  auto cmp = [&](const char* what) {
    double md = 0;
    for (size_t q = 0; q < ref.size(); ++q) md = std::max(md, std::abs(ref[q] - got[q]) / (std::abs(ref[q]) + 1e-300));
    printf("    %s vs plain: max rel diff %.3e\n", what, md);
  };
  cmp("interleaved");
#define PROBE3(A, C, NAME)                                                                                       \
  timeit(NAME, [&] {                                                                                         \
    hipLaunchKernelGGL((k_var3<A, 8, C>), dim3(2 * ncu), dim3(256), 0, 0, (const double*)LT, (int64_t)npad,         \
                       (const double*)Kst, ldk, npad, RT, CT2, m, ticket, part, ldk, clk);                        \
  });                                                                                                           \
  clock_report(2 * ncu)
  PROBE3(0, 0, "var3 register-direct, no barriers");
  PROBE3(0, 1, "var3 + ticket prefetch");
  CK(hipMemcpy(got.data(), part, sizeof(double) * got.size(), hipMemcpyDeviceToHost));
  cmp("var3 tp");
  PROBE3(1, 1, "var3 + ticket prefetch, no loads");
  return 0;
}
