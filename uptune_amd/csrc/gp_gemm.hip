// gp_gemm.hip -- the two dense contractions of GP scoring (the MFMA-bound
// stage of the path):
//
//   MODE 0 (K*):   C[n x m] = Xs[n x d] * (U/ell)[d x m]
//                  epilogue: k* = sf2 exp(-0.5 max(|xs|^2 + |us|^2 - 2C, 0)),
//                  store K*^T [n][ld] and the column partial  sum_j alpha_j k*_j
//   MODE 1 (var):  C[n x m] = L^-1[n x n] * K*^T[n x m]   (lower triangular:
//                  the K loop of row tile rt stops at (rt+1)*128)
//                  epilogue: column partial  sum_c C[c][i]^2
//                  (the library launches the persistent k_gp_var below for
//                  this; MODE 1 of k_gp_gemm2 stays as its reference form)
//
// Tile 128 x 128 per 256-thread workgroup (2 x 2 waves of 64 x 64), K step 32,
// global -> register prefetch of step t+1 while step t computes out of the
// other LDS buffer (one barrier per step).  A (Xs / L^-1) is small and
// L2/MALL resident; B (the candidate stream) is read along m with 16-byte
// loads.  Row tiles of one candidate column tile are dispatched
// consecutively inside one XCD group (blocks b, b+8, ... share an XCD) so the
// B column tile is fetched from HBM once and re-read from that XCD's L2.
//
//   fp64: v_mfma_f64_16x16x4_f64   (C/D: col = lane&15, row = (lane>>4) + 4r)
//   fp32: v_mfma_f32_32x32x2_f32   (C/D: col = lane&31, row = (r&3) + 8(r>>2) + 4(lane>>5))
#include "ut_internal.h"

namespace ut {

typedef double gd4 __attribute__((ext_vector_type(4)));
typedef float gf16 __attribute__((ext_vector_type(16)));

constexpr int G_BM = 128, G_BN = 128, G_NT = 256;

template <typename T>
struct GCfg;
template <>
struct GCfg<double> {
  static constexpr int BK = 16;          // 2 x 36 KB LDS buffers and ~200 VGPRs: 2 waves / SIMD
  static constexpr int LDA = G_BM + 16;  // row stride (elements) of As[k][row]: 288 dwords = 32 mod 64 banks
  static constexpr int LDB = G_BN + 16;
};
template <>
struct GCfg<float> {
  static constexpr int BK = 32;
  static constexpr int LDA = G_BM + 4;
  static constexpr int LDB = G_BN + 4;
};

template <typename T>
__device__ __forceinline__ T to_t(double v) {
  return (T)v;
}

// T: MFMA operand/accumulate type; TS: type K* is stored in (MODE 0).
template <typename T, int MODE, typename TS = T>
__global__ __launch_bounds__(G_NT, 2) void k_gp_gemm2(
    const T* __restrict__ A, int64_t lda, const void* __restrict__ Bv, int64_t ldb, int32_t K, int32_t RT,
    int32_t CT, int64_t m,
    // MODE 0
    const double* __restrict__ inv_ell, const double* __restrict__ xnorm, const double* __restrict__ cnorm,
    const double* __restrict__ alpha, double sf2, int32_t n, TS* __restrict__ kst, int64_t ldk,
    // column partials [RT][ldp]
    double* __restrict__ part, int64_t ldp) {
  constexpr int G_BK = GCfg<T>::BK, LDA = GCfg<T>::LDA, LDB = GCfg<T>::LDB;
  constexpr int PT = G_BK / 2;               // staged elements per thread for A and for B
  __shared__ __attribute__((aligned(16))) T As[2][G_BK * LDA];
  __shared__ __attribute__((aligned(16))) T Bs[2][G_BK * LDB];

  const int32_t b = blockIdx.x;
  const int32_t xcd = b & 7, jj = b >> 3;
  const int32_t rt = jj % RT;
  const int32_t ct = (jj / RT) * 8 + xcd;
  if (ct >= CT) return;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int wm = w >> 1, wn = w & 1;
  const int64_t col0 = (int64_t)ct * G_BN;
  const int32_t row0 = rt * G_BM;
  const int32_t kmax = (MODE == 1) ? min(K, row0 + G_BM) : K;
  const int32_t nk = (kmax + G_BK - 1) / G_BK;

  // staging maps
  const int ar = t >> 1, ak = (t & 1) * PT;   // A: row, first of PT k (2 threads per row)
  constexpr int TPK = G_BN / PT;              // B: threads per k row
  const int bk = t / TPK, bc = (t % TPK) * PT;
  const bool bfull = (col0 + G_BN) <= m;      // MODE 0: whole column tile in range

  T ra[PT], rb[PT];
  auto load = [&](int32_t k0) {
    // A
    if (MODE == 1) {
      const T* src = A + (int64_t)(row0 + ar) * lda + k0 + ak;
#pragma unroll
      for (int u = 0; u < PT; ++u) ra[u] = src[u];
    } else {
#pragma unroll
      for (int u = 0; u < PT; ++u) {
        const int32_t kk = k0 + ak + u;
        ra[u] = (kk < K) ? A[(int64_t)(row0 + ar) * lda + kk] : (T)0;
      }
    }
    // B
    const int32_t kk = k0 + bk;
    if (MODE == 1) {
      const T* src = reinterpret_cast<const T*>(Bv) + (int64_t)kk * ldb + col0 + bc;
#pragma unroll
      for (int u = 0; u < PT; ++u) rb[u] = src[u];
    } else {
      const double* src = reinterpret_cast<const double*>(Bv) + (int64_t)kk * ldb + col0 + bc;
      const double sc = (kk < K) ? inv_ell[kk] : 0.0;
      if (kk < K && bfull) {
#pragma unroll
        for (int u = 0; u < PT; ++u) rb[u] = to_t<T>(src[u] * sc);
      } else {
#pragma unroll
        for (int u = 0; u < PT; ++u) rb[u] = (kk < K && col0 + bc + u < m) ? to_t<T>(src[u] * sc) : (T)0;
      }
    }
  };
  auto store = [&](int buf) {
#pragma unroll
    for (int u = 0; u < PT; ++u) As[buf][(ak + u) * LDA + ar] = ra[u];
#pragma unroll
    for (int u = 0; u < PT; ++u) Bs[buf][bk * LDB + bc + u] = rb[u];
  };

  // accumulators: fp64 4x4 tiles of 16x16 (4 doubles), fp32 2x2 tiles of 32x32 (16 floats)
  gd4 accd[4][4];
  gf16 accf[2][2];
  if constexpr (sizeof(T) == 8) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) accd[i][j] = (gd4){0.0, 0.0, 0.0, 0.0};
  } else {
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) accf[i][j][r] = 0.0f;
  }

  load(0);
  store(0);
  __syncthreads();
  for (int32_t kt = 0; kt < nk; ++kt) {
    const int buf = kt & 1;
    if (kt + 1 < nk) load((kt + 1) * G_BK);
    const T* as = As[buf];
    const T* bs = Bs[buf];
    if constexpr (sizeof(T) == 8) {
#pragma unroll
      for (int ks = 0; ks < G_BK / 4; ++ks) {
        const int kr = ks * 4 + (lane >> 4);
        double af[4], bf[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) af[i] = as[kr * LDA + wm * 64 + i * 16 + (lane & 15)];
#pragma unroll
        for (int j = 0; j < 4; ++j) bf[j] = bs[kr * LDB + wn * 64 + j * 16 + (lane & 15)];
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) accd[i][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(af[i], bf[j], accd[i][j], 0, 0, 0);
      }
    } else {
#pragma unroll
      for (int ks = 0; ks < G_BK / 2; ++ks) {
        const int kr = ks * 2 + (lane >> 5);
        float af[2], bf[2];
#pragma unroll
        for (int i = 0; i < 2; ++i) af[i] = as[kr * LDA + wm * 64 + i * 32 + (lane & 31)];
#pragma unroll
        for (int j = 0; j < 2; ++j) bf[j] = bs[kr * LDB + wn * 64 + j * 32 + (lane & 31)];
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j) accf[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[i], bf[j], accf[i][j], 0, 0, 0);
      }
    }
    if (kt + 1 < nk) store(buf ^ 1);
    __syncthreads();
  }

  // ---- epilogue: per-column partial over this tile's 128 rows ----------------
  double* red = reinterpret_cast<double*>(&As[0][0]);  // [2][128], reused after the final barrier
  if constexpr (sizeof(T) == 8) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int cl = wn * 64 + j * 16 + (lane & 15);
      const int64_t col = col0 + cl;
      double s = 0.0;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int32_t row = row0 + wm * 64 + i * 16 + (lane >> 4) + 4 * r;
          const double x = accd[i][j][r];
          if (MODE == 0) {
            double ks = 0.0;
            if (row < n && col < m) {
              double d2 = xnorm[row] + cnorm[col] - 2.0 * x;
              d2 = d2 > 0.0 ? d2 : 0.0;
              ks = sf2 * exp(-0.5 * d2);
            }
            kst[(int64_t)row * ldk + col] = (TS)ks;
            s += alpha[row] * ks;
          } else {
            s += x * x;
          }
        }
      }
      s += __shfl_xor(s, 16);
      s += __shfl_xor(s, 32);
      if ((lane >> 4) == 0) red[wm * G_BN + cl] = s;
    }
  } else {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int cl = wn * 64 + j * 32 + (lane & 31);
      const int64_t col = col0 + cl;
      double s = 0.0;
#pragma unroll
      for (int i = 0; i < 2; ++i) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int32_t row = row0 + wm * 64 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
          const float x = accf[i][j][r];
          if (MODE == 0) {
            float ks = 0.0f;
            if (row < n && col < m) {
              double d2 = xnorm[row] + cnorm[col] - 2.0 * (double)x;
              d2 = d2 > 0.0 ? d2 : 0.0;
              ks = (float)sf2 * __expf(-0.5f * (float)d2);
            }
            kst[(int64_t)row * ldk + col] = (TS)ks;
            s += alpha[row] * (double)ks;
          } else {
            s += (double)x * (double)x;
          }
        }
      }
      s += __shfl_xor(s, 32);
      if ((lane >> 5) == 0) red[wm * G_BN + cl] = s;
    }
  }
  __syncthreads();
  if (t < G_BN) {
    const int64_t col = col0 + t;
    if (col < m) part[(int64_t)rt * ldp + col] = red[t] + red[G_BN + t];
  }
}

__global__ void k_to_f32(const double* __restrict__ src, float* __restrict__ dst, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) dst[i] = (float)src[i];
}

int launch_gemm_kstar(ut_ctx* c, bool fp32, const void* A, int64_t lda, const double* feat, int64_t ldf, int32_t d,
                      int32_t RT, int32_t CT, int64_t m, void* kst, int64_t ldk, double* part) {
  const int32_t CT8 = ((CT + 7) / 8) * 8;
  // fp32 mode: the small K* contraction stays fp64 (the |a|^2+|b|^2-2ab form
  // cancels), only its output is stored as fp32 for the large var contraction
  if (fp32)
    hipLaunchKernelGGL((k_gp_gemm2<double, 0, float>), dim3(RT * CT8), dim3(G_NT), 0, c->stream, (const double*)A,
                       lda, (const void*)feat, ldf, d, RT, CT, m, c->gp_inv_ell, c->gp_xnorm, c->cnorm.p, c->gp_alpha,
                       c->gp_sf2, c->gp_n, (float*)kst, ldk, part, ldk);
  else
    hipLaunchKernelGGL((k_gp_gemm2<double, 0>), dim3(RT * CT8), dim3(G_NT), 0, c->stream, (const double*)A, lda,
                       (const void*)feat, ldf, d, RT, CT, m, c->gp_inv_ell, c->gp_xnorm, c->cnorm.p, c->gp_alpha,
                       c->gp_sf2, c->gp_n, (double*)kst, ldk, part, ldk);
  UT_LAUNCH_CHECK(c);
  return 0;
}

// ---------------------------------------------------------------------------
// Variance contraction, persistent:  part[rt][col] = sum_{r in tile rt} (L^-1 K*^T)[r][col]^2
//
// One 512-thread workgroup per CU (8 waves as 2 x 4 of 64 x 64 outputs) walks
// (column strip, row tile) work items: 128 rows of L^-1 x 256 candidates, K
// loop over [0, (rt+1)*128) (L^-1 is lower triangular).  Work items of XCD
// group x (blocks b = x mod 8) are the column strips ct = x mod 8, handed out
// by a per-group atomic ticket, the longest row tile of a strip first; the 8
// row tiles of a strip therefore run side by side on one XCD and share the
// strip through its L2.  Tiles are staged by global_load_lds_dwordx4 (1 KiB
// per wave-instruction, lane-linear LDS image) into a 3-deep ring: step kt+1
// stays in flight across the barrier of step kt (counted vmcnt, raw barrier).
// A non-persistent grid of these tiles left CUs idle ~30% of the time: the
// in-order workgroup dispatcher stalls behind long (late row) tiles.
//   A = (L^-1)^T [k][row] (ld npad), B = K*^T [k][col] (ld ldk, ldk % 256 == 0)
//   fp64: v_mfma_f64_16x16x4_f64, BK 16;  fp32: v_mfma_f32_32x32x2_f32, BK 32
// ---------------------------------------------------------------------------
constexpr int V_NT = 512, V_ST = 3;

template <typename T>
struct VCfg {
  static constexpr int BK = 64 / (int)sizeof(T) * 2;  // 16 (f64), 32 (f32): 16 KiB A + 32 KiB B per stage
  static constexpr int SA = BK * VAR_BM, SB = BK * VAR_BN, STAGE = SA + SB;
  static constexpr int PER_INSTR = 1024 / (int)sizeof(T);  // elements one glds wave-instruction moves
};

template <typename T>
__device__ __forceinline__ void var_issue(const T* __restrict__ AT, int64_t lda, const T* __restrict__ B, int64_t ldb,
                                          int32_t row0, int64_t col0, int32_t k0, T* st, int w, int lane) {
  using C = VCfg<T>;
  constexpr int EPL = 16 / (int)sizeof(T);  // elements per lane
  // wave w: A instructions 2w, 2w+1 (16 in all), B instructions 4w .. 4w+3 (32 in all)
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int q = 2 * w + u;
    const int e = q * C::PER_INSTR + lane * EPL;  // linear index in the [BK][BM] tile
    const T* src = AT + (int64_t)(k0 + e / VAR_BM) * lda + row0 + (e % VAR_BM);
    __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)(st + q * C::PER_INSTR), 16, 0, 0);
  }
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int q = 4 * w + u;
    const int e = q * C::PER_INSTR + lane * EPL;  // linear index in the [BK][BN] tile
    const T* src = B + (int64_t)(k0 + e / VAR_BN) * ldb + col0 + (e % VAR_BN);
    __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)(st + C::SA + q * C::PER_INSTR), 16,
                                     0, 0);
  }
}

template <typename T>
__global__ __launch_bounds__(V_NT, 1) void k_gp_var(const T* __restrict__ AT, int64_t lda, const T* __restrict__ B,
                                                     int64_t ldb, int32_t K, int32_t RT, int32_t CT, int64_t m,
                                                     int32_t* __restrict__ ticket, double* __restrict__ part,
                                                     int64_t ldp) {
  using C = VCfg<T>;
  constexpr int BK = C::BK;
  // ALL LDS in one object: a second __shared__ beside the glds ring makes
  // hipcc wait vmcnt(0) before every step's first ds_read (drains the ring)
  __shared__ __attribute__((aligned(16))) T lds[V_ST * C::STAGE + 16 / sizeof(T)];
  int32_t& s_item = *reinterpret_cast<int32_t*>(lds + V_ST * C::STAGE);
  const int t = threadIdx.x, lane = t & 63;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const int wm = w >> 2, wn = w & 3;
  const int32_t xcd = blockIdx.x & 7;

  for (;;) {
    if (t == 0) s_item = atomicAdd(&ticket[xcd], 1);
    __syncthreads();  // also: the previous item's epilogue is done with the LDS
    const int32_t j = s_item;
    const int32_t ct = (j / RT) * 8 + xcd;
    if (ct >= CT) break;  // uniform: every wave of the block leaves together
    const int32_t rt = RT - 1 - (j % RT);
    const int64_t col0 = (int64_t)ct * VAR_BN;
    const int32_t row0 = rt * VAR_BM;
    const int32_t nk = min(K, row0 + VAR_BM) / BK;

    typedef double d4 __attribute__((ext_vector_type(4)));
    typedef float f16 __attribute__((ext_vector_type(16)));
    d4 accd[4][4];
    f16 accf[2][2];
    if constexpr (sizeof(T) == 8) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) accd[i][jj] = (d4){0.0, 0.0, 0.0, 0.0};
    } else {
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int jj = 0; jj < 2; ++jj)
#pragma unroll
          for (int r = 0; r < 16; ++r) accf[i][jj][r] = 0.0f;
    }

    var_issue<T>(AT, lda, B, ldb, row0, col0, 0, lds, w, lane);
    if (nk > 1) var_issue<T>(AT, lda, B, ldb, row0, col0, BK, lds + C::STAGE, w, lane);
    for (int32_t kt = 0; kt < nk; ++kt) {
      // 6 glds per wave per stage: leave stage kt+1 in flight, retire stage kt
      if (kt + 1 < nk)
        asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
      else
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();  // all waves' stage kt landed; all reads of stage kt-1 done
      asm volatile("" ::: "memory");
      if (kt + 2 < nk)
        var_issue<T>(AT, lda, B, ldb, row0, col0, (kt + 2) * BK, lds + ((kt + 2) % V_ST) * C::STAGE, w, lane);
      const T* as = lds + (kt % V_ST) * C::STAGE;
      const T* bs = as + C::SA;
      if constexpr (sizeof(T) == 8) {
#pragma unroll
        for (int ks = 0; ks < BK / 4; ++ks) {
          const int kr = ks * 4 + (lane >> 4);
          double af[4], bf[4];
#pragma unroll
          for (int i = 0; i < 4; ++i) af[i] = as[kr * VAR_BM + wm * 64 + i * 16 + (lane & 15)];
#pragma unroll
          for (int jj = 0; jj < 4; ++jj) bf[jj] = bs[kr * VAR_BN + wn * 64 + jj * 16 + (lane & 15)];
#pragma unroll
          for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int jj = 0; jj < 4; ++jj)
              accd[i][jj] = __builtin_amdgcn_mfma_f64_16x16x4f64(af[i], bf[jj], accd[i][jj], 0, 0, 0);
        }
      } else {
#pragma unroll
        for (int ks = 0; ks < BK / 2; ++ks) {
          const int kr = ks * 2 + (lane >> 5);
          float af[2], bf[2];
#pragma unroll
          for (int i = 0; i < 2; ++i) af[i] = as[kr * VAR_BM + wm * 64 + i * 32 + (lane & 31)];
#pragma unroll
          for (int jj = 0; jj < 2; ++jj) bf[jj] = bs[kr * VAR_BN + wn * 64 + jj * 32 + (lane & 31)];
#pragma unroll
          for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int jj = 0; jj < 2; ++jj)
              accf[i][jj] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[i], bf[jj], accf[i][jj], 0, 0, 0);
        }
      }
    }

    // epilogue: column sums of squares over this tile's 128 rows
    __syncthreads();
    double* red = reinterpret_cast<double*>(lds);  // [2][256]
    if constexpr (sizeof(T) == 8) {
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) {
        const int cl = wn * 64 + jj * 16 + (lane & 15);
        double s = 0.0;
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int r = 0; r < 4; ++r) s += accd[i][jj][r] * accd[i][jj][r];
        s += __shfl_xor(s, 16);
        s += __shfl_xor(s, 32);
        if ((lane >> 4) == 0) red[wm * VAR_BN + cl] = s;
      }
    } else {
#pragma unroll
      for (int jj = 0; jj < 2; ++jj) {
        const int cl = wn * 64 + jj * 32 + (lane & 31);
        double s = 0.0;
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int r = 0; r < 16; ++r) s += (double)accf[i][jj][r] * (double)accf[i][jj][r];
        s += __shfl_xor(s, 32);
        if ((lane >> 5) == 0) red[wm * VAR_BN + cl] = s;
      }
    }
    __syncthreads();
    if (t < VAR_BN) {
      const int64_t col = col0 + t;
      if (col < m) part[(int64_t)rt * ldp + col] = red[t] + red[VAR_BN + t];
    }
  }
}

int launch_gemm_var(ut_ctx* c, bool fp32, const void* LinvT, int64_t lda, const void* kst, int64_t ldk, int32_t npad,
                    int64_t m, double* part) {
  UT_CHECK(c, npad % VAR_BM == 0 && ldk % VAR_BN == 0 && ldk >= m, UT_EINVAL, "gemm_var: bad padding");
  const int32_t RT = npad / VAR_BM;
  const int32_t CT = (int32_t)((m + VAR_BN - 1) / VAR_BN);
  const int64_t items = (int64_t)RT * CT;
  // one block per CU (the 144 KiB LDS ring allows no more), a multiple of 8 so
  // every XCD group has workers; never more blocks than work items
  int32_t nb = (c->n_cu / 8) * 8;
  if (items < nb) nb = (int32_t)(((items + 7) / 8) * 8);
  UT_HIP(c, hipMemsetAsync(c->gp_ctr, 0, sizeof(int32_t) * 8, c->stream));
  if (fp32)
    hipLaunchKernelGGL(k_gp_var<float>, dim3(nb), dim3(V_NT), 0, c->stream, (const float*)LinvT, lda,
                       (const float*)kst, ldk, npad, RT, CT, m, c->gp_ctr, part, ldk);
  else
    hipLaunchKernelGGL(k_gp_var<double>, dim3(nb), dim3(V_NT), 0, c->stream, (const double*)LinvT, lda,
                       (const double*)kst, ldk, npad, RT, CT, m, c->gp_ctr, part, ldk);
  UT_LAUNCH_CHECK(c);
  return 0;
}

// dst[c][r] = src[r][c] (n x n, n % 64 == 0), optionally also as fp32
__global__ __launch_bounds__(256) void k_transpose(const double* __restrict__ src, int32_t n, double* __restrict__ dst,
                                                   float* __restrict__ dst_f) {
  __shared__ double tile[64][65];
  const int32_t r0 = blockIdx.y * 64, c0 = blockIdx.x * 64;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  for (int r = ty; r < 64; r += 4) tile[r][tx] = src[(int64_t)(r0 + r) * n + c0 + tx];
  __syncthreads();
  for (int r = ty; r < 64; r += 4) {
    const double v = tile[tx][r];
    dst[(int64_t)(c0 + r) * n + r0 + tx] = v;
    if (dst_f) dst_f[(int64_t)(c0 + r) * n + r0 + tx] = (float)v;
  }
}

int launch_transpose(ut_ctx* c, const double* src, int32_t n, double* dst, float* dst_f) {
  UT_CHECK(c, n % 64 == 0, UT_EINVAL, "transpose: n % 64 != 0");
  hipLaunchKernelGGL(k_transpose, dim3(n / 64, n / 64), dim3(256), 0, c->stream, src, n, dst, dst_f);
  UT_LAUNCH_CHECK(c);
  return 0;
}

int launch_to_f32(ut_ctx* c, const double* src, float* dst, int64_t n) {
  hipLaunchKernelGGL(k_to_f32, dim3(grid1(n, 256)), dim3(256), 0, c->stream, src, dst, n);
  UT_LAUNCH_CHECK(c);
  return 0;
}

}  // namespace ut
