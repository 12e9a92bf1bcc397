// gp.hip -- Gaussian-process surrogate (fit + batched posterior + acquisition).
//
// No reference arithmetic exists for this stage; the spec is
// SURVEY.md §8(a) row a7 / "GP spec for a7":
//   features u (unit encoding), us = u / ell (ARD), y standardised,
//   K = sf2 * exp(-0.5 |xs_i - xs_j|^2) + (sn2 + jitter) I,  L = chol(K),
//   alpha = K^-1 ys,  k* = sf2 * exp(-0.5 |us - xs_j|^2)  (via |a|^2+|b|^2-2ab),
//   mu = k*.alpha,  var = max(sf2 - |L^-1 k*|^2, 0),
//   EI = I Phi(I/sigma) + sigma phi(I/sigma), I = f_best - mu - xi  (max(I,0) if sigma == 0)
//   UCB score = kappa * sigma - mu
// The fp64 oracle is oracle/gp.py.
//
// Fit (per round, O(n^3), small): blocked right-looking Cholesky (NB = 64,
// panel factor + solve in LDS, trailing update tiles), blocked triangular
// inverse by block rows, two mat-vecs for alpha.
//
// Score (per candidate, the MFMA-bound stage): both dense contractions are
//   C[n x m] = A[n x K] * B[K x m]
// with A small and row-major (L2/MALL resident) and B the candidate-major
// stream (columns = candidates, coalesced along m):
//   GEMM1: A = Xs [n x d],    B = U^T (features, [d][m]) -> K*^T  [n][m] + mu partials
//   GEMM2: A = L^-1 [n x n],  B = K*^T [n][m]  (lower-triangular A: K loop stops
//          at the tile's diagonal)  -> |L^-1 k*|^2 partials
// Both run in gp_gemm.hip (fp64 MFMA by default, fp32 MFMA when
// ut_gp_set_precision(ctx, 32); with 16 the variance GEMM runs as three fp16
// MFMA products of hi/lo split operands, fp32-class accuracy).
#include <cstring>

#include <thread>

#include "ut_internal.h"

namespace ut {

constexpr int NB = 64;     // Cholesky / inverse block
constexpr int NPAD = 128;  // training set padded to the GEMM row tile

// ---------------------------------------------------------------------------
// fit
// ---------------------------------------------------------------------------
// The fit's kernels are a chain of small, latency-bound launches on the fit
// stream, beside the round's hash / proposal / encode on the other streams.
// With g_fit_prio set (UT_FIT_SETPRIO) every fit wave raises its issue
// priority (s_setprio 3): where it shares a SIMD with the hash's waves, its
// instructions go first.
__device__ int32_t g_fit_prio = 0;
__device__ __forceinline__ void fit_prio() {
  if (g_fit_prio) __builtin_amdgcn_s_setprio(3);
}

int set_fit_prio(int32_t on) {
  if (hipMemcpyToSymbol(HIP_SYMBOL(g_fit_prio), &on, sizeof(on)) != hipSuccess) return UT_EHIP;
  return set_fit_prio_gemm(on);
}

__global__ void k_gp_prep_train(const double* __restrict__ X, int32_t n, int32_t npad, int32_t d,
                                const double* __restrict__ inv_ell, double* __restrict__ Xs,
                                double* __restrict__ xnorm) {
  fit_prio();
  const int32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= npad) return;
  double s = 0.0;
  for (int32_t k = 0; k < d; ++k) {
    const double v = (j < n) ? X[(int64_t)j * d + k] * inv_ell[k] : 0.0;
    Xs[(int64_t)j * d + k] = v;
    s += v * v;
  }
  xnorm[j] = s;
}

// categorical K* operands of the training rows (gp_gemm.hip "Categorical K*"):
// XsT_num [dpad_num][npad] = the numeric features of Xs, transposed, and their
// norms in feature order; one thread per row
__global__ void k_gp_num_train(const double* __restrict__ Xs, int32_t npad, int32_t d,
                               const int32_t* __restrict__ num_feat, int32_t n_num, int32_t dpad_num,
                               double* __restrict__ XsT_num, double* __restrict__ xnorm_num) {
  fit_prio();
  const int32_t r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= npad) return;
  double s = 0.0;
  for (int32_t k = 0; k < dpad_num; ++k) {
    const double v = k < n_num ? Xs[(int64_t)r * d + num_feat[k]] : 0.0;
    XsT_num[(int64_t)k * npad + r] = v * KSTAR_T_SCALE;   // the K* operand, in 2^(1/256) units (gp_gemm.hip)
    s += v * v;
  }
  xnorm_num[r] = s;
}

// the training rows' weighted one-hot codes [cat_k / 128][npad][128] (zeroed
// before): ENUM option o -> 2 at code column ccol + o, BOOL b -> 1 at ccol + b;
// X (unscaled features, rows < n) was checked one-hot on the host
__global__ void k_gp_cat_train(const DevParam* __restrict__ params, int32_t P, const int32_t* __restrict__ cat_ccol,
                               const double* __restrict__ X, int32_t n, int32_t d, int32_t npad,
                               int8_t* __restrict__ acat) {
  fit_prio();
  const int32_t r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= n) return;
  for (int32_t p = 0; p < P; ++p) {
    const int32_t cc = cat_ccol[p];
    if (cc < 0) continue;
    const DevParam pr = params[p];
    const double* x = X + (int64_t)r * d + pr.feat_col;
    int32_t o = 0;
    if (pr.kind == UT_BOOL) {
      o = x[0] != 0.0 ? 1 : 0;
    } else {
      for (int32_t k = 0; k < (int32_t)pr.n_opt; ++k)
        if (x[k] == 1.0) { o = k; break; }
    }
    const int32_t q = cc + o;
    acat[((int64_t)(q >> 7) * npad + r) * 128 + (q & 127)] = (int8_t)(pr.kind == UT_BOOL ? 1 : 2);
  }
}

// mean / std (ddof=0) / standardise / f_best = min(ys); one workgroup
__global__ __launch_bounds__(256) void k_gp_ystats(const double* __restrict__ y, int32_t n, int32_t npad,
                                                   double* __restrict__ ys, double* __restrict__ stats) {
  fit_prio();
  __shared__ double red[256];
  const int t = threadIdx.x;
  double s = 0.0;
  for (int32_t i = t; i < n; i += 256) s += y[i];
  red[t] = s;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if (t < w) red[t] += red[t + w];
    __syncthreads();
  }
  const double mean = red[0] / (double)n;
  __syncthreads();
  s = 0.0;
  for (int32_t i = t; i < n; i += 256) {
    const double dlt = y[i] - mean;
    s += dlt * dlt;
  }
  red[t] = s;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if (t < w) red[t] += red[t + w];
    __syncthreads();
  }
  double sd = sqrt(red[0] / (double)n);
  if (!(sd > 0.0)) sd = 1.0;
  __syncthreads();
  double mn = 1.0 / 0.0;
  for (int32_t i = t; i < npad; i += 256) {
    const double v = (i < n) ? (y[i] - mean) / sd : 0.0;
    ys[i] = v;
    if (i < n) mn = v < mn ? v : mn;
  }
  red[t] = mn;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if (t < w) red[t] = red[t + w] < red[t] ? red[t + w] : red[t];
    __syncthreads();
  }
  if (t == 0) {
    stats[0] = red[0];
    stats[1] = mean;
    stats[2] = sd;
  }
}

// 64 x 64 tile  acc = A[64 x K] * B[64 x K]^T  (both row-major in global,
// leading dims lda / ldb) on v_mfma_f64_16x16x4; each wave 32 x 32.
typedef double fd4 __attribute__((ext_vector_type(4)));
__device__ void tile64_nt(const double* __restrict__ A, int64_t lda, const double* __restrict__ B, int64_t ldb,
                          int32_t K, double* As, double* Bs, fd4 (&acc)[2][2]) {
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int wr = w >> 1, wc = w & 1;
  for (int32_t k0 = 0; k0 < K; k0 += 16) {
    for (int e = t; e < 64 * 16; e += 256) {
      const int r = e >> 4, kk = e & 15;
      const bool in = (k0 + kk) < K;
      As[kk * 80 + r] = in ? A[(int64_t)r * lda + k0 + kk] : 0.0;
      Bs[kk * 80 + r] = in ? B[(int64_t)r * ldb + k0 + kk] : 0.0;
    }
    __syncthreads();
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      const int kr = ks * 4 + (lane >> 4);
      double af[2], bf[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) af[i] = As[kr * 80 + wr * 32 + i * 16 + (lane & 15)];
#pragma unroll
      for (int j = 0; j < 2; ++j) bf[j] = Bs[kr * 80 + wc * 32 + j * 16 + (lane & 15)];
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(af[i], bf[j], acc[i][j], 0, 0, 0);
    }
    __syncthreads();
  }
}

// acc element (i, j, r) -> tile row / column
__device__ __forceinline__ int tile_row(int i, int r) { return ((threadIdx.x >> 6) >> 1) * 32 + i * 16 + ((threadIdx.x & 63) >> 4) + 4 * r; }
__device__ __forceinline__ int tile_col(int j) { return ((threadIdx.x >> 6) & 1) * 32 + j * 16 + (threadIdx.x & 15); }

// Panel kb, step 1 (one workgroup): L_kk = chol(A_kk) written to K, and
// inv(L_kk) written as the diagonal block of L^-1.
//
// This is the serial spine of the fit (NB column steps, then NB substitution
// steps, per diagonal block), so every step is kept short.  Thread t owns row
// r = t & 63 and columns 16 g .. 16 g + 15 of the block (g = wave) in
// registers.  Cholesky step c: the wave that owns column c takes the pivot by
// readlane, scales its column and publishes l = L[:, c] (0 above the
// diagonal) in a double-buffered LDS column; after ONE barrier every wave
// applies the rank-1 update a[j] -= l_r l_s to its 16 columns.  Entries above
// the diagonal are updated as well but never read.  The inverse solves
// L X = I for all 64 columns at once, each wave its 16 columns with no
// barrier: step s broadcasts row s of the partial solution by readlane.
// (The previous LDS version took 122 us per block at n = 1024, 70% of the fit.)
__device__ __forceinline__ double readlane_f64(double v, int lane) {
  const uint64_t u = __builtin_bit_cast(uint64_t, v);
  const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)u, lane);
  const uint32_t hi = __builtin_amdgcn_readlane((uint32_t)(u >> 32), lane);
  return __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
}

// the diagonal block kb from a[] (thread t: row t & 63, columns 16 (t >> 6) ..
// + 15 of the updated block); col [2][NB], Ls [NB][NB + 1], invd [NB] in LDS.
// MERGED (ut_ctx::chol_merged): the substitution for inv(L_kk) runs inside the
// column loop instead of after it: at step c, row c of the solution is final
// (its accumulator took every earlier column's update), so each wave reads it
// from lane c and applies column c of L to the rows below, behind the same
// barrier as the factor's rank-1 update.  The same operations in the same
// order as the separate sweep (x_c = acc_c * (1 / piv_c), acc_r -= l_r x_c by
// fma, the rows' final scaling by 1 / piv_r), so the same bits, with 64 steps
// of latency fewer.
template <bool MERGED>
__device__ __forceinline__ void chol_diag_core(double (&a)[16], double* __restrict__ K, double* __restrict__ Li,
                                               int32_t npad, int32_t kb, int32_t* flag, double (*col)[NB],
                                               double* Ls, double* invd) {
  const int t = threadIdx.x, r = t & 63;
  const int g = __builtin_amdgcn_readfirstlane(t >> 6);
  const int64_t base = (int64_t)kb * NB;
  double* rowp = K + (base + r) * npad + base + 16 * g;
  if constexpr (MERGED) {
    double b[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) b[j] = (16 * g + j == r) ? 1.0 : 0.0;
    for (int cb = 0; cb < NB / 16; ++cb) {
#pragma unroll
      for (int cc = 0; cc < 16; ++cc) {
        const int c = 16 * cb + cc;
        double* cl = col[c & 1];
        if (g == cb) {  // wave-uniform: the owner of column c
          const double dv = readlane_f64(a[cc], c);
          if (r == 0 && !(dv > 0.0)) atomicOr(flag, 1);
          const double piv = sqrt(dv > 0.0 ? dv : 1e-300);
          const double ip = 1.0 / piv;
          const double l = a[cc] * ip;
          cl[r] = r > c ? l : 0.0;
          if (r == 0) invd[c] = ip;
          a[cc] = r > c ? l : (r == c ? piv : a[cc]);
        }
        __syncthreads();  // column c published; the buffer written at step c+1 was last read at step c-1
        const double lr = cl[r];
        const double is = invd[c];
#pragma unroll
        for (int j = 0; j < 16; ++j) a[j] = __builtin_fma(-lr, cl[16 * g + j], a[j]);
#pragma unroll
        for (int j = 0; j < 16; ++j) b[j] = __builtin_fma(-lr, readlane_f64(b[j], c) * is, b[j]);
      }
    }
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const int sc = 16 * g + j;
      rowp[j] = sc <= r ? a[j] : 0.0;
    }
    const double ir = invd[r];   // written at step r, behind that step's barrier
    double* lip = Li + (base + r) * npad + base + 16 * g;
#pragma unroll
    for (int j = 0; j < 16; ++j) lip[j] = b[j] * ir;
    return;
  }
  for (int cb = 0; cb < NB / 16; ++cb) {
#pragma unroll
    for (int cc = 0; cc < 16; ++cc) {
      const int c = 16 * cb + cc;
      double* cl = col[c & 1];
      if (g == cb) {  // wave-uniform: the owner of column c
        const double dv = readlane_f64(a[cc], c);
        if (r == 0 && !(dv > 0.0)) atomicOr(flag, 1);
        const double piv = sqrt(dv > 0.0 ? dv : 1e-300);
        const double l = a[cc] * (1.0 / piv);
        cl[r] = r > c ? l : 0.0;
        a[cc] = r > c ? l : (r == c ? piv : a[cc]);
      }
      __syncthreads();  // column c published; the buffer written at step c+1 was last read at step c-1
      const double lr = cl[r];
#pragma unroll
      for (int j = 0; j < 16; ++j) a[j] = __builtin_fma(-lr, cl[16 * g + j], a[j]);
    }
  }
  // L to K (zeros above the diagonal) and to LDS for the substitution
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const int sc = 16 * g + j;
    const double v = sc <= r ? a[j] : 0.0;
    rowp[j] = v;
    Ls[r * (NB + 1) + sc] = v;
  }
  __syncthreads();
  if (t < NB) invd[t] = 1.0 / Ls[t * (NB + 1) + t];
  __syncthreads();
  // forward substitution L X = I, columns 16 g .. 16 g + 15 of X in b[]
  double b[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) b[j] = (16 * g + j == r) ? 1.0 : 0.0;
  for (int s2 = 0; s2 < NB; ++s2) {
    const double lrs = r > s2 ? Ls[r * (NB + 1) + s2] : 0.0;
    const double is = invd[s2];
#pragma unroll
    for (int j = 0; j < 16; ++j) b[j] = __builtin_fma(-lrs, readlane_f64(b[j], s2) * is, b[j]);
  }
  const double ir = invd[r];
  double* lip = Li + (base + r) * npad + base + 16 * g;
#pragma unroll
  for (int j = 0; j < 16; ++j) lip[j] = b[j] * ir;
}

template <bool MERGED>
__global__ __launch_bounds__(256) void k_chol_diag(double* __restrict__ K, double* __restrict__ Li, int32_t npad,
                                                   int32_t kb, int32_t* flag) {
  fit_prio();
  __shared__ double col[2][NB];
  __shared__ double Ls[NB * (NB + 1)];
  __shared__ double invd[NB];
  const int t = threadIdx.x, r = t & 63;
  const int g = __builtin_amdgcn_readfirstlane(t >> 6);
  const int64_t base = (int64_t)kb * NB;
  const double* rowp = K + (base + r) * npad + base + 16 * g;
  double a[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) a[j] = rowp[j];
  chol_diag_core<MERGED>(a, K, Li, npad, kb, flag, col, Ls, invd);
}

// Panel kb, step 2: row block i > kb:  L_ik = A_ik * inv(L_kk)^T  (NT product)
__global__ __launch_bounds__(256) void k_chol_rows(double* __restrict__ K, const double* __restrict__ Li,
                                                   int32_t npad, int32_t kb) {
  fit_prio();
  __shared__ double As[16 * 80];
  __shared__ double Bs[16 * 80];
  const int64_t base = (int64_t)kb * NB, rb = (int64_t)(kb + 1 + blockIdx.x) * NB;
  fd4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = (fd4){0.0, 0.0, 0.0, 0.0};
  tile64_nt(K + rb * npad + base, npad, Li + base * npad + base, npad, NB, As, Bs, acc);
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) K[(rb + tile_row(i, r)) * npad + base + tile_col(j)] = acc[i][j][r];
}

// Trailing update A_ij -= L_i,kb L_j,kb^T for kb < j <= i < nb.
__global__ __launch_bounds__(256) void k_chol_update(double* __restrict__ K, int32_t npad, int32_t kb) {
  fit_prio();
  __shared__ double As[16 * 80];
  __shared__ double Bs[16 * 80];
  int32_t tid = blockIdx.x;
  int32_t i = 0;
  while ((i + 1) * (i + 2) / 2 <= tid) ++i;
  const int32_t j = tid - i * (i + 1) / 2;
  const int64_t ib = (int64_t)(kb + 1 + i) * NB, jb = (int64_t)(kb + 1 + j) * NB, cb = (int64_t)kb * NB;
  fd4 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) acc[a][b] = (fd4){0.0, 0.0, 0.0, 0.0};
  tile64_nt(K + ib * npad + cb, npad, K + jb * npad + cb, npad, NB, As, Bs, acc);
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int r = 0; r < 4; ++r) K[(ib + tile_row(a, r)) * npad + jb + tile_col(b)] -= acc[a][b][r];
}

// k_chol_update with the next panel's diagonal block factored in the same
// launch: the workgroup that updates block (kb + 1, kb + 1) keeps it in LDS
// and runs k_chol_diag's steps on it while the others update the rest, so the
// fit's serial chain loses one launch per level (ut_ctx::chol_fuse)
template <bool MERGED>
__global__ __launch_bounds__(256) void k_chol_update_diag(double* __restrict__ K, double* __restrict__ Li,
                                                          int32_t npad, int32_t kb, int32_t* flag) {
  fit_prio();
  // As / Bs of the tile product, then (workgroup 0) Ls, col, invd of the diagonal block
  __shared__ double sm[NB * (NB + 1) + 2 * NB + NB];
  double* As = sm;
  double* Bs = sm + 16 * 80;
  const int32_t tid = blockIdx.x;
  int32_t i = 0;
  while ((i + 1) * (i + 2) / 2 <= tid) ++i;
  const int32_t j = tid - i * (i + 1) / 2;
  const int64_t ib = (int64_t)(kb + 1 + i) * NB, jb = (int64_t)(kb + 1 + j) * NB, cb = (int64_t)kb * NB;
  fd4 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) acc[a][b] = (fd4){0.0, 0.0, 0.0, 0.0};
  tile64_nt(K + ib * npad + cb, npad, K + jb * npad + cb, npad, NB, As, Bs, acc);
  if (tid != 0) {
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int r = 0; r < 4; ++r) K[(ib + tile_row(a, r)) * npad + jb + tile_col(b)] -= acc[a][b][r];
    return;
  }
  // block (kb + 1, kb + 1): the updated values (the same arithmetic as the
  // store above) into LDS, then the diagonal steps on them
  double* Ls = sm;
  double(*col)[NB] = reinterpret_cast<double(*)[NB]>(sm + NB * (NB + 1));
  double* invd = sm + NB * (NB + 1) + 2 * NB;
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int tr = tile_row(a, r), tc = tile_col(b);
        Ls[tr * (NB + 1) + tc] = K[(ib + tr) * npad + jb + tc] - acc[a][b][r];
      }
  __syncthreads();
  const int t = threadIdx.x, rr = t & 63, g = t >> 6;
  double av[16];
#pragma unroll
  for (int q = 0; q < 16; ++q) av[q] = Ls[rr * (NB + 1) + 16 * g + q];
  __syncthreads();   // Ls is rewritten by the substitution's setup
  chol_diag_core<MERGED>(av, K, Li, npad, kb + 1, flag, col, Ls, invd);
}

// K = sf2 exp(-0.5 |xs_i - xs_j|^2) + diag I, 64 x 64 tiles on fp64 MFMA;
// padded rows/columns (>= n) form an identity block; block rows from rb0 on
__global__ __launch_bounds__(256) void k_gp_kmat(const double* __restrict__ Xs, const double* __restrict__ xnorm,
                                                 int32_t n, int32_t npad, int32_t d, double sf2, double diag,
                                                 double* __restrict__ K, int32_t rb0) {
  fit_prio();
  __shared__ double As[16 * 80];
  __shared__ double Bs[16 * 80];
  const int64_t ib = (int64_t)(blockIdx.y + rb0) * 64, jb = (int64_t)blockIdx.x * 64;
  fd4 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) acc[a][b] = (fd4){0.0, 0.0, 0.0, 0.0};
  tile64_nt(Xs + ib * d, d, Xs + jb * d, d, d, As, Bs, acc);
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t i = ib + tile_row(a, r), j = jb + tile_col(b);
        double v;
        if (i >= n || j >= n) {
          v = (i == j) ? 1.0 : 0.0;
        } else {
          double d2 = xnorm[i] + xnorm[j] - 2.0 * acc[a][b][r];
          d2 = d2 > 0.0 ? d2 : 0.0;
          v = sf2 * exp(-0.5 * d2);
          if (i == j) v += diag;
        }
        K[i * npad + j] = v;
      }
}

// Batched fp64 GEMM for the recursive triangular inverse.  Pair z at level
// size s (offset o = z * 2s):
//   phase 0:  T_z = B * Ai     B = L[o+s:o+2s, o:o+s],  Ai = Li[o:o+s, o:o+s]  (lower)
//   phase 1:  Li[o+s:o+2s, o:o+s] = -Ci * T_z            Ci = Li[o+s:o+2s, o+s:o+2s]  (lower)
// 64 x 64 output tile per 256-thread workgroup, v_mfma_f64_16x16x4 (each
// wave 32 x 32 = 2 x 2 MFMA tiles), K step 16; the triangular operand limits
// the K range of each tile.
__global__ __launch_bounds__(256) void k_trinv_level(const double* __restrict__ L, double* __restrict__ Li,
                                                     double* __restrict__ T, int32_t npad, int32_t s, int32_t phase) {
  fit_prio();
  __shared__ double As[16 * 80];
  __shared__ double Bs[16 * 80];
  const int32_t z = blockIdx.z;
  const int64_t o = (int64_t)z * 2 * s;
  const int32_t s2 = (int32_t)min((int64_t)s, (int64_t)npad - o - s);  // ragged last pair (multiple of 64)
  const int32_t tr = blockIdx.y * 64, tc = blockIdx.x * 64;  // output tile inside the s2 x s block
  if (s2 <= 0 || tr >= s2) return;
  const double* A;
  const double* B;
  int64_t lda, ldb;
  int32_t k_lo, k_hi;
  double* C;
  int64_t ldc;
  double sign;
  if (phase == 0) {
    A = L + (o + s) * npad + o; lda = npad;                       // B (dense)
    B = Li + o * npad + o; ldb = npad;                            // Ai (lower): rows k >= tc contribute
    k_lo = tc; k_hi = s;
    C = T + (int64_t)z * s * s; ldc = s; sign = 1.0;
  } else {
    A = Li + (o + s) * npad + (o + s); lda = npad;                // Ci (lower): k <= tr + 63
    B = T + (int64_t)z * s * s; ldb = s;
    k_lo = 0; k_hi = min(tr + 64, s2);
    C = Li + (o + s) * npad + o; ldc = npad; sign = -1.0;
  }
  typedef double d4 __attribute__((ext_vector_type(4)));
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int wr = w >> 1, wc = w & 1;
  d4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = (d4){0.0, 0.0, 0.0, 0.0};
  for (int32_t k0 = k_lo; k0 < k_hi; k0 += 16) {
    // A tile 64 x 16 -> As[k][row]; B tile 16 x 64 -> Bs[k][col]
    for (int e = t; e < 64 * 16; e += 256) {
      const int r = e >> 4, kk = e & 15;
      As[kk * 80 + r] = A[(int64_t)(tr + r) * lda + k0 + kk];
      const int kb = e >> 6, c = e & 63;
      Bs[kb * 80 + c] = B[(int64_t)(k0 + kb) * ldb + tc + c];
    }
    __syncthreads();
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      const int kr = ks * 4 + (lane >> 4);
      double af[2], bf[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) af[i] = As[kr * 80 + wr * 32 + i * 16 + (lane & 15)];
#pragma unroll
      for (int j = 0; j < 2; ++j) bf[j] = Bs[kr * 80 + wc * 32 + j * 16 + (lane & 15)];
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(af[i], bf[j], acc[i][j], 0, 0, 0);
    }
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = tr + wr * 32 + i * 16 + (lane >> 4) + 4 * r;
        const int col = tc + wc * 32 + j * 16 + (lane & 15);
        C[(int64_t)row * ldc + col] = sign * acc[i][j][r];
      }
}

// The same two products for levels s >= TRB_MIN, where k_trinv_level's 64 x 64
// tiles and plain loads dominate the fit (at n = 4096 the top level is 75 % of
// the inverse's 23 GFLOP).  128 x 128 output tile per 256-thread workgroup
// (2 x 2 waves of 64 x 64, 4 x 4 v_mfma_f64_16x16x4 sub-tiles each), 16-k
// stages through a 2-deep global_load_lds ring (k_gp_var_pp's pipeline), two
// workgroups per CU.
//   right operand, [k][col] row-major (Ai, T): one 1-KiB wave-instruction per k row;
//   left operand, [row][k] row-major (the L block, Ci): one wave-instruction
//   moves 8 rows x 16 k; lane l fetches 16-B chunk (l & 7) ^ ((row >> 1) & 7)
//   of its row, so an MFMA fragment read (16 rows at one k) hits 16 distinct
//   bank pairs.
// k runs upward in MFMA groups of 4 from a multiple of 64, as in k_trinv_level;
// the extra products a 128-wide tile takes on are exact zeros of the
// triangular operand, so the two kernels give the same bits.
constexpr int TRB_MIN = 256, TRB_BM = 128, TRB_BK = 16, TRB_SL = TRB_BM * TRB_BK;

__global__ __launch_bounds__(256, 2) void k_trinv_big(const double* __restrict__ L, double* __restrict__ Li,
                                                      double* __restrict__ T, int32_t npad, int32_t s, int32_t phase) {
  fit_prio();
  // one __shared__ object (see k_gp_var): [stage][left | right]
  __shared__ __attribute__((aligned(16))) double lds[2 * 2 * TRB_SL];
  const int32_t z = blockIdx.z;
  const int64_t o = (int64_t)z * 2 * s;
  const int32_t s2 = (int32_t)min((int64_t)s, (int64_t)npad - o - s);  // multiple of 128 (npad % NPAD == 0)
  const int32_t tr = blockIdx.y * TRB_BM, tc = blockIdx.x * TRB_BM;
  if (s2 <= 0 || tr >= s2) return;
  const double* A;
  const double* B;
  int64_t lda, ldb, ldc;
  int32_t k_lo, k_hi;
  double* C;
  double sign;
  if (phase == 0) {
    A = L + (o + s) * npad + o; lda = npad;
    B = Li + o * npad + o; ldb = npad;
    k_lo = tc; k_hi = s;
    C = T + (int64_t)z * s * s; ldc = s; sign = 1.0;
  } else {
    A = Li + (o + s) * npad + (o + s); lda = npad;
    B = T + (int64_t)z * s * s; ldb = s;
    k_lo = 0; k_hi = min(tr + TRB_BM, s2);
    C = Li + (o + s) * npad + o; ldc = npad; sign = -1.0;
  }
  const int t = threadIdx.x, lane = t & 63;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const int wm = w >> 1, wn = w & 1;
  auto issue = [&](int32_t k0, double* st) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int q = 4 * w + u;
      const int row = 8 * q + (lane >> 3);
      const int ch = (lane & 7) ^ ((row >> 1) & 7);
      __builtin_amdgcn_global_load_lds(A + (int64_t)(tr + row) * lda + k0 + 2 * ch,
                                       (__attribute__((address_space(3))) void*)(st + q * 128), 16, 0, 0);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int q = 4 * w + u;
      __builtin_amdgcn_global_load_lds(B + (int64_t)(k0 + q) * ldb + tc + lane * 2,
                                       (__attribute__((address_space(3))) void*)(st + TRB_SL + q * 128), 16, 0, 0);
    }
  };
  typedef double d4 __attribute__((ext_vector_type(4)));
  d4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = (d4){0.0, 0.0, 0.0, 0.0};
  const int32_t nk = (k_hi - k_lo) / TRB_BK;
  issue(k_lo, lds);
  for (int32_t kt = 0; kt < nk; ++kt) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // stage kt landed everywhere; stage kt-1 fully read
    asm volatile("" ::: "memory");
    if (kt + 1 < nk) issue(k_lo + (kt + 1) * TRB_BK, lds + ((kt + 1) & 1) * 2 * TRB_SL);
    const double* as = lds + (kt & 1) * 2 * TRB_SL;
    const double* bs = as + TRB_SL;
#pragma unroll
    for (int ks = 0; ks < TRB_BK / 4; ++ks) {
      const int kr = ks * 4 + (lane >> 4);
      double af[4], bf[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) bf[j] = bs[kr * TRB_BM + wn * 64 + j * 16 + (lane & 15)];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int row = wm * 64 + i * 16 + (lane & 15);
        af[i] = as[row * TRB_BK + 2 * ((kr >> 1) ^ ((row >> 1) & 7)) + (kr & 1)];
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(af[i], bf[j], acc[i][j], 0, 0, 0);
    }
  }
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = tr + wm * 64 + i * 16 + (lane >> 4) + 4 * r;
        const int col = tc + wn * 64 + j * 16 + (lane & 15);
        C[(int64_t)row * ldc + col] = sign * acc[i][j][r];
      }
}

// out = Linv * v  (one wave per row)
__global__ __launch_bounds__(256) void k_lower_mv(const double* __restrict__ Li, int32_t npad,
                                                  const double* __restrict__ v, double* __restrict__ out) {
  fit_prio();
  const int32_t r = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (r >= npad) return;
  double s = 0.0;
  for (int32_t c = lane; c <= r; c += 64) s += Li[(int64_t)r * npad + c] * v[c];
  for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off);
  if (lane == 0) out[r] = s;
}

// out = Linv^T * v, read through LinvT (row c of LinvT = column c of L^-1,
// nonzero from c on): one wave per row, coalesced (the column-strided read of
// L^-1 ran on npad / 64 workgroups at ~250 GB/s)
__global__ __launch_bounds__(256) void k_upper_mv(const double* __restrict__ LiT, int32_t npad,
                                                  const double* __restrict__ v, double* __restrict__ out) {
  fit_prio();
  const int32_t r = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (r >= npad) return;
  double s = 0.0;
  for (int32_t c = r + lane; c < npad; c += 64) s += LiT[(int64_t)r * npad + c] * v[c];
  for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off);
  if (lane == 0) out[r] = s;
}

// ---------------------------------------------------------------------------
// incremental fit: append block row b (64 rows) to an existing factor
// ---------------------------------------------------------------------------
// With the old factor L (rows < 64 b) and its inverse L^-1, the new rows'
// kernel block [K21 K22] extends it as
//   [[L, 0], [B, D]],  B = K21 L^-T,  D = chol(K22 - B B^T)
// and the inverse as
//   [[L^-1, 0], [-D^-1 B L^-1, D^-1]].
// A few small launches per block (O(n^2) work against the O(n^3) refit); the
// scratch T holds B [64][npad] at offset 0 and E = B L^-1, transposed
// ([npad][64]), at offset 64 npad.  Padded rows (>= n) are identity rows of
// K, so they stay identity rows of L^-1.

// The three products of block b, split over K in APP_KC chunks (one
// workgroup per tile x chunk, so a few hundred workgroups instead of b long
// serial K loops) and summed in chunk order by k_app_red (deterministic):
//   MODE 0  B[j][c]     = sum_c' K21[j][c'] L^-1[c][c']   tile cb < b, c' < 64 cb + 64
//   MODE 1  (B B^T)[j][j'] = sum_c' B[j][c'] B[j'][c']     one tile,   c' < 64 b
//   MODE 2  E^T[c][j]   = sum_c' B[j][c'] L^-1[c'][c]     tile cb < b, 64 cb <= c' < 64 b
//           (L^-1 read through LinvT, whose rows are its columns)
constexpr int APP_KC = 256;

struct AppGemm {
  const double* A;
  const double* B;
  int32_t klo, khi;
};

template <int MODE>
__device__ __forceinline__ AppGemm app_gemm(const double* Li, const double* LinvT, const double* K,
                                            const double* T, int32_t npad, int32_t b, int64_t t) {
  if (MODE == 0) return {Li + t * 64 * npad, K + (int64_t)b * 64 * npad, 0, (int32_t)(t * 64 + 64)};
  if (MODE == 1) return {T, T, 0, b * 64};
  return {T, LinvT + t * 64 * npad, (int32_t)(t * 64), b * 64};
}

template <int MODE>
__global__ __launch_bounds__(256) void k_app_part(const double* __restrict__ Li, const double* __restrict__ LinvT,
                                                  const double* __restrict__ K, const double* __restrict__ T,
                                                  int32_t npad, int32_t b, int32_t maxq, double* __restrict__ W) {
  fit_prio();
  __shared__ double As[16 * 80];
  __shared__ double Bs[16 * 80];
  const int64_t q = blockIdx.x, t = blockIdx.y;
  const AppGemm g = app_gemm<MODE>(Li, LinvT, K, T, npad, b, t);
  const int32_t k0 = g.klo + (int32_t)q * APP_KC;
  if (k0 >= g.khi) return;
  fd4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = (fd4){0.0, 0.0, 0.0, 0.0};
  tile64_nt(g.A + k0, npad, g.B + k0, npad, min(APP_KC, g.khi - k0), As, Bs, acc);
  double* w = W + (t * maxq + q) * 4096;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) w[tile_row(i, r) * 64 + tile_col(j)] = acc[i][j][r];
}

// MODE 0 -> B into T [64][npad];  MODE 1 -> K22 -= B B^T (in place; k_chol_diag
// factors it next);  MODE 2 -> E^T into Et [npad][64]
template <int MODE>
__global__ __launch_bounds__(256) void k_app_red(const double* __restrict__ Li, const double* __restrict__ LinvT,
                                                 double* __restrict__ K, double* __restrict__ T, int32_t npad,
                                                 int32_t b, int32_t maxq, const double* __restrict__ W,
                                                 double* __restrict__ Et) {
  fit_prio();
  const int64_t t = blockIdx.x, base = (int64_t)b * 64;
  const AppGemm g = app_gemm<MODE>(Li, LinvT, K, T, npad, b, t);
  const int32_t nq = (g.khi - g.klo + APP_KC - 1) / APP_KC;
  const double* w = W + t * maxq * 4096;
  for (int e = threadIdx.x; e < 4096; e += 256) {
    double s = 0.0;
    for (int32_t q = 0; q < nq; ++q) s += w[(int64_t)q * 4096 + e];
    const int i = e >> 6, j = e & 63;
    if (MODE == 0) T[(int64_t)j * npad + t * 64 + i] = s;
    else if (MODE == 1) K[(base + i) * npad + base + j] -= s;
    else Et[(t * 64 + j) * 64 + i] = s;
  }
}

// new L^-1 rows: C = -D^-1 E for column blocks cb < b (written to L^-1 and
// LinvT); workgroup cb == b copies D^-1 (k_chol_diag's output) into LinvT
__global__ __launch_bounds__(256) void k_app_c(double* __restrict__ Li, double* __restrict__ LinvT,
                                               const double* __restrict__ Et, int32_t npad, int32_t b) {
  fit_prio();
  __shared__ double As[16 * 80];
  __shared__ double Bs[16 * 80];
  const int64_t cb = blockIdx.x, base = (int64_t)b * 64;
  if (cb == b) {
    for (int e = threadIdx.x; e < 64 * 64; e += 256) {
      const int j = e >> 6, cc = e & 63;
      LinvT[(base + cc) * npad + base + j] = Li[(base + j) * npad + base + cc];
    }
    return;
  }
  fd4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = (fd4){0.0, 0.0, 0.0, 0.0};
  tile64_nt(Li + base * npad + base, npad, Et + cb * 64 * 64, 64, 64, As, Bs, acc);
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t row = base + tile_row(i, r), col = cb * 64 + tile_col(j);
        const double v = -acc[i][j][r];
        Li[row * npad + col] = v;
        LinvT[col * npad + row] = v;
      }
}

// ---------------------------------------------------------------------------
// score
// ---------------------------------------------------------------------------
// scaled candidate norms |u / ell|^2
__global__ void k_gp_cnorm(const double* __restrict__ feat, int64_t ld, int64_t m, int32_t d,
                           const double* __restrict__ inv_ell, double* __restrict__ cn) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= m) return;
  double s = 0.0;
  for (int32_t k = 0; k < d; ++k) {
    const double v = feat[(int64_t)k * ld + i] * inv_ell[k];
    s += v * v;
  }
  cn[i] = s;
}

__device__ __forceinline__ double acq_score(int kind, double mu, double var, double f_best, double xi,
                                            double kappa) {
  const double sigma = sqrt(var);
  if (kind == UT_ACQ_UCB) return kappa * sigma - mu;
  const double I = f_best - mu - xi;
  if (!(sigma > 0.0)) return I > 0.0 ? I : 0.0;
  const double z = I / sigma;
  const double Phi = 0.5 * erfc(-z * 0.70710678118654752440);
  const double phi = exp(-0.5 * z * z) * 0.39894228040143267794;
  return I * Phi + sigma * phi;
}

__global__ void k_gp_finalize(int64_t m, int32_t RT1, int32_t RT2, const double* __restrict__ mu_part,
                              const double* __restrict__ var_part, int64_t ldp, double sf2,
                              const double* __restrict__ stats, const int32_t* __restrict__ fit_flag, int32_t kind,
                              double xi, double kappa, const uint8_t* __restrict__ dup, double* __restrict__ mu_out,
                              double* __restrict__ var_out, double* __restrict__ score_out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= m) return;
  double mu = 0.0, vs = 0.0;
  for (int32_t r = 0; r < RT1; ++r) mu += mu_part[(int64_t)r * ldp + i];
  for (int32_t r = 0; r < RT2; ++r) vs += var_part[(int64_t)r * ldp + i];
  double var = sf2 - vs;
  var = var > 0.0 ? var : 0.0;
  double sc = acq_score(kind, mu, var, stats[0], xi, kappa);
  if (*fit_flag != 0) {  // failed (asynchronous) fit: nothing is selectable
    mu = var = sc = __builtin_nan("");
  }
  if (dup && dup[i]) sc = -1.0 / 0.0;
  if (mu_out) mu_out[i] = mu;
  if (var_out) var_out[i] = var;
  if (score_out) score_out[i] = sc;
}

// precision 8 (gp_i8.hip): |v|^2 and the mean mu = v . beta (beta = L^-1 y)
// from the int8 contraction's partials; a candidate is finished here only if
//   | |v|^2 - s | <= E (2 sqrt(s) + E) + s (2n + 64) 2^-53     (s = the computed sum)
// is at most tol * (sf2 - s) -- its variance is then within tol relative of the
// exact one -- and the mean's bound Emu = sum_r e_r |beta_r| (+ the fp64
// rounding of the sums, (2n + 64) 2^-53 |mu| |beta|-weighted, below Emu's own
// 2^-40 slack at these sizes) is at most tol * sigma: the mean within tol of
// the posterior's own scale.  Every other candidate (near a training point sf2 - |v|^2 cancels;
// or a failed fit) is appended to idx_out for the fp64 recompute (k_gp_fix_i8),
// one atomic per wave; its outputs are written anyway and overwritten there.
// Duplicates (dup[i], score -inf) are never flagged.
__global__ void k_gp_finalize_i8(int64_t m, int32_t RT1, int32_t RT2, const double* __restrict__ mu_part,
                                 const double* __restrict__ var_part, int64_t ldp, double sf2,
                                 const double* __restrict__ stats, const int32_t* __restrict__ fit_flag, int32_t kind,
                                 double xi, double kappa, const uint8_t* __restrict__ dup, double* __restrict__ mu_out,
                                 double* __restrict__ var_out, double* __restrict__ score_out,
                                 const double* __restrict__ Ebound, double tol, int32_t n, int64_t* __restrict__ idx_out,
                                 unsigned long long* __restrict__ count) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int lane = threadIdx.x & 63;
  bool flag = false;
  if (i < m) {
    double mu = 0.0, vs = 0.0;
    for (int32_t r = 0; r < RT1; ++r) mu += mu_part[(int64_t)r * ldp + i];
    for (int32_t r = 0; r < RT2; ++r) vs += var_part[(int64_t)r * ldp + i];
    double var = sf2 - vs;
    var = var > 0.0 ? var : 0.0;
    const double E = Ebound[0], Emu = Ebound[1];
    const double bound = E * (2.0 * sqrt(vs) + E) + vs * (double)(2 * n + 64) * 0x1p-53;
    flag = !(bound <= tol * var) || !(Emu <= tol * sqrt(var));   // (NaN: flagged)
    double sc = acq_score(kind, mu, var, stats[0], xi, kappa);
    if (*fit_flag != 0) {
      mu = var = sc = __builtin_nan("");
      flag = false;   // nothing to recompute: the fit failed
    }
    if (dup && dup[i]) {
      // a duplicate of the history is a training point, where sf2 - |v|^2
      // cancels and the bound always fails: its score is -inf whatever the
      // variance, so it is not recomputed (its var output stays this tier's)
      sc = -1.0 / 0.0;
      flag = false;
    }
    if (mu_out) mu_out[i] = mu;
    if (var_out) var_out[i] = var;
    if (score_out) score_out[i] = sc;
  }
  const unsigned long long ball = __ballot(flag);
  const uint32_t nf = __builtin_popcountll(ball);
  unsigned long long base = 0;
  if (lane == 0 && nf) base = atomicAdd(count, (unsigned long long)nf);
  base = __shfl(base, 0, 64);
  if (flag) idx_out[base + __builtin_popcountll(ball & ((1ull << lane) - 1ull))] = i;
}

// the flagged candidates' fp64 mean and variance (recomputed K* columns through
// the fp64 contraction, RT partials each of v^2 and of v . beta) -> mu, var, score
__global__ void k_gp_fix_i8(int64_t nf, const int64_t* __restrict__ idx, int32_t RT, const double* __restrict__ mpart,
                            const double* __restrict__ vpart, int64_t ldv, double sf2,
                            const double* __restrict__ stats, int32_t kind, double xi, double kappa,
                            const uint8_t* __restrict__ dup, double* __restrict__ mu_out, double* __restrict__ var_out,
                            double* __restrict__ score_out) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= nf) return;
  const int64_t i = idx[j];
  double mu = 0.0, vs = 0.0;
  for (int32_t r = 0; r < RT; ++r) mu += mpart[(int64_t)r * ldv + j];
  for (int32_t r = 0; r < RT; ++r) vs += vpart[(int64_t)r * ldv + j];
  double var = sf2 - vs;
  var = var > 0.0 ? var : 0.0;
  double sc = acq_score(kind, mu, var, stats[0], xi, kappa);
  if (dup && dup[i]) sc = -1.0 / 0.0;
  if (mu_out) mu_out[i] = mu;
  if (var_out) var_out[i] = var;
  if (score_out) score_out[i] = sc;
}

// ---------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------
static void launch_chol_diag(ut_ctx* c, int32_t npad, int32_t kb) {
  hipLaunchKernelGGL(c->chol_merged ? k_chol_diag<true> : k_chol_diag<false>, dim3(1), dim3(256), 0, c->stream,
                     c->gp_K, c->gp_Linv, npad, kb, c->gp_flag);
}

static int gp_alloc(ut_ctx* c, int32_t npad_need, int32_t d) {
  if (c->gp_cap_n >= npad_need && c->gp_d == d && c->gp_Xs) return 0;
  // room for a growing training set (the tuning loop adds a few rows per fit):
  // a new padded size then reuses the buffers instead of freeing and
  // allocating ~5 n^2 doubles behind a device-wide sync (2.5-10 ms per 128
  // rows in the C5 loop).  Every kernel indexes with the fit's own npad.
  const int64_t npad = ((npad_need + npad_need / 4 + NPAD - 1) / NPAD) * NPAD;
  if (c->gp_Xs_f) {
    UT_HIP(c, ut::sync_all(c));
    ut::dfree(c->gp_Xs_f); ut::dfree(c->gp_LinvT); ut::dfree(c->gp_LinvT_f); ut::dfree(c->gp_T); ut::dfree(c->gp_ctr);
    ut::dfree(c->gp_XsT);
    c->gp_Xs_f = nullptr; c->gp_LinvT = nullptr; c->gp_LinvT_f = nullptr; c->gp_T = nullptr; c->gp_ctr = nullptr;
    c->gp_XsT = nullptr;
  }
  if (c->gp_Xs) {
    UT_HIP(c, ut::sync_all(c));
    ut::dfree(c->gp_Xs); ut::dfree(c->gp_xnorm); ut::dfree(c->gp_K); ut::dfree(c->gp_Linv);
    ut::dfree(c->gp_y); ut::dfree(c->gp_tmp); ut::dfree(c->gp_alpha); ut::dfree(c->gp_beta); ut::dfree(c->gp_inv_ell);
    ut::dfree(c->gp_stats); ut::dfree(c->gp_flag);
  }
  UT_HIP(c, ut::dmalloc((void**)&c->gp_Xs, sizeof(double) * npad * d));
  UT_HIP(c, ut::dmalloc((void**)&c->gp_xnorm, sizeof(double) * npad));
  UT_HIP(c, ut::dmalloc((void**)&c->gp_K, sizeof(double) * npad * npad));
  UT_HIP(c, ut::dmalloc((void**)&c->gp_Linv, sizeof(double) * npad * npad));
  UT_HIP(c, ut::dmalloc((void**)&c->gp_y, sizeof(double) * npad));
  UT_HIP(c, ut::dmalloc((void**)&c->gp_tmp, sizeof(double) * npad * (d + 1)));
  UT_HIP(c, ut::dmalloc((void**)&c->gp_alpha, sizeof(double) * npad));
  UT_HIP(c, ut::dmalloc((void**)&c->gp_beta, sizeof(double) * npad));
  UT_HIP(c, ut::dmalloc((void**)&c->gp_inv_ell, sizeof(double) * d));
  UT_HIP(c, ut::dmalloc((void**)&c->gp_stats, sizeof(double) * 4));
  UT_HIP(c, ut::dmalloc((void**)&c->gp_flag, sizeof(int32_t)));
  UT_HIP(c, ut::dmalloc((void**)&c->gp_T, sizeof(double) * npad * npad));
  UT_HIP(c, ut::dmalloc((void**)&c->gp_Xs_f, sizeof(float) * npad * d));
  UT_HIP(c, ut::dmalloc((void**)&c->gp_LinvT, sizeof(double) * npad * npad));
  // fp32: (L^-1)^T; h3: the blocked fp16 hi / lo planes, rows padded to 256
  UT_HIP(c, ut::dmalloc((void**)&c->gp_LinvT_f, sizeof(float) * (((npad + 255) / 256) * 256) * npad));
  UT_HIP(c, ut::dmalloc((void**)&c->gp_ctr, sizeof(int32_t) * 32));
  UT_HIP(c, ut::dmalloc((void**)&c->gp_XsT, sizeof(double) * npad * kstar_dpad(d)));
  c->gp_cap_n = npad;
  c->gp_d = d;
  return 0;
}

// rows [r0, r1) of X [n][d] have exact one-hot ENUM blocks and 0 / 1 BOOL
// features: the categorical K* reads the training rows as option codes
static bool cat_rows_ok(const Space& s, const double* X, int32_t d, int32_t r0, int32_t r1) {
  for (int32_t r = r0; r < r1; ++r) {
    const double* row = X + (size_t)r * d;
    for (int32_t p : s.host_cat) {
      const DevParam& q = s.host_params[p];
      const double* x = row + q.feat_col;
      if (q.kind == UT_BOOL) {
        if (!(x[0] == 0.0 || x[0] == 1.0)) return false;
        continue;
      }
      int32_t ones = 0;
      for (int32_t k = 0; k < (int32_t)q.n_opt; ++k) {
        if (x[k] == 1.0) ++ones;
        else if (x[k] != 0.0) return false;
      }
      if (ones != 1) return false;
    }
  }
  return true;
}

// The fit's device work on c->stream (the fit stream), in two parts split at
// ev_fit_x: part 0 the staging copies from the pinned host buffer and the
// scaled inputs; part 1 the factor and L^-1 (a refit, or block rows appended
// to the previous factor), beta / alpha, and the scoring precision's
// operands.  Enqueues only: every buffer is allocated by the caller.
static int fit_device(ut_ctx* c, int part, int32_t n, int32_t n0, int32_t d, int32_t npad, int32_t dpn, bool app,
                      int32_t xr0, double diag, double sf2) {
  int rc;
  const Space& sp = c->space;
  double* hX = c->fit_host;
  double* hy = hX + (size_t)n * d;
  double* hinv = hy + n;
  double* dX = c->gp_tmp;           // [n][d] staging (gp_tmp holds npad*(d+1))
  double* dy = c->gp_tmp + (int64_t)npad * d;
  if (part == 0) {
    UT_HIP(c, hipMemcpyAsync(c->gp_inv_ell, hinv, sizeof(double) * d, hipMemcpyHostToDevice, c->stream));
    UT_HIP(c, hipMemcpyAsync(dX + (size_t)xr0 * d, hX + (size_t)xr0 * d, sizeof(double) * (size_t)(n - xr0) * d,
                             hipMemcpyHostToDevice, c->stream));
    UT_HIP(c, hipMemcpyAsync(dy, hy, sizeof(double) * n, hipMemcpyHostToDevice, c->stream));
    if (!app) UT_HIP(c, hipMemsetAsync(c->gp_flag, 0, sizeof(int32_t), c->stream));
    hipLaunchKernelGGL(k_gp_prep_train, dim3(grid1(npad, 256)), dim3(256), 0, c->stream, dX, n, npad, d,
                       c->gp_inv_ell, c->gp_Xs, c->gp_xnorm);
    // the candidate side of K* needs only the scaled inputs: fp64 scoring starts
    // its K* here while the factorisation below is still running
    if ((rc = launch_xs_t(c, c->gp_Xs, npad, d, kstar_dpad(d), c->gp_XsT))) return rc;
    if (c->cat_on) {
      hipLaunchKernelGGL(k_gp_num_train, dim3(grid1(npad, 256)), dim3(256), 0, c->stream, c->gp_Xs, npad, d,
                         sp.d_num_feat, sp.n_num, dpn, c->gp_XsT_num.p, c->gp_xnorm_num.p);
      UT_HIP(c, hipMemsetAsync(c->gp_acat.p, 0, (size_t)sp.cat_k * npad, c->stream));
      hipLaunchKernelGGL(k_gp_cat_train, dim3(grid1(n, 256)), dim3(256), 0, c->stream, sp.d_params, sp.P, sp.d_cat_ccol,
                         dX, n, d, npad, c->gp_acat.p);
      UT_LAUNCH_CHECK(c);
    }
    // precision 8: K*'s training operand as int8 digit planes (gp_kq.hip;
    // numeric fits only, gp_score_impl)
    if (c->gp_prec == 8 && c->kstar_q && !c->cat_on &&
        (rc = launch_split_x8(c, c->gp_XsT, kstar_dpad(d), npad)))
      return rc;
    return 0;
  }
  if (app) {
    // (the previous precision-8 refit left (L^-1)^T to its readers)
    if ((rc = gp_ensure_linvt(c))) return rc;
    // block rows b0 .. b1 hold the new rows (b0 may also hold old ones: it is
    // recomputed whole)
    const int32_t b0 = n0 / NB, b1 = (n - 1) / NB;
    hipLaunchKernelGGL(k_gp_kmat, dim3(b1 + 1, b1 - b0 + 1), dim3(256), 0, c->stream, c->gp_Xs, c->gp_xnorm, n,
                       npad, d, sf2, diag, c->gp_K, b0);
    hipLaunchKernelGGL(k_gp_ystats, dim3(1), dim3(256), 0, c->stream, dy, n, npad, c->gp_y, c->gp_stats);
    double* Et = c->gp_T + (int64_t)NB * npad;
    for (int32_t b = b0; b <= b1; ++b) {
      const int32_t maxq = (b * NB + APP_KC - 1) / APP_KC;
      if (b > 0) {
        double* W = c->app_ws.p;
        hipLaunchKernelGGL(k_app_part<0>, dim3(maxq, b), dim3(256), 0, c->stream, c->gp_Linv, c->gp_LinvT,
                           c->gp_K, c->gp_T, npad, b, maxq, W);
        hipLaunchKernelGGL(k_app_red<0>, dim3(b), dim3(256), 0, c->stream, c->gp_Linv, c->gp_LinvT, c->gp_K,
                           c->gp_T, npad, b, maxq, W, Et);
        hipLaunchKernelGGL(k_app_part<1>, dim3(maxq, 1), dim3(256), 0, c->stream, c->gp_Linv, c->gp_LinvT,
                           c->gp_K, c->gp_T, npad, b, maxq, W);
        hipLaunchKernelGGL(k_app_red<1>, dim3(1), dim3(256), 0, c->stream, c->gp_Linv, c->gp_LinvT, c->gp_K,
                           c->gp_T, npad, b, maxq, W, Et);
      }
      launch_chol_diag(c, npad, b);
      if (b > 0) {
        double* W = c->app_ws.p;
        hipLaunchKernelGGL(k_app_part<2>, dim3(maxq, b), dim3(256), 0, c->stream, c->gp_Linv, c->gp_LinvT,
                           c->gp_K, c->gp_T, npad, b, maxq, W);
        hipLaunchKernelGGL(k_app_red<2>, dim3(b), dim3(256), 0, c->stream, c->gp_Linv, c->gp_LinvT, c->gp_K,
                           c->gp_T, npad, b, maxq, W, Et);
      }
      hipLaunchKernelGGL(k_app_c, dim3(b + 1), dim3(256), 0, c->stream, c->gp_Linv, c->gp_LinvT, Et, npad, b);
    }
    UT_LAUNCH_CHECK(c);
  } else {
    hipLaunchKernelGGL(k_gp_kmat, dim3(npad / 64, npad / 64), dim3(256), 0, c->stream, c->gp_Xs,
                       c->gp_xnorm, n, npad, d, sf2, diag, c->gp_K, 0);
    hipLaunchKernelGGL(k_gp_ystats, dim3(1), dim3(256), 0, c->stream, dy, n, npad, c->gp_y, c->gp_stats);
    UT_LAUNCH_CHECK(c);
    const int32_t nb = npad / NB;
    UT_HIP(c, hipMemsetAsync(c->gp_Linv, 0, sizeof(double) * npad * npad, c->stream));
    const bool fuse = c->chol_fuse > 0 || (c->chol_fuse < 0 && npad >= 2048);
    for (int32_t kb = 0; kb < nb; ++kb) {
      // (fused: diagonal blocks after the first come from the previous update)
      if (!fuse || kb == 0)
        launch_chol_diag(c, npad, kb);
      const int32_t T = nb - kb - 1;
      if (T > 0) {
        hipLaunchKernelGGL(k_chol_rows, dim3(T), dim3(256), 0, c->stream, c->gp_K, c->gp_Linv, npad, kb);
        if (fuse)
          hipLaunchKernelGGL(c->chol_merged ? k_chol_update_diag<true> : k_chol_update_diag<false>,
                             dim3(T * (T + 1) / 2), dim3(256), 0, c->stream, c->gp_K, c->gp_Linv, npad, kb, c->gp_flag);
        else
          hipLaunchKernelGGL(k_chol_update, dim3(T * (T + 1) / 2), dim3(256), 0, c->stream, c->gp_K, npad, kb);
      }
    }
    UT_LAUNCH_CHECK(c);
    // off-diagonal blocks of L^-1 by recursive doubling (diagonal blocks came from k_chol_diag)
    for (int32_t lv = NB; lv < npad; lv *= 2) {
      const int32_t pairs = (int32_t)((npad - lv + 2 * lv - 1) / (2 * lv));
      if (c->trinv_big && lv >= TRB_MIN) {
        // k_trinv_big's tiles: every pair's sizes are multiples of 128
        UT_CHECK(c, npad % TRB_BM == 0 && lv % TRB_BM == 0, UT_EINVAL, "gp_fit: npad not a multiple of 128");
        const dim3 gb(lv / TRB_BM, lv / TRB_BM, pairs);
        hipLaunchKernelGGL(k_trinv_big, gb, dim3(256), 0, c->stream, c->gp_K, c->gp_Linv, c->gp_T, npad, lv, 0);
        hipLaunchKernelGGL(k_trinv_big, gb, dim3(256), 0, c->stream, c->gp_K, c->gp_Linv, c->gp_T, npad, lv, 1);
        continue;
      }
      const dim3 grid(lv / 64, lv / 64, pairs);
      hipLaunchKernelGGL(k_trinv_level, grid, dim3(256), 0, c->stream, c->gp_K, c->gp_Linv, c->gp_T, npad, lv, 0);
      hipLaunchKernelGGL(k_trinv_level, grid, dim3(256), 0, c->stream, c->gp_K, c->gp_Linv, c->gp_T, npad, lv, 1);
    }
    UT_LAUNCH_CHECK(c);
  }
  hipLaunchKernelGGL(k_lower_mv, dim3(grid1(npad, 4)), dim3(256), 0, c->stream, c->gp_Linv, npad, c->gp_y,
                     c->gp_beta);
  UT_LAUNCH_CHECK(c);
  if (c->gp_prec == 32 && (rc = launch_to_f32(c, c->gp_Xs, c->gp_Xs_f, (int64_t)npad * d))) return rc;
  // precision 8 scores from the digit planes of L^-1 and beta alone: a refit
  // leaves (L^-1)^T and alpha = L^-T beta to the paths that read them (the fp64
  // recompute, the next append: gp_ensure_linvt), off the chain the variance
  // GEMM waits for
  if (c->gp_prec == 8 && !app) {
    if ((rc = launch_split_i8(c, n, npad))) return rc;
    c->gp_linvt_stale = true;
    return 0;
  }
  // (an append wrote its rows of LinvT itself)
  if ((!app || c->gp_prec == 32) &&
      (rc = launch_transpose(c, c->gp_Linv, npad, c->gp_LinvT, c->gp_prec == 32 ? c->gp_LinvT_f : nullptr)))
    return rc;
  hipLaunchKernelGGL(k_upper_mv, dim3(grid1(npad, 4)), dim3(256), 0, c->stream, c->gp_LinvT, npad, c->gp_beta,
                     c->gp_alpha);
  UT_LAUNCH_CHECK(c);
  c->gp_linvt_stale = false;
  if (c->gp_prec == 16 && (rc = launch_split_h3(c, c->gp_Linv, npad, reinterpret_cast<_Float16*>(c->gp_LinvT_f))))
    return rc;
  if (c->gp_prec == 8 && (rc = launch_split_i8(c, n, npad))) return rc;
  return 0;
}

// (L^-1)^T and alpha of a precision-8 refit, on c->stream, once (fit_device)
int gp_ensure_linvt(ut_ctx* c) {
  if (!c->gp_linvt_stale) return 0;
  const int32_t npad = c->gp_npad_fit;
  int rc;
  if ((rc = launch_transpose(c, c->gp_Linv, npad, c->gp_LinvT, nullptr))) return rc;
  hipLaunchKernelGGL(k_upper_mv, dim3(grid1(npad, 4)), dim3(256), 0, c->stream, c->gp_LinvT, npad, c->gp_beta,
                     c->gp_alpha);
  UT_LAUNCH_CHECK(c);
  c->gp_linvt_stale = false;
  return 0;
}

// Host work over the training rows in 8 threads when it is large (C4: 3,680
// rows x 707 features, 20.8 MB to stage and every one-hot block to check:
// ~2-3 ms on one thread, most of it with the device idle between rounds)
template <class F>
static bool par_rows(int32_t r0, int32_t r1, int32_t d, F&& f) {
  const size_t work = (size_t)(r1 > r0 ? r1 - r0 : 0) * (size_t)d;
  const unsigned hw = std::thread::hardware_concurrency();
  const int32_t nt = work < ((size_t)1 << 19) ? 1 : (int32_t)std::min<unsigned>(8, hw > 1 ? hw : 1);
  if (nt <= 1) return f(r0, r1);
  const int32_t step = (r1 - r0 + nt - 1) / nt;
  std::vector<std::thread> th;
  std::vector<char> ok(nt, 1);
  for (int32_t t = 0; t < nt; ++t) {
    const int32_t a = r0 + t * step, b = std::min(r1, a + step);
    if (a >= b) break;
    th.emplace_back([&, t, a, b] { ok[t] = f(a, b) ? 1 : 0; });
  }
  for (auto& x : th) x.join();
  for (char v : ok)
    if (!v) return false;
  return true;
}

// Stage a fit (X, y, 1/ell in pinned memory, every buffer allocated, the
// append / categorical decisions taken) whose device work gp_fit_flush
// enqueues on the fit stream, ordered after everything already enqueued on the
// caller's stream (earlier rounds read the GP state being replaced).  Scoring
// waits on ev_fit; failure (not positive definite) is reported by gp_wait_fit
// and, on the device, by NaN scores from k_gp_finalize.
int gp_fit_enqueue(ut_ctx* c, const double* X, const double* y, int32_t n, int32_t d, const ut_gp_hyper* h) {
  UT_CHECK(c, n >= 1 && d >= 1 && X && y && h && h->lengthscale_host, UT_EINVAL, "gp_fit: bad arguments");
  const int32_t npad = ((n + NPAD - 1) / NPAD) * NPAD;
  UT_CHECK(c, c->gp_prec != 8 || npad <= I8_MAX_K, UT_EINVAL,
           "gp_fit: precision 8 takes at most 16384 training points (exact int32 digit sums)");
  // a fit staged and never used is enqueued first (its staging is about to be
  // reused; an append compares against it), then the previous fit's copies out
  // of the pinned staging (and its factor) are complete once ev_fit is
  int rc = gp_fit_flush(c);
  if (rc) return rc;
  if (c->fit_pending) UT_HIP(c, hipEventSynchronize(c->ev_fit));
  // Incremental fit: new rows appended to the previous fit's training set
  // (its rows a bitwise prefix of X, same hyperparameters, same padded size,
  // a positive-definite previous factor) extend L^-1 by block rows instead of
  // refactoring (k_app_*).  y is restandardised in full either way.
  const int32_t n0 = c->gp_n;
  bool app = false;
  if (c->fit_append && c->gp_ready && c->gp_Xs && n > n0 && npad == c->gp_npad_fit && d == c->gp_d &&
      c->gp_prec == c->gp_fit_prec && c->gp_sf2 == h->sigma_f2 && c->gp_diag_fit == h->sigma_n2 + h->jitter) {
    const double* oinv = c->fit_host + (size_t)n0 * d + n0;
    app = std::memcmp(c->fit_host, X, sizeof(double) * n0 * d) == 0;
    for (int32_t k = 0; app && k < d; ++k) {
      const double v = 1.0 / h->lengthscale_host[k];
      app = std::memcmp(&v, oinv + k, sizeof(double)) == 0;
    }
    if (app) {
      if (!c->flag_host) UT_HIP(c, hipHostMalloc((void**)&c->flag_host, sizeof(int32_t), hipHostMallocDefault));
      UT_HIP(c, hipMemcpyAsync(c->flag_host, c->gp_flag, sizeof(int32_t), hipMemcpyDeviceToHost, c->fit_stream));
      UT_HIP(c, hipStreamSynchronize(c->fit_stream));
      app = *c->flag_host == 0;
    }
  }
  if ((rc = gp_alloc(c, npad, d))) return rc;
  c->pr_f2_valid = false;   // |L^-1|_F^2 (pruned scoring) belongs to the previous factor
  c->pr_ab_valid = false;
  c->pr_xf_valid = false;
  const size_t need = (size_t)n * d + n + d;
  bool fresh = false;   // a new staging buffer holds no previous rows
  if (c->fit_host_n < need) {
    if (c->fit_host) hipHostFree(c->fit_host);
    c->fit_host = nullptr;
    c->fit_host_n = 0;
    // room for growth: the tuning loop appends a few rows per fit
    const size_t cap = need + need / 4 + 4096;
    UT_HIP(c, hipHostMalloc((void**)&c->fit_host, sizeof(double) * cap, hipHostMallocDefault));
    c->fit_host_n = cap;
    fresh = true;
  }
  double* hX = c->fit_host;
  double* hy = hX + (size_t)n * d;
  double* hinv = hy + n;
  // an append stages and copies only the new rows: the staging prefix was just
  // compared equal to X's (unless the staging buffer was just reallocated), and
  // the device staging (gp_tmp, same npad) still holds the previous fit's rows
  const int32_t xr0 = app && !fresh ? n0 : 0;
  par_rows(xr0, n, d, [&](int32_t a, int32_t b) {
    std::memcpy(hX + (size_t)a * d, X + (size_t)a * d, sizeof(double) * (size_t)(b - a) * d);
    return true;
  });
  std::memcpy(hy, y, sizeof(double) * n);
  for (int32_t k = 0; k < d; ++k) hinv[k] = 1.0 / h->lengthscale_host[k];
  // categorical K*: every ENUM / BOOL feature under one lengthscale and every
  // training row one-hot there (an append checks only its new rows)
  const Space& sp = c->space;
  // (and the candidates' code rows fit one workgroup's LDS: a space with
  // thousands of ENUM options scores with the dense contraction)
  bool cat = c->cat_enable && c->has_space && sp.n_cat > 0 && d == sp.n_feat && code_rows_lds(sp.cat_k) <= c->max_lds;
  double cinv = 0.0;
  if (cat) {
    cinv = hinv[sp.host_params[sp.host_cat[0]].feat_col];
    for (int32_t p : sp.host_cat) {
      const DevParam& q = sp.host_params[p];
      for (int32_t f = 0; f < q.n_feat && cat; ++f) cat = std::memcmp(&hinv[q.feat_col + f], &cinv, sizeof(double)) == 0;
      if (!cat) break;
    }
  }
  if (cat) {
    const bool prefix_ok = app && c->cat_x_ok;
    cat = par_rows(prefix_ok ? n0 : 0, n, d, [&](int32_t a, int32_t b) { return cat_rows_ok(sp, X, d, a, b); });
  }
  c->cat_x_ok = cat;
  c->cat_on = cat;
  if (cat) {
    int32_t pw = 0;
    for (int32_t p : sp.host_cat) pw += sp.host_params[p].kind == UT_BOOL ? 1 : 2;
    const double base = cinv * cinv;
    c->cat_c1 = 0.5 * base;
    c->cat_c0 = -0.5 * base * (double)pw;
  }
  const double diag = h->sigma_n2 + h->jitter;
  // every buffer the device work touches exists before it is enqueued
  const int32_t dpn = cat_dpad(c);
  if (c->cat_on) {
    if ((rc = ensure(c, c->gp_XsT_num, (size_t)(dpn > 0 ? dpn : 1) * npad))) return rc;
    if ((rc = ensure(c, c->gp_xnorm_num, (size_t)npad))) return rc;
    if ((rc = ensure(c, c->gp_acat, (size_t)sp.cat_k * npad))) return rc;
  }
  if (app) {
    size_t ws = 0;
    for (int32_t b = std::max(n0 / NB, 1); b <= (n - 1) / NB; ++b)
      ws = std::max(ws, (size_t)b * ((b * NB + APP_KC - 1) / APP_KC) * 4096);
    if (ws && (rc = ensure(c, c->app_ws, ws))) return rc;
  }
  if (c->gp_prec == 8) {
    if ((rc = alloc_split_i8(c, npad))) return rc;
    c->gp_i8_eb = i8_kstar_exp(h->sigma_f2);
    if (c->kstar_q && !c->cat_on && (rc = alloc_split_x8(c, npad, kstar_dpad(d)))) return rc;
  }
  c->gp_n = n;
  c->gp_sf2 = h->sigma_f2;
  c->gp_fit_prec = c->gp_prec;
  c->gp_npad_fit = npad;
  c->gp_diag_fit = diag;
  c->gp_fit_kind = app ? 1 : 0;
  c->gp_ready = true;
  ut_ctx::FitJob& j = c->fit_job;
  j.n = n, j.n0 = n0, j.d = d, j.npad = npad, j.dpn = dpn, j.xr0 = xr0;
  j.app = app, j.diag = diag, j.sf2 = h->sigma_f2;
  j.on = true;
  c->fit_prefit_set = false;
  return c->fit_defer ? 0 : gp_fit_flush(c);
}

// The staged fit's place on the caller's stream: recorded before a proposal
// is enqueued, so the fit flushed after it still runs beside it.
int gp_fit_prefit(ut_ctx* c) {
  if (!c->fit_job.on || c->fit_prefit_set) return 0;
  UT_HIP(c, hipEventRecord(c->ev_prefit, c->stream));
  c->fit_prefit_set = true;
  return 0;
}

// Enqueue the staged fit's device work on the fit stream, ordered after what
// the caller's stream held at gp_fit_prefit (or now).  Scoring waits on
// ev_fit_x (scaled inputs) / ev_fit (the factor).
int gp_fit_flush(ut_ctx* c) {
  if (!c->fit_job.on) return 0;
  const ut_ctx::FitJob j = c->fit_job;
  c->fit_job.on = false;
  // (a launch that fails below leaves no usable factor)
  c->gp_ready = false;
  if (!c->fit_prefit_set) UT_HIP(c, hipEventRecord(c->ev_prefit, c->stream));
  c->fit_prefit_set = false;
  UT_HIP(c, hipStreamWaitEvent(c->fit_stream, c->ev_prefit, 0));
  int rc;
  {
    StreamScope on_fit(c, c->fit_stream);
    if ((rc = fit_device(c, 0, j.n, j.n0, j.d, j.npad, j.dpn, j.app, j.xr0, j.diag, j.sf2))) return rc;
    UT_HIP(c, hipEventRecord(c->ev_fit_x, c->stream));   // the scaled inputs: fp64 K* may start
    if ((rc = fit_device(c, 1, j.n, j.n0, j.d, j.npad, j.dpn, j.app, j.xr0, j.diag, j.sf2))) return rc;
    UT_HIP(c, hipEventRecord(c->ev_fit, c->stream));
  }
  c->fit_pending = true;
  c->gp_ready = true;
  return 0;
}

// Wait for the enqueued fit and check it (positive definite).
int gp_wait_fit(ut_ctx* c) {
  int rc;
  if ((rc = gp_fit_flush(c))) return rc;
  if (!c->fit_pending) return 0;
  // the flag is read on the fit stream itself, after the fit (a pinned
  // asynchronous copy and that stream's sync: ~10 us once the fit is done,
  // where a blocking hipMemcpy took ~1 ms per call in the C5 loop)
  if (!c->flag_host) UT_HIP(c, hipHostMalloc((void**)&c->flag_host, sizeof(int32_t), hipHostMallocDefault));
  UT_HIP(c, hipMemcpyAsync(c->flag_host, c->gp_flag, sizeof(int32_t), hipMemcpyDeviceToHost, c->fit_stream));
  UT_HIP(c, hipStreamSynchronize(c->fit_stream));
  const int32_t flag = *c->flag_host;
  if (flag != 0) {
    c->gp_ready = false;
    return set_err(c, UT_ENOTPD, "gp_fit: kernel matrix is not positive definite (raise jitter)");
  }
  return 0;
}

int gp_encode_scaled(ut_ctx* c, const double* values, int64_t ld, int64_t m) {
  UT_CHECK(c, c->gp_ready, UT_EINVAL, "gp_score: call ut_gp_fit first");
  if (m <= 0) return 0;
  int rc;
  if ((rc = gp_fit_flush(c))) return rc;
  // 1/ell comes with the fit's scaled training inputs
  if (c->fit_pending) UT_HIP(c, hipStreamWaitEvent(c->stream, c->ev_fit_x, 0));
  const int64_t ldk = ((m + VAR_BN - 1) / VAR_BN) * VAR_BN;   // as gp_score_impl
  if ((rc = ensure(c, c->cnorm, (size_t)ldk))) return rc;
  if (c->cat_on) {   // numeric U', norms and the one-hot codes (categorical K*)
    const int32_t dpn = cat_dpad(c);
    if ((rc = ensure(c, c->ucand, (size_t)(dpn > 0 ? dpn : 1) * ldk))) return rc;
    if ((rc = ensure(c, c->bcat, (size_t)c->space.cat_k * ldk))) return rc;
    c->ucand_cat = true;
    return launch_encode_scaled_cat(c, values, ld, m, c->ucand.p, dpn, ldk, c->cnorm.p, c->bcat.p);
  }
  const int32_t dpad = kstar_dpad(c->gp_d);
  if ((rc = ensure(c, c->ucand, (size_t)dpad * ldk))) return rc;
  c->ucand_cat = false;
  return launch_encode_scaled(c, values, ld, m, c->ucand.p, dpad, ldk, c->cnorm.p);
}

// the categorical operands of the current fit for launch_gemm_kstar
static KstarCat kstar_cat(ut_ctx* c, const int8_t* bcat) {
  KstarCat k;
  k.acat = c->gp_acat.p;
  k.bcat = bcat;
  k.nkc = c->space.cat_k / 128;
  k.c0 = c->cat_c0;
  k.c1 = c->cat_c1;
  return k;
}

static int gather_kstar_cols(ut_ctx* c, bool cat, int32_t dpad, int64_t ldk, const int64_t* idx, int64_t base,
                             int64_t nc, int64_t ldc, double* mu_part = nullptr);

int gp_score_impl(ut_ctx* c, const double* feat, int64_t ld, int64_t m, const ut_acq* acq, const uint8_t* dup,
                  double* mu, double* var, double* score, hipEvent_t dup_ready) {
  UT_CHECK(c, c->gp_ready, UT_EINVAL, "gp_score: call ut_gp_fit first");
  UT_CHECK(c, acq != nullptr, UT_EINVAL, "gp_score: acq is NULL");
  if (m <= 0) return 0;
  if (int rc0 = gp_fit_flush(c)) return rc0;
  const int prec = c->gp_fit_prec;
  const bool fp32 = prec != 64;  // fp32, h3 (f16x3) and i8: K* stores a reduced-precision K*
  const bool i8 = prec == 8;
  // the mean in K*'s fp64 epilogue (k* . alpha, before k* is rounded): fp32 and h3
  const bool kmu = fp32 && !i8;
  // fp64 and i8: K* needs only the scaled training inputs (ev_fit_x) and the
  // mean comes from the variance epilogue, mu = (L^-1 k*) . (L^-1 y), so K*
  // overlaps the rest of an asynchronous fit and only the variance GEMM waits
  // for L^-1 (i8: |mu - mu^| <= Emu, gp_i8.hip).  fp32 / h3 keep the mean in
  // K*'s fp64 epilogue and wait for the whole fit.
  if (c->fit_pending) UT_HIP(c, hipStreamWaitEvent(c->stream, kmu ? c->ev_fit : c->ev_fit_x, 0));
  mark(c, "fit_wait");   // (the wait is not K* time)
  const int32_t n = c->gp_n, d = c->gp_d;
  const int32_t npad = ((n + NPAD - 1) / NPAD) * NPAD;
  // the categorical K* when the candidates came through ut's encoder
  // (gp_encode_scaled in categorical mode); a caller's feature matrix takes the
  // dense contraction over every feature
  const bool cat = !feat && c->cat_on && c->ucand_cat;
  const int32_t dpad = cat ? cat_dpad(c) : kstar_dpad(d);
  // K* rows padded to whole variance column tiles: the variance kernel reads
  // full 256-candidate strips (the K* kernel writes zeros past m)
  const int64_t ldk = ((m + VAR_BN - 1) / VAR_BN) * VAR_BN;
  const int32_t RT = npad / NPAD;
  int rc;
  if ((rc = ensure(c, c->kst, (size_t)npad * ldk))) return rc;
  // (i8: the variance and mean partials come per 64-row tile)
  if ((rc = ensure(c, c->mu_part, (size_t)(i8 ? 2 * RT : RT) * ldk))) return rc;
  if ((rc = ensure(c, c->var_part, (size_t)(i8 ? 2 * RT : RT) * ldk))) return rc;
  if ((rc = ensure(c, c->cnorm, (size_t)ldk))) return rc;
  if ((rc = ensure(c, c->ucand, (size_t)(dpad > 0 ? dpad : 1) * ldk))) return rc;
  if (i8) {
    UT_CHECK(c, npad <= I8_MAX_K, UT_EINVAL, "gp_score: precision 8 takes at most 16384 training points");
    if ((rc = ensure(c, c->pr_idx, (size_t)ldk))) return rc;
    if ((rc = ensure(c, c->pr_count, 1))) return rc;
  }
  if (feat) {
    if ((rc = launch_prep_cand(c, feat, ld, m, d, dpad, c->ucand.p, ldk, c->cnorm.p))) return rc;
    c->ucand_cat = false;
    mark(c, "cnorm");
  }
  if (i8 && c->kstar_q && !c->cat_on && c->gp_x8.p) {
    // the distance contraction on the int8 MFMA (gp_kq.hip): beside the round's
    // hash its MFMAs issue under the hash's integer VALU work (C2 ~1 % per
    // round).  Categorical fits keep the fp64-MFMA K* (C3 HPL-64: K* 43 against
    // 28.5 ms, the round 288 against 270; C4 no better; scripts/r06_lines.sh)
    if ((rc = launch_gemm_kstar_q(c, true, c->gp_XsT, npad, c->ucand.p, dpad, m, c->kst.p, ldk, nullptr, -1, nullptr,
                                  nullptr, KstarCat(), nullptr, c->u8, c->scol)))
      return rc;
  } else if ((rc = launch_gemm_kstar(c, prec, cat ? c->gp_XsT_num.p : c->gp_XsT, npad, c->ucand.p, dpad, m, c->kst.p,
                                     ldk, kmu ? c->mu_part.p : nullptr, -1, nullptr, nullptr,
                                     cat ? kstar_cat(c, c->bcat.p) : KstarCat(), cat ? c->gp_xnorm_num.p : nullptr))) {
    return rc;
  }
  mark(c, "kstar");
  if (c->fit_pending && !kmu) UT_HIP(c, hipStreamWaitEvent(c->stream, c->ev_fit, 0));
  // fp64 / fp32 / h3: the variance GEMM runs alone, the side stream's hash +
  // dedup share the CUs with K* only (C2: 27.95 -> 28.2 ms per round when they
  // spilled into it, the GEMM at 0.74 instead of 0.80 of peak; round 1).  i8:
  // it starts when K* ends and the hash's tail runs beside it (only the
  // finalize needs the dup mask): C2 16.60 -> 16.40 ms at ell 0.2, 19.62 ->
  // 19.36 at ell 2, C3 / C4 unchanged (their hash ends before K*;
  // scripts/ab/r06_varjoin*.sh, r06_sched.sh)
  if (dup_ready && !i8) UT_HIP(c, hipStreamWaitEvent(c->stream, dup_ready, 0));
  mark(c, "var_wait");  // the wait for the fit (and the dup mask) is not variance time
  if (i8) {
    if ((rc = launch_gemm_var_i8(c, npad, reinterpret_cast<const int8_t*>(c->kst.p), ldk, m, c->var_part.p,
                                 c->mu_part.p)))
      return rc;
  } else if ((rc = launch_gemm_var(c, prec, fp32 ? (const void*)c->gp_LinvT_f : (const void*)c->gp_LinvT, npad,
                                   c->kst.p, ldk, npad, m, c->var_part.p, fp32 ? nullptr : c->gp_beta,
                                   fp32 ? nullptr : c->mu_part.p))) {
    return rc;
  }
  mark(c, "var");
  if (dup_ready) UT_HIP(c, hipStreamWaitEvent(c->stream, dup_ready, 0));
  if (i8) {
    // the bound test, then the fp64 recompute of the candidates it did not clear
    UT_HIP(c, hipMemsetAsync(c->pr_count.p, 0, sizeof(int64_t), c->stream));
    hipLaunchKernelGGL(k_gp_finalize_i8, dim3(grid1(m, 256)), dim3(256), 0, c->stream, m, 2 * RT, 2 * RT, c->mu_part.p,
                       c->var_part.p, ldk, c->gp_sf2, c->gp_stats, c->gp_flag, acq->kind, acq->xi, acq->kappa, dup,
                       mu, var, score, c->gp_i8rs.p + 2 * npad, c->i8_tol, n, c->pr_idx.p,
                       reinterpret_cast<unsigned long long*>(c->pr_count.p));
    UT_LAUNCH_CHECK(c);
    mark(c, "finalize");
    int64_t nf = 0;
    UT_HIP(c, hipMemcpyAsync(&nf, c->pr_count.p, sizeof(int64_t), hipMemcpyDeviceToHost, c->stream));
    UT_HIP(c, hipStreamSynchronize(c->stream));
    c->i8_recomputed = nf;
    if (nf > 0 && (rc = gp_ensure_linvt(c))) return rc;   // (the fp64 contraction reads (L^-1)^T)
    if (nf * 2 > m) {
      // most candidates need fp64: the whole K* (fp64, over the planes) and the
      // fp64 contraction, with the mean from its epilogue
      c->i8_recomputed = -1;
      if ((rc = ensure(c, c->pr_mpart, (size_t)RT * ldk))) return rc;
      if ((rc = launch_gemm_kstar(c, 64, cat ? c->gp_XsT_num.p : c->gp_XsT, npad, c->ucand.p, dpad, m, c->kst.p, ldk,
                                  nullptr, -1, nullptr, nullptr, cat ? kstar_cat(c, c->bcat.p) : KstarCat(),
                                  cat ? c->gp_xnorm_num.p : nullptr)))
        return rc;
      if ((rc = launch_gemm_var(c, 64, c->gp_LinvT, npad, c->kst.p, ldk, npad, m, c->var_part.p, c->gp_beta,
                                c->pr_mpart.p)))
        return rc;
      hipLaunchKernelGGL(k_gp_finalize, dim3(grid1(m, 256)), dim3(256), 0, c->stream, m, RT, RT, c->pr_mpart.p,
                         c->var_part.p, ldk, c->gp_sf2, c->gp_stats, c->gp_flag, acq->kind, acq->xi, acq->kappa, dup,
                         mu, var, score);
      UT_LAUNCH_CHECK(c);
    } else if (nf > 0) {
      const int64_t ldf = (nf + VAR_BN - 1) / VAR_BN * VAR_BN;
      if ((rc = ensure(c, c->pr_mpart, (size_t)RT * ldf))) return rc;
      if ((rc = gather_kstar_cols(c, cat, dpad, ldk, c->pr_idx.p, 0, nf, ldf))) return rc;
      if ((rc = launch_gemm_var(c, 64, c->gp_LinvT, npad, c->pr_kst.p, ldf, npad, nf, c->pr_vpart.p, c->gp_beta,
                                c->pr_mpart.p)))
        return rc;
      hipLaunchKernelGGL(k_gp_fix_i8, dim3(grid1(nf, 256)), dim3(256), 0, c->stream, nf, c->pr_idx.p, RT,
                         c->pr_mpart.p, c->pr_vpart.p, ldf, c->gp_sf2, c->gp_stats, acq->kind, acq->xi, acq->kappa,
                         dup, mu, var, score);
      UT_LAUNCH_CHECK(c);
    }
    mark(c, "recompute");
    return 0;
  }
  // h3's variance partials come per 256-row tile
  const int32_t RTv = prec == 16 ? (npad + 255) / 256 : RT;
  hipLaunchKernelGGL(k_gp_finalize, dim3(grid1(m, 256)), dim3(256), 0, c->stream, m, RT, RTv, c->mu_part.p,
                     c->var_part.p, ldk, c->gp_sf2, c->gp_stats, c->gp_flag, acq->kind, acq->xi, acq->kappa, dup,
                     mu, var, score);
  UT_LAUNCH_CHECK(c);
  mark(c, "finalize");
  return 0;
}


// ---------------------------------------------------------------------------
// Selection-exact EI-bound pruning (ut_gp_topk_pruned).
//   var = sf2 - sum_r (L^-1 k*)_r^2 and every term is >= 0, so the partial
//   sum over the first R row tiles bounds var from above; EI (and UCB with
//   kappa >= 0) increases with sigma, so the same holds for the score.  The
//   R-tile partials are bitwise the first R partials of the full GEMM (same
//   tiles, same k order) and fp addition of non-negative terms and sf2 - x are
//   monotone, so var_exact <= var_bound holds in floating point too; the score
//   bound gets a 1e-12 relative margin for the acquisition's own rounding.
// ---------------------------------------------------------------------------
// The score bound of a candidate from the first RTv row tiles of the
// variance contraction.  The mean is exact (every row's k* went into it).
//   var_ub = sf2 - S_R, S_R = the sum of the first RTv partials; the score of
//   var_ub, raised by a 1e-12 relative margin for the rounding of the
//   acquisition function, bounds the exact score from above.
//   Exactness test: the rows past the bound contribute at most
//   T = sum_{r >= R} v_r^2 <= |L^-1|_F^2 |k*|^2 (|v_r| <= |L^-1_r| |k*|), the
//   computed partials at most 1.001 T, and the exact path's running sum starts
//   from the same S_R (its first RTv partials are bitwise these) and only adds
//   non-negative terms, so its var lies in [max(sf2 - S_hi, 0), var_ub] with
//   S_hi = (S_R + 1.001 T)(1 + 2^-40).  When both ends round to the same double
//   the exact var IS var_ub, and so is the exact score: it is stored without
//   the margin and flagged exact, and ties with it can be broken by index
//   (a flat GP -- every k* ~ 0 -- gives every candidate the same score).
__global__ void k_prune_bound(int64_t m, int32_t RTm, const double* __restrict__ mu_part, int32_t RTv,
                              const double* __restrict__ var_part, int64_t ldp, double sf2,
                              const double* __restrict__ stats, const int32_t* __restrict__ fit_flag, int32_t kind,
                              double xi, double kappa, const uint8_t* __restrict__ dup, double* __restrict__ mu_out,
                              double* __restrict__ ub_out, const double* __restrict__ k2_part,
                              const double* __restrict__ linv_f2, uint8_t* __restrict__ exact_out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= m) return;
  double mu = 0.0, vs = 0.0, k2 = 0.0;
  for (int32_t r = 0; r < RTm; ++r) mu += mu_part[(int64_t)r * ldp + i];
  for (int32_t r = 0; r < RTv; ++r) vs += var_part[(int64_t)r * ldp + i];
  double var = sf2 - vs;
  var = var > 0.0 ? var : 0.0;
  double ub = acq_score(kind, mu, var, stats[0], xi, kappa);
  bool exact = false;
  if (k2_part && RTv < RTm) {
    for (int32_t r = 0; r < RTm; ++r) k2 += k2_part[(int64_t)r * ldp + i];
    const double tail = 1.001 * (*linv_f2) * k2;
    const double s_hi = (vs + tail) * (1.0 + 0x1p-40);
    double var_lo = sf2 - s_hi;
    var_lo = var_lo > 0.0 ? var_lo : 0.0;
    exact = tail == tail && var_lo == var;   // (NaN tail: not exact)
  } else if (RTv >= RTm) {
    exact = true;   // the bound GEMM covered every row
  }
  if (!exact) ub = ub + fabs(ub) * 1e-12 + 1e-300;
  if (*fit_flag != 0) {
    mu = ub = __builtin_nan("");
    exact = false;
  }
  if (dup && dup[i]) ub = -1.0 / 0.0;
  mu_out[i] = mu;
  ub_out[i] = ub;
  if (exact_out) exact_out[i] = exact ? 1 : 0;
}

// The bound of the f32 pass (ut_gp_set_prune_pass 32, k_gp_kstar_f32c): the
// stored bound rows in fp64 as before, every other k*^ = sf2 2^t^ with |k*^ -
// k*| <= rho k*^ / (1 - rho) + 2^-125 sf2 (v_exp_f32 flushes below 2^-126), its
// f32 tile sums within 2^-19 of sum |alpha| k*^.  rho = 2^dt (1 + 2^-21) - 1 per
// candidate, dt = (Kc + 9) 2^-24 (2 |c0| + max_r |x_r|^2 + |u|^2) / ln 2 (log2
// units; Kc the contraction length, c0 the categorical offset; the f32
// contraction's bound, see k_gp_kstar_f32c).  Per candidate:
//   mean  |mu - mu^| <= dmu = (rho / (1 - rho) + 2^-19) S + 2^-125 sf2 sum|alpha|
//         + RT 2^-51 sum_rt |mu^_rt|: S = sum_r |alpha_r| k*^_r over the f32 rows (part3),
//         mu the fp64 k* . alpha the survivors are scored with (k_gp_kstar's
//         fp64 epilogue on their columns: its bound-row tile partials are these
//         bitwise, its other tiles within the first term; the last term the
//         different rounding of the two sums over tiles);
//   bound rows  exact k*: var <= var_ub = sf2 - |v^_R|^2 (as k_prune_bound);
//   lower end (rows past R: |L^-1|_F^2 |k*|^2 as k_prune_bound's tail)
//         var >= var_lo = sf2 - (|v^_R|^2 + 1.001 |L^-1|_F^2 ((1 + rho') |k*^| +
//         sqrt(n) 2^-125 sf2)^2);
// the score bound is the acquisition at (mu^ - dmu, var_ub), raised by
// k_prune_bound's 1e-12 margin -- unless both ends pin the exact score: var_lo
// == var_ub and the mean's two ends give the same I = f_best - mu - xi (EI) or
// the same score (UCB); then the exact score is that double, stored as is and
// flagged exact (a flat GP keeps its index tie-break).  fp64 rounding of the
// sums: a 2^-36 margin.  cst: [0] |L^-1|_F^2, [1 + SQ_BLOCKS] sum |alpha|,
// [2 + SQ_BLOCKS] max_r |x_r|^2.
constexpr int SQ_BLOCKS = 1024;
__global__ void k_prune_bound32(int64_t m, int32_t RTm, const double* __restrict__ mu_part,
                                const double* __restrict__ sa_part, const double* __restrict__ k2_part, int32_t RTv,
                                const double* __restrict__ var_part, int64_t ldp, double sf2, int32_t n,
                                const double* __restrict__ stats, const int32_t* __restrict__ fit_flag, int32_t kind,
                                double xi, double kappa, const uint8_t* __restrict__ dup,
                                const double* __restrict__ cst, double* __restrict__ ub_out,
                                uint8_t* __restrict__ exact_out, int32_t Kc, double c0abs,
                                const double* __restrict__ cnorm) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= m) return;
  double mu = 0.0, mabs = 0.0, sa = 0.0, k2 = 0.0, vs = 0.0;
  for (int32_t r = 0; r < RTm; ++r) {
    const int64_t o = (int64_t)r * ldp + i;
    mu += mu_part[o];
    mabs += fabs(mu_part[o]);
    sa += sa_part[o];
    k2 += k2_part[o];
  }
  for (int32_t r = 0; r < RTv; ++r) vs += var_part[(int64_t)r * ldp + i];
  const double F2 = cst[0], A1 = cst[1 + SQ_BLOCKS];
  const double tiny = 0x1p-125 * sf2;
  const double dt = (Kc + 9.0) * 0x1p-24 * (2.0 * c0abs + cst[2 + SQ_BLOCKS] + cnorm[i]) * 1.4426950408889634 *
                        (1.0 + 0x1p-20) + Kc * 0x1p-120;
  const double rho = (exp2(dt) * (1.0 + 0x1p-21) - 1.0) * (1.0 + 0x1p-20) + 0x1p-50;
  const double rp = rho / (1.0 - rho);   // |k*^ - k*| / k*^ (rho < 1/2, or the bound is useless: NaN below)
  const double dmu = ((rp + 0x1p-19) * sa * (1.0 + 0x1p-18) + tiny * A1 + (double)RTm * 0x1p-51 * mabs) *
                     (1.0 + 0x1p-20);
  double var_ub = sf2 - vs;   // the bound rows' partials: bitwise the exact GEMM's first RTv (k_prune_bound)
  var_ub = var_ub > 0.0 ? var_ub : 0.0;
  const double kn = (1.0 + rp) * sqrt(k2 * (1.0 + 0x1p-18)) + sqrt((double)n) * tiny;
  const double tail = 1.001 * F2 * kn * kn;
  double var_lo = sf2 - (vs + tail) * (1.0 + 0x1p-36);
  var_lo = var_lo > 0.0 ? var_lo : 0.0;
  double ub = acq_score(kind, mu - dmu, var_ub, stats[0], xi, kappa);
  bool exact = var_lo == var_ub && dmu == dmu;
  if (exact) {
    if (kind == UT_ACQ_UCB)
      exact = ub == acq_score(kind, mu + dmu, var_lo, stats[0], xi, kappa);
    else
      exact = (stats[0] - (mu - dmu) - xi) == (stats[0] - (mu + dmu) - xi);
  }
  if (!exact) ub = ub + fabs(ub) * 1e-12 + 1e-300;
  if (!(rho < 0.5)) {   // no usable bound: the candidate survives
    ub = 1.0 / 0.0;
    exact = false;
  }
  if (*fit_flag != 0) {
    ub = __builtin_nan("");
    exact = false;
  }
  if (dup && dup[i]) ub = -1.0 / 0.0;
  ub_out[i] = ub;
  exact_out[i] = exact ? 1 : 0;
}

// max of x[0 .. n) (one workgroup): the f32-contraction bound's max_r |x_r|^2
__global__ __launch_bounds__(256) void k_max_n(const double* __restrict__ x, int32_t n, double* __restrict__ out) {
  __shared__ double red[4];
  double v = 0.0;
  for (int32_t e = threadIdx.x; e < n; e += 256) v = fmax(v, x[e]);
  for (int d = 32; d > 0; d >>= 1) v = fmax(v, __shfl_xor(v, d, 64));
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x == 0) *out = fmax(fmax(red[0], red[1]), fmax(red[2], red[3]));
}

// sum of squares of cnt doubles (|L^-1|_F^2), deterministic: pass 1 writes one
// partial per block (grid-stride), pass 2 (one block) adds them in order
template <bool ABS>   // ABS: sum |x| instead
__global__ __launch_bounds__(256) void k_sumsq_part(const double* __restrict__ x, int64_t cnt,
                                                    double* __restrict__ part) {
  __shared__ double red[4];
  double s = 0.0;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < cnt; e += (int64_t)gridDim.x * 256)
    s += ABS ? fabs(x[e]) : x[e] * x[e];
  for (int d = 32; d > 0; d >>= 1) s += __shfl_xor(s, d, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) part[blockIdx.x] = (red[0] + red[1]) + (red[2] + red[3]);
}
__global__ __launch_bounds__(256) void k_sumsq_final(const double* __restrict__ part, int32_t n,
                                                     double* __restrict__ out) {
  __shared__ double red[4];
  double s = 0.0;
  for (int32_t e = threadIdx.x; e < n; e += 256) s += part[e];
  for (int d = 32; d > 0; d >>= 1) s += __shfl_xor(s, d, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) *out = (red[0] + red[1]) + (red[2] + red[3]);
}

// the categorical K* codes of gathered candidates: 16-byte pieces of their
// 128-byte rows, code block blockIdx.y (zeros past n and for empty slots)
__global__ void k_gather_code_rows(const int8_t* __restrict__ bcat, int64_t ldk, const int64_t* __restrict__ idx,
                                   int64_t base, int64_t n, int64_t ldo, int8_t* __restrict__ out) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t kb = blockIdx.y;
  const int64_t j = e >> 3;
  const int piece = (int)(e & 7);
  if (j >= ldo) return;
  uint4 v = make_uint4(0u, 0u, 0u, 0u);
  if (j < n) {
    const int64_t q = idx[j];
    if (q >= 0) v = reinterpret_cast<const uint4*>(bcat + (kb * ldk + (q - base)) * 128)[piece];
  }
  reinterpret_cast<uint4*>(out + (kb * ldo + j) * 128)[piece] = v;
}

__global__ void k_gather_cols(const double* __restrict__ kst, int64_t ldk, const int64_t* __restrict__ idx,
                                  int64_t base, int64_t n, int64_t ldo, double* __restrict__ out) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t r = blockIdx.y;
  if (j >= ldo) return;
  double v = 0.0;
  if (j < n) {
    const int64_t q = idx[j];
    if (q >= 0) v = kst[r * ldk + (q - base)];
  }
  out[r * ldo + j] = v;
}

// exact scores of the gathered candidates: compact[j], and scattered to full[idx[j]]
// mu_full: the bound pass's exact mean by global index; or (nullptr) the fp64
// mean partials k* . alpha of these columns' K* (gather_kstar_cols: the f32
// bound pass has no exact mean)
__global__ void k_prune_exact(int64_t n, const int64_t* __restrict__ idx, int64_t base, int32_t RT,
                              const double* __restrict__ var_part, int64_t ldp, const double* __restrict__ mu_full,
                              double sf2, const double* __restrict__ stats, const int32_t* __restrict__ fit_flag,
                              int32_t kind, double xi, double kappa, double* __restrict__ compact,
                              double* __restrict__ full, const double* __restrict__ mu_part) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  const int64_t q = idx[j];
  if (q < 0) {
    if (compact) compact[j] = -1.0 / 0.0;
    return;
  }
  double vs = 0.0, mu = 0.0;
  for (int32_t r = 0; r < RT; ++r) vs += var_part[(int64_t)r * ldp + j];
  if (mu_full) {
    mu = mu_full[q - base];
  } else {
    for (int32_t r = 0; r < RT; ++r) mu += mu_part[(int64_t)r * ldp + j];
  }
  double var = sf2 - vs;
  var = var > 0.0 ? var : 0.0;
  double sc = acq_score(kind, mu, var, stats[0], xi, kappa);
  if (*fit_flag != 0) sc = __builtin_nan("");
  if (compact) compact[j] = sc;
  if (full) full[q - base] = sc;
}

// survivors: bound >= tau (tau = the k-th best exact score of the threshold
// set, a device scalar); appended with one atomic per wave
// survivors: candidates that may be in the top-k.  An exact candidate (its
// stored score is its exact score) survives iff (score, -index) >= (tau,
// -tau_index), the k-th best pair of the threshold set -- a lower bound on the
// k-th best pair overall; any other survives iff its bound >= tau.
__global__ void k_prune_survivors(int64_t m, const double* __restrict__ ub, const double* __restrict__ tau_p,
                                  const int64_t* __restrict__ tau_idx_p, const uint8_t* __restrict__ exact,
                                  int64_t cand_base, int64_t* __restrict__ out, unsigned long long* __restrict__ count) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int lane = threadIdx.x & 63;
  const double tau = *tau_p;
  const int64_t tau_g = *tau_idx_p;
  bool keep = false;
  if (i < m) {
    const double b = ub[i];
    if (exact && exact[i])
      keep = b > tau || (b == tau && (tau_g < 0 || cand_base + i <= tau_g));
    else
      keep = b >= tau;
  }
  const unsigned long long ball = __ballot(keep);
  const uint32_t n = __builtin_popcountll(ball);
  unsigned long long base = 0;
  if (lane == 0 && n) base = atomicAdd(count, (unsigned long long)n);
  base = __shfl(base, 0, 64);
  if (keep) out[base + __builtin_popcountll(ball & ((1ull << lane) - 1ull))] = i;
}

__global__ void k_fill(double* __restrict__ p, int64_t n, double v) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = v;
}

// full fp64 K* columns of the candidates idx[0..nc) (global indices - base;
// idx < 0: an empty slot) into c->pr_kst [npad][ldc]: their scaled features
// and norms (and categorical codes) gathered from the K* operands of the
// round (c->ucand / c->cnorm / c->bcat, leading dimension ldk), then the K*
// GEMM on those columns only (pruned scoring's threshold set and survivors,
// precision 8's flagged candidates); mu_part: also their fp64 mean partials
// k* . alpha per row tile [RT][ldc] (pruned scoring's f32 bound pass)
static int gather_kstar_cols(ut_ctx* c, bool cat, int32_t dpad, int64_t ldk, const int64_t* idx, int64_t base,
                             int64_t nc, int64_t ldc, double* mu_part) {
  const int32_t npad = ((c->gp_n + NPAD - 1) / NPAD) * NPAD;
  const int32_t RT = npad / NPAD;
  const double* XsT = cat ? c->gp_XsT_num.p : c->gp_XsT;
  const double* xn = cat ? c->gp_xnorm_num.p : nullptr;
  int r2;
  if ((r2 = ensure(c, c->pr_kst, (size_t)npad * ldc))) return r2;
  if ((r2 = ensure(c, c->pr_vpart, (size_t)RT * ldc))) return r2;
  if ((r2 = ensure(c, c->pr_ucand, (size_t)(dpad > 0 ? dpad : 1) * ldc))) return r2;
  if ((r2 = ensure(c, c->pr_cnorm, (size_t)ldc))) return r2;
  if (dpad > 0)
    hipLaunchKernelGGL(k_gather_cols, dim3(grid1(ldc, 256), (unsigned)dpad), dim3(256), 0, c->stream, c->ucand.p,
                       ldk, idx, base, nc, ldc, c->pr_ucand.p);
  hipLaunchKernelGGL(k_gather_cols, dim3(grid1(ldc, 256), 1u), dim3(256), 0, c->stream, c->cnorm.p, ldk, idx, base,
                     nc, ldc, c->pr_cnorm.p);
  if (cat) {   // the gathered candidates' 128-byte code rows, per code block
    if ((r2 = ensure(c, c->pr_bcat, (size_t)c->space.cat_k * ldc))) return r2;
    hipLaunchKernelGGL(k_gather_code_rows, dim3(grid1(ldc * 8, 256), (unsigned)(c->space.cat_k / 128)), dim3(256), 0,
                       c->stream, c->bcat.p, ldk, idx, base, nc, ldc, c->pr_bcat.p);
  }
  UT_LAUNCH_CHECK(c);
  return launch_gemm_kstar(c, 64, XsT, npad, c->pr_ucand.p, dpad, nc, c->pr_kst.p, ldc, mu_part, -1,
                           c->pr_cnorm.p, nullptr, cat ? kstar_cat(c, c->pr_bcat.p) : KstarCat(), xn);
}

int gp_topk_pruned_impl(ut_ctx* c, const double* feat, int64_t ld, int64_t m, const ut_acq* acq, const uint8_t* dup,
                        int64_t cand_base, int32_t k, int32_t bound_rows, int64_t* out_idx, double* out_score,
                        ut_prune_stats* stats, hipEvent_t dup_ready, bool feat_ours) {
  UT_CHECK(c, c->gp_ready, UT_EINVAL, "gp_topk_pruned: call ut_gp_fit first");
  UT_CHECK(c, c->gp_fit_prec == 64, UT_EINVAL, "gp_topk_pruned: needs an fp64 fit (ut_gp_set_precision 64)");
  UT_CHECK(c, acq->kind == UT_ACQ_EI || (acq->kind == UT_ACQ_UCB && acq->kappa >= 0.0), UT_EINVAL,
           "gp_topk_pruned: the score must increase with sigma (EI, or UCB with kappa >= 0)");
  UT_CHECK(c, k >= 1 && k <= 1024, UT_EINVAL, "gp_topk_pruned: k must be in [1, 1024]");
  if (int rc0 = gp_fit_flush(c)) return rc0;
  // the candidates' K* operands need only the fit's scaled inputs (1/ell):
  // they are prepared while the factorisation still runs, and K* then waits
  // for the whole fit (C3 pruned: the 2.8-ms categorical prep came off the
  // critical path, scripts/ab/r04ad_prep_early.sh)
  if (c->fit_pending) UT_HIP(c, hipStreamWaitEvent(c->stream, c->ev_fit_x, 0));
  const int32_t n = c->gp_n, d = c->gp_d;
  const int32_t npad = ((n + NPAD - 1) / NPAD) * NPAD;
  // feat == nullptr: the K* operands are already in c->ucand / c->cnorm (/ c->bcat),
  // from gp_encode_scaled (a scoring round's fused encode)
  const bool cat = feat ? feat_ours && c->cat_on : c->ucand_cat;   // the categorical K* (ut's encoder)
  const int32_t dpad = cat ? cat_dpad(c) : kstar_dpad(d);
  const int32_t RT = npad / NPAD;
  int32_t R = (bound_rows + NPAD - 1) / NPAD;
  R = R < 1 ? 1 : (R > RT ? RT : R);
  const int64_t ldk = ((m + VAR_BN - 1) / VAR_BN) * VAR_BN;
  int rc;
  if ((rc = ensure(c, c->kst, (size_t)npad * ldk))) return rc;
  if ((rc = ensure(c, c->mu_part, (size_t)RT * ldk))) return rc;
  if ((rc = ensure(c, c->var_part, (size_t)RT * ldk))) return rc;
  if ((rc = ensure(c, c->pr_mpart, (size_t)RT * ldk))) return rc;
  if ((rc = ensure(c, c->cnorm, (size_t)ldk))) return rc;
  if ((rc = ensure(c, c->ucand, (size_t)(dpad > 0 ? dpad : 1) * ldk))) return rc;
  if (cat && (rc = ensure(c, c->bcat, (size_t)c->space.cat_k * ldk))) return rc;
  if ((rc = ensure(c, c->pr_mu, (size_t)ldk))) return rc;
  if ((rc = ensure(c, c->pr_ub, (size_t)ldk))) return rc;
  if ((rc = ensure(c, c->pr_score, (size_t)ldk + 2048))) return rc;   // + the threshold set's two [1024] arrays
  if ((rc = ensure(c, c->pr_idx, (size_t)ldk + 2048))) return rc;
  if ((rc = ensure(c, c->pr_count, 1))) return rc;
  if ((rc = ensure(c, c->pr_k2, (size_t)RT * ldk))) return rc;
  // [0] |L^-1|_F^2, [1..] block partials, then the f32 passes' sum |alpha|, max |x|^2
  if ((rc = ensure(c, c->pr_f2, 3 + SQ_BLOCKS))) return rc;
  const bool f32 = c->prune_pass == 32;   // the bound pass in f32 (k_gp_kstar_f32c)
  if (f32 && (rc = ensure(c, c->pr_sa, (size_t)RT * ldk))) return rc;
  if (f32 && (rc = ensure(c, c->pr_gmu, (size_t)RT * (ldk + 1024)))) return rc;   // survivors / threshold set
  if ((rc = ensure(c, c->pr_exact, (size_t)ldk))) return rc;
  const double* LinvT = c->gp_LinvT;
  // 1. K* with the mean in its epilogue, 2. the first R row tiles of L^-1 K*^T
  if (feat) {
    if (cat) {
      if ((rc = launch_prep_cand_cat(c, feat, ld, m, c->ucand.p, dpad, ldk, c->cnorm.p, c->bcat.p))) return rc;
    } else if ((rc = launch_prep_cand(c, feat, ld, m, d, dpad, c->ucand.p, ldk, c->cnorm.p))) {
      return rc;
    }
    c->ucand_cat = cat;
    mark(c, "prep");
  }
  if (c->fit_pending) UT_HIP(c, hipStreamWaitEvent(c->stream, c->ev_fit, 0));   // K* takes mu = k* . alpha
  mark(c, "fit_wait");   // (the wait is not K* time)
  const double* XsT = cat ? c->gp_XsT_num.p : c->gp_XsT;
  const double* xn = cat ? c->gp_xnorm_num.p : nullptr;
  // K* stores only the bound rows; the mean sums every row.  The few
  // candidates that need every row (threshold set, survivors) get their K*
  // columns recomputed from their features (recompute_cols below): cheaper than
  // writing and re-reading the whole n x m matrix
  if (f32) {
    // the bound rows through the fp64 kernel (tiles < R), every other tile
    // through k_gp_kstar_f32c on f32 copies of the operands (Xs^T once per fit)
    const double* xnn = xn ? xn : c->gp_xnorm;
    // the f32 copy depends on the operand as well as the fit: the numeric
    // block (categorical mode, cat_dpad rows, gp_xnorm_num) or every feature
    // (kstar_dpad rows, gp_xnorm) -- within one categorical fit the feature
    // entry (ut_gp_topk_pruned: cat = false) and the fused DE round (cat =
    // true) take different ones, so the cache is keyed on (fit, cat, dpad)
    if (!c->pr_xf_valid || c->pr_xf_cat != cat || c->pr_xf_dpad != dpad) {
      if ((rc = ensure(c, c->pr_xsT_f, (size_t)dpad * npad))) return rc;
      if ((rc = launch_to_f32(c, XsT, c->pr_xsT_f.p, (int64_t)dpad * npad))) return rc;
      hipLaunchKernelGGL(k_max_n, dim3(1), dim3(256), 0, c->stream, xnn, n, c->pr_f2.p + 2 + SQ_BLOCKS);
      UT_LAUNCH_CHECK(c);
      c->pr_xf_valid = true;
      c->pr_xf_cat = cat;
      c->pr_xf_dpad = dpad;
    }
    if ((rc = ensure(c, c->pr_ucand_f, (size_t)(dpad > 0 ? dpad : 1) * ldk))) return rc;
    if ((rc = launch_to_f32(c, c->ucand.p, c->pr_ucand_f.p, (int64_t)dpad * ldk))) return rc;
    if ((rc = launch_gemm_kstar(c, 64, XsT, npad, c->ucand.p, dpad, m, c->kst.p, ldk, c->mu_part.p, R * NPAD,
                                nullptr, c->pr_k2.p, cat ? kstar_cat(c, c->bcat.p) : KstarCat(), xn, R)))
      return rc;
    UT_HIP(c, hipMemsetAsync(c->pr_sa.p, 0, sizeof(double) * R * ldk, c->stream));
    if (R < RT &&
        (rc = launch_gemm_kstar_f32c(c, c->pr_xsT_f.p, npad, c->pr_ucand_f.p, dpad, m, ldk, R, c->mu_part.p,
                                     c->pr_k2.p, c->pr_sa.p, cat ? kstar_cat(c, c->bcat.p) : KstarCat(), xnn,
                                     c->cnorm.p)))
      return rc;
  } else if ((rc = launch_gemm_kstar(c, 64, XsT, npad, c->ucand.p, dpad, m, c->kst.p, ldk, c->mu_part.p, R * NPAD,
                                     nullptr, c->pr_k2.p, cat ? kstar_cat(c, c->bcat.p) : KstarCat(), xn))) {
    return rc;
  }
  // |L^-1|_F^2 for the variance tail bound, once per fit (the block partials
  // in pr_f2[1..] are scratch, reused pass after pass in stream order)
  auto sumsq = [&](bool abs_, const double* x, int64_t cnt, double* out) -> int {
    if (abs_)
      hipLaunchKernelGGL(k_sumsq_part<true>, dim3(SQ_BLOCKS), dim3(256), 0, c->stream, x, cnt, c->pr_f2.p + 1);
    else
      hipLaunchKernelGGL(k_sumsq_part<false>, dim3(SQ_BLOCKS), dim3(256), 0, c->stream, x, cnt, c->pr_f2.p + 1);
    hipLaunchKernelGGL(k_sumsq_final, dim3(1), dim3(256), 0, c->stream, c->pr_f2.p + 1, SQ_BLOCKS, out);
    UT_LAUNCH_CHECK(c);
    return 0;
  };
  if (!c->pr_f2_valid) {
    if ((rc = sumsq(false, c->gp_Linv, (int64_t)npad * npad, c->pr_f2.p))) return rc;
    c->pr_f2_valid = true;
  }
  if (f32 && !c->pr_ab_valid) {   // the f32 bound's per-fit constants
    double* cst = c->pr_f2.p + 1 + SQ_BLOCKS;
    if ((rc = sumsq(true, c->gp_alpha, n, cst))) return rc;
    c->pr_ab_valid = true;
  }
  mark(c, "kstar");
  if ((rc = launch_gemm_var(c, 64, LinvT, npad, c->kst.p, ldk, R * NPAD, m, c->var_part.p, c->gp_beta,
                            c->pr_mpart.p)))
    return rc;
  mark(c, "bound");
  if (dup_ready) UT_HIP(c, hipStreamWaitEvent(c->stream, dup_ready, 0));   // the dup mask (side stream)
  if (f32)
    hipLaunchKernelGGL(k_prune_bound32, dim3(grid1(m, 256)), dim3(256), 0, c->stream, m, RT, c->mu_part.p,
                       c->pr_sa.p, c->pr_k2.p, R, c->var_part.p, ldk, c->gp_sf2, n, c->gp_stats, c->gp_flag,
                       acq->kind, acq->xi, acq->kappa, dup, c->pr_f2.p, c->pr_ub.p, c->pr_exact.p,
                       dpad + (cat ? 1 : 0), cat ? fabs(c->cat_c0) : 0.0, c->cnorm.p);
  else
    hipLaunchKernelGGL(k_prune_bound, dim3(grid1(m, 256)), dim3(256), 0, c->stream, m, RT, c->mu_part.p, R,
                       c->var_part.p, ldk, c->gp_sf2, c->gp_stats, c->gp_flag, acq->kind, acq->xi, acq->kappa, dup,
                       c->pr_mu.p, c->pr_ub.p, c->pr_k2.p, c->pr_f2.p, c->pr_exact.p);
  UT_LAUNCH_CHECK(c);
  // 3. threshold: exact scores of the best 1024 bounds, tau = their k-th best
  const int32_t kp = (int32_t)(m < 1024 ? m : 1024);
  int64_t* tset = c->pr_idx.p + ldk;                   // [1024] threshold set (global indices)
  double* tsc = c->pr_score.p + ldk;                   // [1024] their bounds
  double* tex = c->pr_score.p + ldk + 1024;            // [1024] their exact scores
  if ((rc = topk_impl(c, c->pr_ub.p, dup, m, cand_base, kp < k ? k : kp, tset, tsc))) return rc;
  // (the f32 pass has no exact mean: the recomputed columns' fp64 k* . alpha)
  double* gmu = f32 ? c->pr_gmu.p : nullptr;
  auto recompute_cols = [&](const int64_t* idx, int64_t base, int64_t nc, int64_t ldc) -> int {
    return gather_kstar_cols(c, cat, dpad, ldk, idx, base, nc, ldc, gmu);
  };
  const int64_t ldt = ((int64_t)kp + VAR_BN - 1) / VAR_BN * VAR_BN;
  if ((rc = recompute_cols(tset, cand_base, kp, ldt))) return rc;
  if ((rc = launch_gemm_var(c, 64, LinvT, npad, c->pr_kst.p, ldt, npad, kp, c->pr_vpart.p, c->gp_beta,
                            c->pr_mpart.p)))
    return rc;
  const double* mu_full = f32 ? nullptr : c->pr_mu.p;
  hipLaunchKernelGGL(k_prune_exact, dim3(grid1(kp, 256)), dim3(256), 0, c->stream, (int64_t)kp, tset, cand_base, RT,
                     c->pr_vpart.p, ldt, mu_full, c->gp_sf2, c->gp_stats, c->gp_flag, acq->kind, acq->xi,
                     acq->kappa, tex, nullptr, gmu);
  UT_LAUNCH_CHECK(c);
  int64_t* tk_i = out_idx;   // the caller's [k] outputs hold tau's top-k for now
  double* tk_s = out_score;
  // tau: the k-th best (exact score, global index) pair of the threshold set
  if ((rc = topk_pairs_impl(c, tex, tset, kp, k, tk_i, tk_s))) return rc;
  // 4. survivors: bound >= tau
  UT_HIP(c, hipMemsetAsync(c->pr_count.p, 0, sizeof(int64_t), c->stream));
  hipLaunchKernelGGL(k_prune_survivors, dim3(grid1(m, 256)), dim3(256), 0, c->stream, m, c->pr_ub.p, tk_s + (k - 1),
                     tk_i + (k - 1), c->pr_exact.p, cand_base, c->pr_idx.p,
                     reinterpret_cast<unsigned long long*>(c->pr_count.p));
  UT_LAUNCH_CHECK(c);
  int64_t ns = 0;
  double tau = 0.0;
  UT_HIP(c, hipMemcpyAsync(&ns, c->pr_count.p, sizeof(int64_t), hipMemcpyDeviceToHost, c->stream));
  UT_HIP(c, hipMemcpyAsync(&tau, tk_s + (k - 1), sizeof(double), hipMemcpyDeviceToHost, c->stream));
  UT_HIP(c, hipStreamSynchronize(c->stream));
  mark(c, "prune");
  const bool dense = ns * 2 > m;
  if (dense) {
    // most candidates survive: the whole K* (this time every row) and the dense variance
    if ((rc = launch_gemm_kstar(c, 64, XsT, npad, c->ucand.p, dpad, m, c->kst.p, ldk, c->mu_part.p, -1, nullptr,
                                nullptr, cat ? kstar_cat(c, c->bcat.p) : KstarCat(), xn)))
      return rc;
    if ((rc = launch_gemm_var(c, 64, LinvT, npad, c->kst.p, ldk, npad, m, c->var_part.p, c->gp_beta,
                              c->pr_mpart.p)))
      return rc;
    hipLaunchKernelGGL(k_gp_finalize, dim3(grid1(m, 256)), dim3(256), 0, c->stream, m, RT, RT, c->mu_part.p,
                       c->var_part.p, ldk, c->gp_sf2, c->gp_stats, c->gp_flag, acq->kind, acq->xi, acq->kappa, dup,
                       nullptr, nullptr, c->pr_score.p);
    UT_LAUNCH_CHECK(c);
  } else {
    // 5. the full variance for the survivors only, their exact scores into a -inf array
    hipLaunchKernelGGL(k_fill, dim3(grid1(m, 256)), dim3(256), 0, c->stream, c->pr_score.p, m, -1.0 / 0.0);
    UT_LAUNCH_CHECK(c);
    if (ns > 0) {
      const int64_t lds = (ns + VAR_BN - 1) / VAR_BN * VAR_BN;
      if ((rc = recompute_cols(c->pr_idx.p, 0, ns, lds))) return rc;
      if ((rc = launch_gemm_var(c, 64, LinvT, npad, c->pr_kst.p, lds, npad, ns, c->pr_vpart.p, c->gp_beta,
                                c->pr_mpart.p)))
        return rc;
      hipLaunchKernelGGL(k_prune_exact, dim3(grid1(ns, 256)), dim3(256), 0, c->stream, ns, c->pr_idx.p, (int64_t)0,
                         RT, c->pr_vpart.p, lds, mu_full, c->gp_sf2, c->gp_stats, c->gp_flag, acq->kind, acq->xi,
                         acq->kappa, nullptr, c->pr_score.p, gmu);
      UT_LAUNCH_CHECK(c);
    }
  }
  mark(c, "var");
  if ((rc = topk_impl(c, c->pr_score.p, dup, m, cand_base, k, out_idx, out_score))) return rc;
  mark(c, "topk");
  if (stats) {
    stats->survivors = dense ? m : ns;
    stats->bound_rows = R * NPAD;
    stats->dense = dense ? 1 : 0;
    stats->threshold = tau;
  }
  return 0;
}

}  // namespace ut
