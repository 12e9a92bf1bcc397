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
// ut_gp_set_precision(ctx, 32)).
#include "ut_internal.h"

namespace ut {

constexpr int NB = 64;     // Cholesky / inverse block
constexpr int NPAD = 128;  // training set padded to the GEMM row tile

// ---------------------------------------------------------------------------
// fit
// ---------------------------------------------------------------------------
__global__ void k_gp_prep_train(const double* __restrict__ X, int32_t n, int32_t npad, int32_t d,
                                const double* __restrict__ inv_ell, double* __restrict__ Xs,
                                double* __restrict__ xnorm) {
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

__global__ void k_gp_kmat(const double* __restrict__ Xs, const double* __restrict__ xnorm, int32_t n, int32_t npad,
                          int32_t d, double sf2, double diag, double* __restrict__ K) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= (int64_t)npad * npad) return;
  const int32_t i = (int32_t)(e / npad), j = (int32_t)(e % npad);
  double v;
  if (i >= n || j >= n) {
    v = (i == j) ? 1.0 : 0.0;  // identity padding keeps the factorisation exact
  } else {
    double dot = 0.0;
    for (int32_t k = 0; k < d; ++k) dot += Xs[(int64_t)i * d + k] * Xs[(int64_t)j * d + k];
    double d2 = xnorm[i] + xnorm[j] - 2.0 * dot;
    d2 = d2 > 0.0 ? d2 : 0.0;
    v = sf2 * exp(-0.5 * d2);
    if (i == j) v += diag;
  }
  K[e] = v;
}

// mean / std (ddof=0) / standardise / f_best = min(ys); one workgroup
__global__ __launch_bounds__(256) void k_gp_ystats(const double* __restrict__ y, int32_t n, int32_t npad,
                                                   double* __restrict__ ys, double* __restrict__ stats) {
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

// unblocked Cholesky of a NB x NB block held in LDS (row-major, stride NB+1)
__device__ void lds_chol(double* A, int32_t* flag) {
  const int t = threadIdx.x;
  for (int c = 0; c < NB; ++c) {
    if (t == 0) {
      const double dv = A[c * (NB + 1) + c];
      if (!(dv > 0.0)) atomicOr(flag, 1);
      A[c * (NB + 1) + c] = sqrt(dv > 0.0 ? dv : 1e-300);
    }
    __syncthreads();
    const double piv = A[c * (NB + 1) + c];
    for (int r = c + 1 + t; r < NB; r += blockDim.x) A[r * (NB + 1) + c] /= piv;
    __syncthreads();
    const int rem = NB - c - 1;
    for (int e = t; e < rem * rem; e += blockDim.x) {
      const int r = c + 1 + e / rem, s = c + 1 + e % rem;
      if (s <= r) A[r * (NB + 1) + s] -= A[r * (NB + 1) + c] * A[s * (NB + 1) + c];
    }
    __syncthreads();
  }
}

// Panel kb: every workgroup factors the diagonal block; workgroup 0 writes
// it back, workgroup w >= 1 solves row block kb + w:  X L_kk^T = A.
__global__ __launch_bounds__(256) void k_chol_panel(double* __restrict__ K, int32_t npad, int32_t kb,
                                                    int32_t* flag) {
  __shared__ double Lkk[NB * (NB + 1)];
  __shared__ double Ab[NB * (NB + 1)];
  const int t = threadIdx.x;
  const int64_t base = (int64_t)kb * NB;
  for (int e = t; e < NB * NB; e += blockDim.x) {
    const int r = e / NB, s = e % NB;
    Lkk[r * (NB + 1) + s] = K[(base + r) * npad + base + s];
  }
  __syncthreads();
  lds_chol(Lkk, flag);
  if (blockIdx.x == 0) {
    for (int e = t; e < NB * NB; e += blockDim.x) {
      const int r = e / NB, s = e % NB;
      K[(base + r) * npad + base + s] = (s <= r) ? Lkk[r * (NB + 1) + s] : 0.0;
    }
    return;
  }
  const int64_t rb = (int64_t)(kb + blockIdx.x) * NB;
  for (int e = t; e < NB * NB; e += blockDim.x) {
    const int r = e / NB, s = e % NB;
    Ab[r * (NB + 1) + s] = K[(rb + r) * npad + base + s];
  }
  __syncthreads();
  if (t < NB) {
    double* row = Ab + t * (NB + 1);
    for (int c = 0; c < NB; ++c) {
      double v = row[c];
      for (int s = 0; s < c; ++s) v -= row[s] * Lkk[c * (NB + 1) + s];
      row[c] = v / Lkk[c * (NB + 1) + c];
    }
  }
  __syncthreads();
  for (int e = t; e < NB * NB; e += blockDim.x) {
    const int r = e / NB, s = e % NB;
    K[(rb + r) * npad + base + s] = Ab[r * (NB + 1) + s];
  }
}

// Trailing update A_ij -= L_i,kb L_j,kb^T for kb < j <= i < nb.
__global__ __launch_bounds__(256) void k_chol_update(double* __restrict__ K, int32_t npad, int32_t kb) {
  __shared__ double Li[NB * (NB + 1)];
  __shared__ double Lj[NB * (NB + 1)];
  // linear tile id -> (i, j), j <= i, both in (kb, nb)
  int32_t tid = blockIdx.x;
  int32_t i = 0;
  while ((i + 1) * (i + 2) / 2 <= tid) ++i;
  const int32_t j = tid - i * (i + 1) / 2;
  const int64_t ib = (int64_t)(kb + 1 + i) * NB, jb = (int64_t)(kb + 1 + j) * NB, cb = (int64_t)kb * NB;
  const int t = threadIdx.x;
  for (int e = t; e < NB * NB; e += blockDim.x) {
    const int r = e / NB, s = e % NB;
    Li[r * (NB + 1) + s] = K[(ib + r) * npad + cb + s];
    Lj[r * (NB + 1) + s] = K[(jb + r) * npad + cb + s];
  }
  __syncthreads();
  for (int e = t; e < NB * NB; e += blockDim.x) {
    const int r = e / NB, s = e % NB;
    double acc = 0.0;
    for (int q = 0; q < NB; ++q) acc += Li[r * (NB + 1) + q] * Lj[s * (NB + 1) + q];
    K[(ib + r) * npad + jb + s] -= acc;
  }
}

// invert the lower-triangular NB x NB block in S (stride NB+1) into X
__device__ void lds_trinv(const double* S, double* X) {
  const int t = threadIdx.x;
  if (t < NB) {
    const int c = t;
    for (int r = 0; r < NB; ++r) {
      double v;
      if (r < c) {
        v = 0.0;
      } else {
        v = (r == c) ? 1.0 : 0.0;
        for (int s = c; s < r; ++s) v -= S[r * (NB + 1) + s] * X[s * (NB + 1) + c];
        v /= S[r * (NB + 1) + r];
      }
      X[r * (NB + 1) + c] = v;
    }
  }
  __syncthreads();
}

// Block row I of L^-1:  Linv_IJ = -inv(L_II) * sum_{K=J}^{I-1} L_IK Linv_KJ
__global__ __launch_bounds__(256) void k_trinv_row(const double* __restrict__ L, double* __restrict__ Li,
                                                   int32_t npad, int32_t I) {
  __shared__ double S[NB * (NB + 1)];
  __shared__ double X[NB * (NB + 1)];
  __shared__ double T[NB * (NB + 1)];
  const int t = threadIdx.x;
  const int32_t J = blockIdx.x;
  const int64_t Ib = (int64_t)I * NB, Jb = (int64_t)J * NB;
  for (int e = t; e < NB * NB; e += blockDim.x) {
    const int r = e / NB, s = e % NB;
    S[r * (NB + 1) + s] = L[(Ib + r) * npad + Ib + s];
  }
  __syncthreads();
  lds_trinv(S, X);
  if (J == I) {
    for (int e = t; e < NB * NB; e += blockDim.x) {
      const int r = e / NB, s = e % NB;
      Li[(Ib + r) * npad + Ib + s] = X[r * (NB + 1) + s];
    }
    // zero the upper blocks of this block row
    for (int64_t e = t; e < (int64_t)NB * (npad - Ib - NB); e += blockDim.x) {
      const int64_t r = e / (npad - Ib - NB), s = e % (npad - Ib - NB);
      Li[(Ib + r) * npad + Ib + NB + s] = 0.0;
    }
    return;
  }
  double acc[16];
#pragma unroll
  for (int q = 0; q < 16; ++q) acc[q] = 0.0;
  for (int32_t Kb = J; Kb < I; ++Kb) {
    __syncthreads();
    for (int e = t; e < NB * NB; e += blockDim.x) {
      const int r = e / NB, s = e % NB;
      S[r * (NB + 1) + s] = L[(Ib + r) * npad + (int64_t)Kb * NB + s];
      T[r * (NB + 1) + s] = Li[((int64_t)Kb * NB + r) * npad + Jb + s];
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int e = t + q * 256;
      const int r = e / NB, s = e % NB;
      double v = 0.0;
      for (int w = 0; w < NB; ++w) v += S[r * (NB + 1) + w] * T[w * (NB + 1) + s];
      acc[q] += v;
    }
  }
  __syncthreads();
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    const int e = t + q * 256;
    T[(e / NB) * (NB + 1) + e % NB] = acc[q];
  }
  __syncthreads();
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    const int e = t + q * 256;
    const int r = e / NB, s = e % NB;
    double v = 0.0;
    for (int w = 0; w <= r; ++w) v += X[r * (NB + 1) + w] * T[w * (NB + 1) + s];
    Li[(Ib + r) * npad + Jb + s] = -v;
  }
}

// out = Linv * v  (one wave per row)
__global__ __launch_bounds__(256) void k_lower_mv(const double* __restrict__ Li, int32_t npad,
                                                  const double* __restrict__ v, double* __restrict__ out) {
  const int32_t r = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (r >= npad) return;
  double s = 0.0;
  for (int32_t c = lane; c <= r; c += 64) s += Li[(int64_t)r * npad + c] * v[c];
  for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off);
  if (lane == 0) out[r] = s;
}

// out = Linv^T * v  (one thread per column)
__global__ void k_lower_tmv(const double* __restrict__ Li, int32_t npad, const double* __restrict__ v,
                            double* __restrict__ out) {
  const int32_t c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= npad) return;
  double s = 0.0;
  for (int32_t r = c; r < npad; ++r) s += Li[(int64_t)r * npad + c] * v[r];
  out[c] = s;
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
                              const double* __restrict__ stats, int32_t kind, double xi, double kappa,
                              const uint8_t* __restrict__ dup, double* __restrict__ mu_out,
                              double* __restrict__ var_out, double* __restrict__ score_out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= m) return;
  double mu = 0.0, vs = 0.0;
  for (int32_t r = 0; r < RT1; ++r) mu += mu_part[(int64_t)r * ldp + i];
  for (int32_t r = 0; r < RT2; ++r) vs += var_part[(int64_t)r * ldp + i];
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
static int gp_alloc(ut_ctx* c, int32_t npad, int32_t d) {
  if (c->gp_cap_n >= npad && c->gp_d == d && c->gp_Xs) return 0;
  if (c->gp_Xs_f) {
    UT_HIP(c, hipStreamSynchronize(c->stream));
    hipFree(c->gp_Xs_f); hipFree(c->gp_Linv_f);
    c->gp_Xs_f = nullptr; c->gp_Linv_f = nullptr;
  }
  if (c->gp_Xs) {
    UT_HIP(c, hipStreamSynchronize(c->stream));
    hipFree(c->gp_Xs); hipFree(c->gp_xnorm); hipFree(c->gp_K); hipFree(c->gp_Linv);
    hipFree(c->gp_y); hipFree(c->gp_tmp); hipFree(c->gp_alpha); hipFree(c->gp_inv_ell);
    hipFree(c->gp_stats); hipFree(c->gp_flag);
  }
  UT_HIP(c, hipMalloc((void**)&c->gp_Xs, sizeof(double) * npad * d));
  UT_HIP(c, hipMalloc((void**)&c->gp_xnorm, sizeof(double) * npad));
  UT_HIP(c, hipMalloc((void**)&c->gp_K, sizeof(double) * npad * npad));
  UT_HIP(c, hipMalloc((void**)&c->gp_Linv, sizeof(double) * npad * npad));
  UT_HIP(c, hipMalloc((void**)&c->gp_y, sizeof(double) * npad));
  UT_HIP(c, hipMalloc((void**)&c->gp_tmp, sizeof(double) * npad * (d + 1)));
  UT_HIP(c, hipMalloc((void**)&c->gp_alpha, sizeof(double) * npad));
  UT_HIP(c, hipMalloc((void**)&c->gp_inv_ell, sizeof(double) * d));
  UT_HIP(c, hipMalloc((void**)&c->gp_stats, sizeof(double) * 4));
  UT_HIP(c, hipMalloc((void**)&c->gp_flag, sizeof(int32_t)));
  UT_HIP(c, hipMalloc((void**)&c->gp_Xs_f, sizeof(float) * npad * d));
  UT_HIP(c, hipMalloc((void**)&c->gp_Linv_f, sizeof(float) * npad * npad));
  c->gp_cap_n = npad;
  c->gp_d = d;
  return 0;
}

int gp_fit_impl(ut_ctx* c, const double* X, const double* y, int32_t n, int32_t d, const ut_gp_hyper* h) {
  UT_CHECK(c, n >= 1 && d >= 1 && X && y && h && h->lengthscale_host, UT_EINVAL, "gp_fit: bad arguments");
  const int32_t npad = ((n + NPAD - 1) / NPAD) * NPAD;
  int rc = gp_alloc(c, npad, d);
  if (rc) return rc;
  c->gp_n = n;
  c->gp_sf2 = h->sigma_f2;
  std::vector<double> inv(d);
  for (int32_t k = 0; k < d; ++k) inv[k] = 1.0 / h->lengthscale_host[k];
  double* dX = c->gp_tmp;           // [n][d] staging (gp_tmp holds npad*(d+1))
  double* dy = c->gp_tmp + (int64_t)npad * d;
  UT_HIP(c, hipMemcpyAsync(c->gp_inv_ell, inv.data(), sizeof(double) * d, hipMemcpyHostToDevice, c->stream));
  UT_HIP(c, hipMemcpyAsync(dX, X, sizeof(double) * n * d, hipMemcpyHostToDevice, c->stream));
  UT_HIP(c, hipMemcpyAsync(dy, y, sizeof(double) * n, hipMemcpyHostToDevice, c->stream));
  UT_HIP(c, hipMemsetAsync(c->gp_flag, 0, sizeof(int32_t), c->stream));
  hipLaunchKernelGGL(k_gp_prep_train, dim3(grid1(npad, 256)), dim3(256), 0, c->stream, dX, n, npad, d,
                     c->gp_inv_ell, c->gp_Xs, c->gp_xnorm);
  hipLaunchKernelGGL(k_gp_kmat, dim3(grid1((int64_t)npad * npad, 256)), dim3(256), 0, c->stream, c->gp_Xs,
                     c->gp_xnorm, n, npad, d, h->sigma_f2, h->sigma_n2 + h->jitter, c->gp_K);
  hipLaunchKernelGGL(k_gp_ystats, dim3(1), dim3(256), 0, c->stream, dy, n, npad, c->gp_y, c->gp_stats);
  UT_LAUNCH_CHECK(c);
  const int32_t nb = npad / NB;
  for (int32_t kb = 0; kb < nb; ++kb) {
    hipLaunchKernelGGL(k_chol_panel, dim3(nb - kb), dim3(256), 0, c->stream, c->gp_K, npad, kb, c->gp_flag);
    const int32_t T = nb - kb - 1;
    if (T > 0)
      hipLaunchKernelGGL(k_chol_update, dim3(T * (T + 1) / 2), dim3(256), 0, c->stream, c->gp_K, npad, kb);
  }
  UT_LAUNCH_CHECK(c);
  for (int32_t I = 0; I < nb; ++I)
    hipLaunchKernelGGL(k_trinv_row, dim3(I + 1), dim3(256), 0, c->stream, c->gp_K, c->gp_Linv, npad, I);
  UT_LAUNCH_CHECK(c);
  hipLaunchKernelGGL(k_lower_mv, dim3(grid1(npad, 4)), dim3(256), 0, c->stream, c->gp_Linv, npad, c->gp_y,
                     c->gp_tmp);
  hipLaunchKernelGGL(k_lower_tmv, dim3(grid1(npad, 256)), dim3(256), 0, c->stream, c->gp_Linv, npad, c->gp_tmp,
                     c->gp_alpha);
  UT_LAUNCH_CHECK(c);
  if (c->gp_prec == 32) {
    if ((rc = launch_to_f32(c, c->gp_Xs, c->gp_Xs_f, (int64_t)npad * d))) return rc;
    if ((rc = launch_to_f32(c, c->gp_Linv, c->gp_Linv_f, (int64_t)npad * npad))) return rc;
  }
  c->gp_fit_prec = c->gp_prec;
  int32_t flag = 0;
  UT_HIP(c, hipMemcpyAsync(&flag, c->gp_flag, sizeof(int32_t), hipMemcpyDeviceToHost, c->stream));
  UT_HIP(c, hipStreamSynchronize(c->stream));
  c->gp_ready = (flag == 0);
  UT_CHECK(c, flag == 0, UT_ENOTPD, "gp_fit: kernel matrix is not positive definite (raise jitter)");
  return 0;
}

int gp_score_impl(ut_ctx* c, const double* feat, int64_t ld, int64_t m, const ut_acq* acq, const uint8_t* dup,
                  double* mu, double* var, double* score) {
  UT_CHECK(c, c->gp_ready, UT_EINVAL, "gp_score: call ut_gp_fit first");
  UT_CHECK(c, acq != nullptr, UT_EINVAL, "gp_score: acq is NULL");
  if (m <= 0) return 0;
  const int32_t n = c->gp_n, d = c->gp_d;
  const int32_t npad = ((n + NPAD - 1) / NPAD) * NPAD;
  const int32_t RT = npad / NPAD;
  const int32_t CT = (int32_t)((m + NPAD - 1) / NPAD);
  const int64_t ldk = (int64_t)CT * NPAD;
  const bool fp32 = c->gp_fit_prec == 32;
  int rc;
  if ((rc = ensure(c, c->kst, (size_t)npad * ldk))) return rc;
  if ((rc = ensure(c, c->mu_part, (size_t)RT * ldk))) return rc;
  if ((rc = ensure(c, c->var_part, (size_t)RT * ldk))) return rc;
  if ((rc = ensure(c, c->cnorm, (size_t)ldk))) return rc;
  hipLaunchKernelGGL(k_gp_cnorm, dim3(grid1(m, 256)), dim3(256), 0, c->stream, feat, ld, m, d, c->gp_inv_ell,
                     c->cnorm.p);
  mark(c, "cnorm");
  if ((rc = launch_gemm_kstar(c, fp32, (const void*)c->gp_Xs, d, feat, ld, d, RT,
                              CT, m, c->kst.p, ldk, c->mu_part.p)))
    return rc;
  mark(c, "kstar");
  if ((rc = launch_gemm_var(c, fp32, fp32 ? (const void*)c->gp_Linv_f : (const void*)c->gp_Linv, npad, c->kst.p,
                            ldk, npad, RT, CT, m, c->var_part.p)))
    return rc;
  mark(c, "var");
  hipLaunchKernelGGL(k_gp_finalize, dim3(grid1(m, 256)), dim3(256), 0, c->stream, m, RT, RT, c->mu_part.p,
                     c->var_part.p, ldk, c->gp_sf2, c->gp_stats, acq->kind, acq->xi, acq->kappa, dup, mu, var,
                     score);
  UT_LAUNCH_CHECK(c);
  mark(c, "finalize");
  return 0;
}

}  // namespace ut
