// gp_i8.hip -- the fp64-tier variance contraction on the int8 MFMA
// (ut_gp_set_precision(ctx, 8); "Ozaki" slicing with exact int32 accumulation).
//
// The variance needs |v|^2 with v = L^-1 k* for every candidate, an n x n by
// n x m contraction (gp_gemm.hip k_gp_var_pp on the fp64 MFMA).  Here both
// operands are cut into S = 6 signed 8-bit digit planes and the contraction
// runs on v_mfma_i32_32x32x32_i8 (64x the fp64 MFMA's rate per CU):
//
//   row i of L^-1:  x_ik = L^-1_ik 2^-ea_i  (power of two: |x| <= 0.49)
//   column c of K*: y_kc = k*_kc 2^-eb      (eb from sf2 >= k*: |y| <= 0.49)
//   X = rint(x 2^48) = sum_{p=1..6} a_p 256^(6-p), a_p in [-128, 127] ("balanced"
//   digits: the bytes of X + 0x808080808080, each XOR 0x80, taken from the bits
//   of the fp64 sum x + 24.50196..., whose ulp is 2^-48 -- i8_biased), Y likewise.
//   x y ~ sum_{p+q <= 7} a_p b_q 2^-8(p+q):  21 of the 36 digit products, in
//   six groups g = p + q whose int32 sums T_g = sum_k sum_{p+q=g} a_p b_q are
//   exact (|a b| <= 2^14, at most 6 pairs per group: K < 2^14 rows keep every
//   T_g below 2^31), and
//   v_ic = 2^(ea_i + eb) 2^-16 (T_2 + 2^-8 (T_3 + ... + 2^-8 T_7))   in fp64.
//
// Error (per element, in units of 2^(ea_i + eb)): the digit rounding of x and y
// (|dx|, |dy| <= 2^-49, times |y|, |x| <= 0.4901) and the dropped pairs
// p + q >= 8 (<= 2^14 (5 2^-64 + 4 2^-72 + ...) < 5.02 2^-50) stay below
// C = 3.5 2^-49, so |v_ic - v^_ic| <= e_i = (i + 1) C 2^(ea_i + eb) for every
// candidate, and |v - v^| <= E = |e|_2 (k_i8_errsum).  With s = |v^|^2 the
// exact |v|^2 lies within E (2 |v^| + E) of s, plus the fp64 rounding of the
// recombination and the sums (< s (2n + 64) 2^-53).  k_gp_finalize_i8 (gp.hip)
// accepts a candidate when that bound is <= tau * (sf2 - s) (tau: ut_gp_set_i8_tol,
// default 2^-20), i.e. its variance is within tau relative of the exact one;
// every other candidate -- next to a training point, where sf2 - |v|^2 is a
// cancellation -- is recomputed in fp64 (gp.hip gp_score_impl).  The mean is
// k* . alpha from K*'s fp64 epilogue, as in the fp32 tier.
//
// Layouts (bytes): A = [6][npad/32][npad][32] (L^-1 rows), B = [6][npad/32][ldk][32]
// (written by k_gp_kstar<int8_t>); row / candidate r's 16-byte chunk c of a
// 32-k piece sits at position c ^ ((r >> 3) & 1), so the 32x32x32 MFMA's
// fragment reads (32 rows x 2 chunks per ds_read_b128) hit distinct banks.
#include "ut_internal.h"

namespace ut {

constexpr int I8_PL = I8_BM * I8_BK;   // one plane's piece of a stage: 64 rows x 32 k = 2 KiB
constexpr double I8_C = 3.5 * 0x1p-49;

template <int N>
__device__ __forceinline__ void i8_vm_wait() {
  static_assert(N >= 0 && N < 64, "vmcnt");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
}

// ---------------------------------------------------------------------------
// fit side: L^-1 -> digit planes, row scales 2^(ea_i + eb), e_i^2
// one 256-thread workgroup per padded row; thread t digitises k = 4t .. 4t + 3
// (+ 1024 j), one dword per plane
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_split_i8(const double* __restrict__ Linv, int32_t n, int32_t npad,
                                                  int32_t eb, int8_t* __restrict__ A, double* __restrict__ rs,
                                                  double* __restrict__ e2) {
  __shared__ double red[4];
  const int32_t r = blockIdx.x;
  const int t = threadIdx.x;
  const int32_t kend = r < n ? r + 1 : 0;   // L^-1 row r is zero past the diagonal
  const double* row = Linv + (int64_t)r * npad;
  double mx = 0.0;
  for (int32_t k = t; k < kend; k += 256) mx = fmax(mx, fabs(row[k]));
  for (int o = 32; o > 0; o >>= 1) mx = fmax(mx, __shfl_xor(mx, o));
  if ((t & 63) == 0) red[t >> 6] = mx;
  __syncthreads();
  mx = fmax(fmax(red[0], red[1]), fmax(red[2], red[3]));
  // 2^ea >= mx / 0.49: |x| <= 0.49 (to the rounding of the quotient)
  const int32_t ea = mx > 0.0 ? ilogb(mx / 0.49) + 1 : 0;
  const int64_t plane = (int64_t)npad * npad;
  for (int32_t k0 = 4 * t; k0 < npad; k0 += 1024) {
    uint32_t lo[4], hi[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const double v = k0 + u < kend ? row[k0 + u] : 0.0;
      const uint64_t b = i8_biased(__builtin_ldexp(v, -ea));
      lo[u] = (uint32_t)b;
      hi[u] = (uint32_t)(b >> 32);
    }
    uint32_t pl[I8_S];
    i8_planes(lo, hi, pl);
    const int64_t o = i8_off(r, k0, npad);
#pragma unroll
    for (int p = 0; p < I8_S; ++p) *reinterpret_cast<uint32_t*>(A + p * plane + o) = pl[p];
  }
  if (t == 0) {
    const bool live = kend > 0 && mx > 0.0;
    const double sc = live ? __builtin_ldexp(1.0, ea + eb) : 0.0;
    rs[r] = sc;
    const double e = (double)kend * I8_C * sc;
    e2[r] = e * e;
  }
}

// E = sqrt(sum_r e2[r]) and Emu = sum_r e_r |beta_r| (beta = L^-1 y; one
// workgroup, fixed order), both rounded up.  The mean comes from the variance
// epilogue, mu^ = v^ . beta, so |mu - mu^| <= sum_r |v_r - v^_r| |beta_r| <= Emu.
__global__ __launch_bounds__(256) void k_i8_errsum(const double* __restrict__ e2, const double* __restrict__ beta,
                                                   int32_t npad, double* __restrict__ E) {
  __shared__ double red[2][4];
  const int t = threadIdx.x;
  double s = 0.0, sm = 0.0;
  for (int32_t r = t; r < npad; r += 256) {
    s += e2[r];
    sm = __builtin_fma(sqrt(e2[r]), fabs(beta[r]), sm);
  }
  for (int o = 32; o > 0; o >>= 1) {
    s += __shfl_xor(s, o);
    sm += __shfl_xor(sm, o);
  }
  if ((t & 63) == 0) {
    red[0][t >> 6] = s;
    red[1][t >> 6] = sm;
  }
  __syncthreads();
  if (t == 0) {
    E[0] = sqrt((red[0][0] + red[0][1]) + (red[0][2] + red[0][3])) * (1.0 + 0x1p-40);
    E[1] = ((red[1][0] + red[1][1]) + (red[1][2] + red[1][3])) * (1.0 + 0x1p-40);
  }
}

int alloc_split_i8(ut_ctx* c, int32_t npad) {
  int rc;
  if ((rc = ensure(c, c->gp_i8a, (size_t)I8_S * npad * npad))) return rc;
  return ensure(c, c->gp_i8rs, (size_t)2 * npad + 2);   // [rs | e2 | E | Emu]
}

int launch_split_i8(ut_ctx* c, int32_t n, int32_t npad) {
  UT_CHECK(c, c->gp_i8a.n >= (size_t)I8_S * npad * npad && c->gp_i8rs.n >= (size_t)2 * npad + 2, UT_EINVAL,
           "split_i8: planes not allocated (alloc_split_i8)");
  double* rs = c->gp_i8rs.p;
  hipLaunchKernelGGL(k_split_i8, dim3(npad), dim3(256), 0, c->stream, c->gp_Linv, n, npad, c->gp_i8_eb,
                     c->gp_i8a.p, rs, rs + npad);
  hipLaunchKernelGGL(k_i8_errsum, dim3(1), dim3(256), 0, c->stream, rs + npad, c->gp_beta, npad, rs + 2 * npad);
  UT_LAUNCH_CHECK(c);
  return 0;
}

// ---------------------------------------------------------------------------
// the contraction: part[rt][col] = sum_{rows of tile rt} v^_{row,col}^2
//
// Persistent, TWO 256-thread workgroups per CU (one's barrier waits and
// epilogue overlap the other's MFMAs, as k_gp_var_pp); a work item is the
// row-tile pair (RT - 1 - p, p) of one 128-candidate strip (every item the
// same length), handed out per XCD in groups of P pairs x Sg strips so the
// group shares each L^-1 stage through L2.  The pair's second (short) tile
// walks its k stages in descending order: at every step the strip's P
// workgroups then read at most two distinct K* stages, the rest L2 hits.
// Tile 64 rows x 128 candidates; waves 2 x 2 of 32 rows x 64 candidates (two
// 32 x 32 MFMA column tiles share the wave's A fragments; B planes streamed
// one at a time); a 2-stage ring of 32-k stages (6 A planes x 2 KiB + 6 B
// planes x 4 KiB = 36 KiB), filled by global_load_lds (9 per wave per stage).
// The wave's rows [32 wm, +32) see zeros once k passes them (L^-1 is lower
// triangular): those stages skip their MFMAs.  Probe on random digits
// (scripts/exp/i8var_probe.hip, n = 1024, m = 2^20): 9.26 ms against 10.0 for
// 64-candidate tiles with a 3-stage ring.
// ---------------------------------------------------------------------------
constexpr int I8_WN = 128;                 // candidates per tile
constexpr int I8_BPL = I8_WN * I8_BK;      // one B plane's piece of a stage (4 KiB)

__global__ __launch_bounds__(256, 2) void k_gp_var_i8(const int8_t* __restrict__ Ad, const int8_t* __restrict__ Bd,
                                                      int32_t npad, int64_t ldk, int32_t RT, int32_t CT, int64_t m,
                                                      int32_t* __restrict__ ticket, const double* __restrict__ rs,
                                                      const double* __restrict__ beta, double* __restrict__ part,
                                                      double* __restrict__ mpart, int32_t Sg) {
  constexpr int STAGE = I8_S * (I8_PL + I8_BPL);
  constexpr int NW = 6 * I8_S / 4;   // glds per wave per stage
  __shared__ __attribute__((aligned(16))) int8_t lds[2 * STAGE + 4 * I8_WN * 8 + 2 * I8_BM * 8 + 16];
  double* red = reinterpret_cast<double*>(lds + 2 * STAGE);   // [2][128] sums of v^2, [2][128] of v beta
  double* srs = red + 4 * I8_WN;                               // row scales of the tile
  double* sbt = srs + I8_BM;                                   // beta of the tile's rows
  int32_t& s_item = *reinterpret_cast<int32_t*>(sbt + I8_BM);
  const int t = threadIdx.x, lane = t & 63;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const int wm = w >> 1, wn = w & 1;
  const int32_t xcd = __builtin_amdgcn_readfirstlane(blockIdx.x & 7);
  const int64_t aplane = (int64_t)npad * npad, bplane = (int64_t)npad * ldk;

  // stage kt of tile (row0, col0): A planes 2 KiB (2 pieces), B planes 4 KiB (4 pieces);
  // wave w moves pieces w + 4j
  auto issue = [&](int32_t row0, int64_t col0, int32_t kt, int8_t* st) {
#pragma unroll
    for (int j = 0; j < NW; ++j) {
      const int u = w + 4 * j;
      const int8_t* src;
      int8_t* dst;
      if (u < 2 * I8_S) {
        const int pl = u >> 1, h = u & 1;
        src = Ad + pl * aplane + ((int64_t)kt * npad + row0) * 32 + h * 1024;
        dst = st + pl * I8_PL + h * 1024;
      } else {
        const int v = u - 2 * I8_S, pl = v >> 2, h = v & 3;
        src = Bd + pl * bplane + ((int64_t)kt * ldk + col0) * 32 + h * 1024;
        dst = st + I8_S * I8_PL + pl * I8_BPL + h * 1024;
      }
      __builtin_amdgcn_global_load_lds(src + lane * 16, (__attribute__((address_space(3))) void*)dst, 16, 0, 0);
    }
  };

  const int32_t P = (RT + 1) / 2;
  const int c = lane >> 5;
  const int ra = wm * 32 + (lane & 31);
  const int aoff = ra * 32 + ((c ^ ((ra >> 3) & 1)) << 4);
  int boff[2];
#pragma unroll
  for (int jj = 0; jj < 2; ++jj) {
    const int cb = wn * 64 + jj * 32 + (lane & 31);
    boff[jj] = I8_S * I8_PL + cb * 32 + ((c ^ ((cb >> 3) & 1)) << 4);
  }
  for (;;) {
    if (t == 0) s_item = atomicAdd(&ticket[xcd], 1);
    __syncthreads();
    // (every item quantity scalar: the glds bases and loop bounds in SGPRs)
    const int32_t j = __builtin_amdgcn_readfirstlane(s_item);
    const int32_t G = j / (P * Sg), q = j % (P * Sg), p = q % P;
    const int32_t ct = (G * Sg + q / P) * 8 + xcd;
    if (ct >= CT) break;   // uniform: the whole workgroup leaves
    const int nrt = RT - 1 - p == p ? 1 : 2;
    for (int ri = 0; ri < nrt; ++ri) {
      if (ri > 0) __syncthreads();   // the previous tile's ring, red and srs are read
      const int32_t rt = __builtin_amdgcn_readfirstlane(ri == 0 ? RT - 1 - p : p);
      const int32_t row0 = rt * I8_BM;
      const int64_t col0 = (int64_t)ct * I8_WN;
      const int32_t nk = (row0 + I8_BM) / I8_BK;   // >= 2
      const bool rev = ri > 0;
      auto ktof = [&](int32_t u) -> int32_t { return rev ? nk - 1 - u : u; };
      i8v16 acc[2][I8_S];
#pragma unroll
      for (int jj = 0; jj < 2; ++jj)
#pragma unroll
        for (int g = 0; g < I8_S; ++g)
#pragma unroll
          for (int r = 0; r < 16; ++r) acc[jj][g][r] = 0;
      if (w < 2 && lane < 32)   // 64 row scales / betas: one 512-B glds each, retired with stage 0
        __builtin_amdgcn_global_load_lds((w == 0 ? rs : beta) + row0 + lane * 2,
                                         (__attribute__((address_space(3))) void*)(w == 0 ? srs : sbt), 16, 0, 0);
      issue(row0, col0, ktof(0), lds);
      for (int32_t u = 0; u < nk; ++u) {
        i8_vm_wait<0>();                        // stage u landed (this wave's pieces)
        __builtin_amdgcn_s_barrier();           // every wave's stage u landed; stage u - 1 fully read
        asm volatile("" ::: "memory");
        if (u + 1 < nk) issue(row0, col0, ktof(u + 1), lds + ((u + 1) & 1) * STAGE);
        const int32_t kt = ktof(u);
        if (kt * I8_BK >= row0 + 32 * wm + 32) continue;   // rows of this wave: all zero here
        const int8_t* st = lds + (u & 1) * STAGE;
        i8v4 af[I8_S];
#pragma unroll
        for (int pp = 0; pp < I8_S; ++pp) af[pp] = *reinterpret_cast<const i8v4*>(st + pp * I8_PL + aoff);
#pragma unroll
        for (int qb = 0; qb < I8_S; ++qb) {
          i8v4 bf[2];
#pragma unroll
          for (int jj = 0; jj < 2; ++jj) bf[jj] = *reinterpret_cast<const i8v4*>(st + qb * I8_BPL + boff[jj]);
          // digit products of group g = pa + qb (0-based): pairs with (pa + 1) + (qb + 1) <= 7
#pragma unroll
          for (int pa = 0; pa + qb < I8_S; ++pa)
#pragma unroll
            for (int jj = 0; jj < 2; ++jj)
              acc[jj][pa + qb] = __builtin_amdgcn_mfma_i32_32x32x32_i8(af[pa], bf[jj], acc[jj][pa + qb], 0, 0, 0);
        }
      }
      // epilogue: v = 2^-16 (T_2 + 2^-8 (T_3 + ...)) * 2^(ea_row + eb), column sums
      // of v^2 and of v beta (the mean, mu = (L^-1 k*) . (L^-1 y))
      // (C/D map of the 32x32 MFMA: row (r & 3) + 8 (r >> 2) + 4 (lane >> 5), column lane & 31)
#pragma unroll
      for (int jj = 0; jj < 2; ++jj) {
        double s = 0.0, sm = 0.0;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          double v = (double)acc[jj][I8_S - 1][r];
#pragma unroll
          for (int g = I8_S - 2; g >= 0; --g) v = __builtin_fma(v, 0x1p-8, (double)acc[jj][g][r]);
          const int rr = wm * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
          v *= 0x1p-16 * srs[rr];
          s = __builtin_fma(v, v, s);
          sm = __builtin_fma(v, sbt[rr], sm);
        }
        s += __shfl_xor(s, 32);
        sm += __shfl_xor(sm, 32);
        if (lane < 32) {
          red[wm * I8_WN + wn * 64 + jj * 32 + lane] = s;
          red[2 * I8_WN + wm * I8_WN + wn * 64 + jj * 32 + lane] = sm;
        }
      }
      __syncthreads();
      if (t < I8_WN) {
        const int64_t col = col0 + t;
        if (col < m) {
          part[(int64_t)rt * ldk + col] = red[t] + red[I8_WN + t];
          mpart[(int64_t)rt * ldk + col] = red[2 * I8_WN + t] + red[3 * I8_WN + t];
        }
      }
    }
  }
}

int launch_gemm_var_i8(ut_ctx* c, int32_t npad, const int8_t* kst8, int64_t ldk, int64_t m, double* part,
                       double* mpart) {
  UT_CHECK(c, npad % 128 == 0 && npad <= I8_MAX_K && ldk % I8_WN == 0 && ldk >= m, UT_EINVAL,
           "gemm_var_i8: bad padding");
  UT_CHECK(c, c->gp_i8a.p && c->gp_i8rs.p, UT_EINVAL, "gemm_var_i8: the fit has no int8 planes");
  const int32_t RT = npad / I8_BM, CT = (int32_t)((m + I8_WN - 1) / I8_WN);
  const int32_t P = (RT + 1) / 2;
  const int64_t items = (int64_t)P * CT;
  int32_t nb = 2 * (c->n_cu / 8) * 8;   // two workgroups per CU, a multiple of 8 (every XCD group works)
  if (items < nb) nb = (int32_t)(((items + 7) / 8) * 8);
  const int32_t W = nb / 8, Sg = W / P > 1 ? W / P : 1;
  UT_HIP(c, hipMemsetAsync(c->gp_ctr, 0, sizeof(int32_t) * 8, c->stream));
  hipLaunchKernelGGL(k_gp_var_i8, dim3(nb), dim3(256), 0, c->stream, c->gp_i8a.p, kst8, npad, ldk, RT, CT, m,
                     c->gp_ctr, c->gp_i8rs.p, c->gp_beta, part, mpart, Sg);
  UT_LAUNCH_CHECK(c);
  return 0;
}

}  // namespace ut
