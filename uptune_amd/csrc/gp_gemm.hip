// gp_gemm.hip -- the two dense contractions of GP scoring (the MFMA-bound
// stage of the path), both persistent (one or two workgroups per CU pulling
// work items from per-XCD tickets) and staged by global_load_lds:
//
//   k_gp_kstar:  C = (X/ell) (U/ell)^T, epilogue k* = sf2 exp(-0.5 max(|x|^2+|u|^2-2C, 0)),
//                stores K*^T [n][ldk] and the column partial  sum_r alpha_r k*_r   (mean)
//   k_gp_var:    V = L^-1 K*^T (L^-1 lower triangular: row tile rt stops its K
//                loop at (rt+1)*128), epilogue column partial  sum_r V[r][c]^2   (variance)
//
//   fp64: v_mfma_f64_16x16x4_f64   (C/D: col = lane&15, row = (lane>>4) + 4r)
//   fp32: v_mfma_f32_32x32x2_f32   (C/D: col = lane&31, row = (r&3) + 8(r>>2) + 4(lane>>5))
#include <type_traits>

#include "ut_internal.h"

namespace ut {

// the fit kernels here (see gp.hip g_fit_prio): s_setprio 3 when set
__device__ int32_t g_fit_prio_g = 0;
__device__ __forceinline__ void fit_prio_g() {
  if (g_fit_prio_g) __builtin_amdgcn_s_setprio(3);
}

int set_fit_prio_gemm(int32_t on) {
  return hipMemcpyToSymbol(HIP_SYMBOL(g_fit_prio_g), &on, sizeof(on)) == hipSuccess ? 0 : UT_EHIP;
}

__global__ void k_to_f32(const double* __restrict__ src, float* __restrict__ dst, int64_t n) {
  fit_prio_g();
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) dst[i] = (float)src[i];
}

// ---------------------------------------------------------------------------
// K* contraction, persistent:  C = Xs U'  (Xs = X/ell [n][d], U' = U/ell [d][m])
//   k*[r][c] = sf2 exp(-0.5 max(|xs_r|^2 + |u'_c|^2 - 2 C[r][c], 0))  (0 outside n x m)
//   stored as K*^T [r][ldk] (TS), plus the column partial sum_r alpha_r k*[r][c]
// 256-thread workgroups (2 x 2 waves of 64 x 64) on 128 x 128 tiles, K = dpad
// in steps of 16, a 2-stage glds ring (64 KiB) so TWO workgroups share a CU
// and one's exp/store epilogue overlaps the other's MFMAs.  Work items are
// handed out per XCD group like k_gp_var's.
//   A = Xs^T [dpad][npad] (rows >= d zero), B = U' [dpad][ldk] (rows >= d and
//   columns >= m zero; written by k_gp_prep_cand)
// ---------------------------------------------------------------------------
constexpr int K_NT = 256, K_BM = 128, K_BN = 128, K_BK = 16;
constexpr int KSTAR_SPARE_PER_XCD = 2;

// f16x3 operand layout (k_gp_var_h3): 256-row x 32-k blocks of 16 KiB per
// plane, pre-swizzled into the variance kernel's LDS image
constexpr int H3_BM = 256, H3_BN = 256, H3_BK = 32;
constexpr int H3_BLK = H3_BM * H3_BK;          // fp16 elements per block (16 KiB)
constexpr int H3_STAGE = 4 * H3_BLK;           // A hi, A lo, B hi, B lo
constexpr int H3_NS = 2;                       // ring slots (128 KiB)
typedef _Float16 vh8 __attribute__((ext_vector_type(8)));

// element offset of (r, k) inside a blocked plane with K columns
__device__ __forceinline__ int64_t h3_blk_off(int64_t r, int32_t k, int32_t K) {
  const int rr = (int)(r & (H3_BM - 1)), c = (k & (H3_BK - 1)) >> 3;
  return ((r >> 8) * (K / H3_BK) + (k >> 5)) * H3_BLK + rr * H3_BK + ((c ^ ((rr >> 2) & 3)) << 3) + (k & 7);
}
  // CUs left to an in-flight GP fit (launch_gemm_kstar)

// (sf2_exp2t_nonpos, EXP_TAB, KSTAR_T_MIN: ut_internal.h)

constexpr int K_SA = K_BK * K_BM, K_SB = K_BK * K_BN, K_STAGE = K_SA + K_SB;

__device__ __forceinline__ void kstar_issue(const double* __restrict__ AT, int64_t lda, const double* __restrict__ B,
                                            int64_t ldb, int32_t row0, int64_t col0, int32_t k0, double* st, int w,
                                            int lane, int32_t dpad) {
  // 16 KiB of A and 16 KiB of B per stage = 32 wave-instructions, 8 per wave;
  // wave w loads k rows 4w .. 4w+3, none past dpad (a multiple of 4: the last
  // stage of a dpad that is not a multiple of 16 is partial)
  if (k0 + 4 * w >= dpad) return;
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int q = 4 * w + u;  // 0..15: A tile row k = q (128 doubles = 1 KiB)
    const double* src = AT + (int64_t)(k0 + q) * lda + row0 + lane * 2;
    __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)(st + q * 128), 16, 0, 0);
  }
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int q = 4 * w + u;
    const double* src = B + (int64_t)(k0 + q) * ldb + col0 + lane * 2;
    __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)(st + K_SA + q * 128), 16, 0, 0);
  }
}

typedef double kd4 __attribute__((ext_vector_type(4)));
typedef int32_t ki4 __attribute__((ext_vector_type(4)));

// Categorical K* (CAT): ENUM and BOOL params are one-hot blocks of the GP
// features (SURVEY.md §8 GP spec: Enum one-hot, Bool {0, 1}), and with one
// lengthscale ell over those blocks a block contributes to |x - u|^2 exactly
//   2 / ell^2 (ENUM) or 1 / ell^2 (BOOL)  when the two configurations' options
//   differ, and 0 when they match.
// So -|x - u|^2 / 2 over the categorical features is c0 + c1 * M with
//   M = sum_j w_j [opt_x(j) == opt_u(j)],  w_j = 2 (ENUM), 1 (BOOL),
//   c1 = 1 / (2 ell^2),  c0 = -c1 * sum_j w_j,
// and M is the integer dot product of the training rows' weighted one-hot
// codes with the candidates' 0/1 codes (ENUM: n_opt columns, BOOL: 2).  That
// product runs on v_mfma_i32_16x16x64_i8 (exact int32, 4x the fp64 MFMA's
// rate per instruction at 16x the K), ahead of the fp64 contraction over the
// remaining ("numeric") features, and c0 + c1 M starts the fp64 accumulator.
// At C3 (HPL-64: 79 of 119 features one-hot / 0-1) the fp64 contraction's K
// drops 120 -> 40, at C4 (gcc: 552 of 707) 708 -> 156.
//   int8 stage: 128 code columns x 128 rows (A) / candidates (B) = 16 KiB per
//   operand, the fp64 stage's footprint; global layout [k / 128][row][128 B],
//   LDS row r's 16-B chunk c at position c ^ (r & 7) (swizzled through the
//   glds source address: the fragment reads are at most 2-way conflicted).
//   The i8 MFMA's C/D rows are 4 (l >> 4) + q where the fp64 MFMA's are
//   (l >> 4) + 4 q, so the A fragment of MFMA row rho loads tile row
//   sigma(rho) = (rho >> 2) + 4 (rho & 3): iacc[i][jj][q] then sits where
//   acc[i][jj][q] does (scripts/exp/i8_mfma_probe.hip checks both maps).
__device__ __forceinline__ void kcat_issue(const int8_t* __restrict__ Ab, const int8_t* __restrict__ Bb,
                                           double* st, int w, int lane) {
  uint8_t* sb = reinterpret_cast<uint8_t*>(st);
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int q = 4 * w + u;                      // rows 8q .. 8q + 7 of the tile (1 KiB)
    const int r = 8 * q + (lane >> 3);
    const int cch = (lane & 7) ^ (r & 7);         // the global chunk that lands at position lane & 7
    __builtin_amdgcn_global_load_lds(Ab + r * 128 + cch * 16, (__attribute__((address_space(3))) void*)(sb + q * 1024),
                                     16, 0, 0);
    __builtin_amdgcn_global_load_lds(Bb + r * 128 + cch * 16,
                                     (__attribute__((address_space(3))) void*)(sb + K_SA * 8 + q * 1024), 16, 0, 0);
  }
}

// MU: also the column partial of the mean, sum_r alpha_r k*_r (fp32 scoring;
// fp64 takes the mean from the variance epilogue instead)
template <typename TS, bool MU, bool CAT>
__global__ __launch_bounds__(K_NT, 2) void k_gp_kstar(const double* __restrict__ AT, int64_t lda,
                                                      const double* __restrict__ B, int64_t ldb, int32_t dpad,
                                                      int32_t RT, int32_t CT, const double* __restrict__ xnorm,
                                                      const double* __restrict__ cnorm,
                                                      const double* __restrict__ alpha, double sf2, int32_t n,
                                                      int64_t m, int32_t* __restrict__ ticket, TS* __restrict__ kst,
                                                      int64_t ldk, double* __restrict__ part, double kscale,
                                                      int64_t lo_off, int32_t store_rt, double* __restrict__ part2,
                                                      const int8_t* __restrict__ acat, const int8_t* __restrict__ bcat,
                                                      int32_t nkc, double cat_c0, double cat_c1, int32_t RTe) {
  // part2 (MU, fp64/fp32 only; pruned scoring): the column partial sum_r k*_r^2
  // as well, for the tail bound of the variance (gp.hip k_prune_bound)
  // TS = _Float16 (h3): k* * kscale split into fp16 hi + lo, stored candidate-major
  // in the blocked layout of k_gp_var_h3 (K = npad = RT * K_BM; ldk % 256 == 0);
  // the lo plane starts lo_off elements after the hi plane.  h3 permutes the
  // tile's training rows over the MFMA rows, pi(rho) = 4 (rho & 3) + (rho >> 2),
  // so that a lane's four accumulator rows (l >> 4) + 4 r hold the training
  // rows 4 (l >> 4) + r: four consecutive k of one candidate, 8 contiguous bytes
  // per plane in the blocked layout, stored straight from registers (round 3
  // transposed the tile through LDS with 128 ds_write_b16 per lane per item)
  constexpr bool H3 = sizeof(TS) == 2;
  // TS = int8_t (precision 8): y = k* * kscale (<= 0.49) as six balanced digit
  // planes of the int8 variance contraction (gp_i8.hip), four consecutive
  // training rows of a candidate per dword: the row permutation of h3
  constexpr bool I8 = sizeof(TS) == 1;
  constexpr bool PERM = H3 || I8;
  // one __shared__ object (see k_gp_var): the 2-stage ring, the exp table,
  // then the ticket slot
  constexpr int RED_OFF = 0;
  constexpr int MAIN = 2 * K_STAGE;
  // + the item's epilogue operands, staged by glds with its first K stage:
  // |x_r|^2 and alpha_r of its 128 rows, |u_c|^2 of its 128 columns (read from
  // LDS in the epilogue instead of 16 + 16 + 4 doubles held in VGPRs per lane:
  // the fp64 MU variant spilled 100 B/lane)
  __shared__ __attribute__((aligned(16))) double lds[MAIN + EXP_TAB + 2 + 3 * K_BM];
  double* etab = lds + MAIN;
  int32_t& s_item = *reinterpret_cast<int32_t*>(lds + MAIN + EXP_TAB);
  double* const rowop = lds + MAIN + EXP_TAB + 2;   // [xnorm 128][alpha 128][cnorm 128]
  const int t = threadIdx.x, lane = t & 63;
  // h3: the table carries the split's power-of-two scale, so ks below is
  // k* * kscale exactly (and the mean's alpha is divided by it: the product is
  // unchanged bit for bit)
  if (t < EXP_TAB) etab[t] = (sf2 * exp2((double)t / EXP_TAB)) * (PERM ? kscale : 1.0);  // published by the first ticket barrier
  const double ikscale = 1.0 / kscale;   // a power of two
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const int wm = w >> 1, wn = w & 1;
  const int32_t xcd = blockIdx.x & 7;
  // dpad % 4 == 0: whole 16-k stages, then one stage of k_rem k4 steps
  const int32_t nk_full = dpad / K_BK, k_rem = (dpad % K_BK) / 4;
  const int32_t nk = nk_full + (k_rem ? 1 : 0);
  const int32_t ncs = CAT ? nkc : 0;          // int8 stages first, then the fp64 ones
  const int32_t ntot = ncs + nk;
  const int npad_a = RT * K_BM;
  // the i8 MFMA's row rho of A is tile row sigma(rho) (see above); h3: the
  // f64 MFMA's row rho is tile row pi(rho), and the i8 one's row rho itself
  const int sig = PERM ? (lane & 15) : ((lane & 15) >> 2) + 4 * (lane & 3);
  const int arow = PERM ? 4 * (lane & 3) + ((lane & 15) >> 2) : (lane & 15);
  typedef kd4 d4;

  // the next item's ticket is taken at the start of the current one, so its
  // atomic round trip overlaps the item's first K stage instead of sitting
  // between two items (one ticket past the end per workgroup is drawn and unused)
  int32_t nxt = 0;
  if (t == 0) nxt = atomicAdd(&ticket[xcd], 1);
  for (;;) {
    if (t == 0) s_item = nxt;
    __syncthreads();
    const int32_t j = s_item;
    // (RTe <= RT: the item's row tiles; RT sizes the operands' layout)
    const int32_t ct = (j / RTe) * 8 + xcd;
    if (ct >= CT) break;
    if (t == 0) nxt = atomicAdd(&ticket[xcd], 1);
    const int32_t rt = j % RTe;
    const int64_t col0 = (int64_t)ct * K_BN;
    const int32_t row0 = rt * K_BM;

    auto issue_stage = [&](int32_t s2, double* st) {
      if (CAT && s2 < ncs)
        kcat_issue(acat + ((int64_t)s2 * npad_a + row0) * 128, bcat + ((int64_t)s2 * ldb + col0) * 128, st, w, lane);
      else
        kstar_issue(AT, lda, B, ldb, row0, col0, (s2 - ncs) * K_BK, st, w, lane, dpad);
    };
    if (ntot > 0) issue_stage(0, lds);
    {  // one 1-KiB glds per operand (rows < npad, columns < ldk are in range)
      const double* src = w == 0 ? xnorm + row0 : (w == 1 ? alpha + row0 : cnorm + col0);
      if (w < 3 && (MU || w != 1))
        __builtin_amdgcn_global_load_lds(src + lane * 2, (__attribute__((address_space(3))) void*)(rowop + w * K_BM),
                                         16, 0, 0);
    }
    d4 acc[4][4];
    if constexpr (CAT) {
      // the int8 stages: M into int32 accumulators (dead once acc is started)
      ki4 iacc[4][4];
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) iacc[i][jj] = (ki4){0, 0, 0, 0};
      for (int32_t s2 = 0; s2 < ncs; ++s2) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();  // stage s2 landed everywhere; stage s2-1 fully read
        asm volatile("" ::: "memory");
        if (s2 + 1 < ntot) issue_stage(s2 + 1, lds + ((s2 + 1) & 1) * K_STAGE);
        const int8_t* as8 = reinterpret_cast<const int8_t*>(lds + (s2 & 1) * K_STAGE);
        const int8_t* bs8 = as8 + K_SA * 8;
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
          const int c16 = (lane >> 4) + 4 * kk;
          ki4 af[4], bf[4];
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int row = wm * 64 + i * 16 + sig;
            af[i] = *reinterpret_cast<const ki4*>(as8 + row * 128 + ((c16 ^ (row & 7)) << 4));
          }
#pragma unroll
          for (int jj = 0; jj < 4; ++jj) {
            const int col = wn * 64 + jj * 16 + (lane & 15);
            bf[jj] = *reinterpret_cast<const ki4*>(bs8 + col * 128 + ((c16 ^ (col & 7)) << 4));
          }
#pragma unroll
          for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int jj = 0; jj < 4; ++jj)
              iacc[i][jj] = __builtin_amdgcn_mfma_i32_16x16x64_i8(af[i], bf[jj], iacc[i][jj], 0, 0, 0);
        }
      }
      // c0 + c1 M starts the fp64 accumulators
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int jj = 0; jj < 4; ++jj)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            acc[i][jj][r] = __builtin_fma((double)iacc[i][jj][r], cat_c1, cat_c0);   // (in t units: see the launch)
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) acc[i][jj] = (d4){0.0, 0.0, 0.0, 0.0};
    }
    for (int32_t s2 = ncs; s2 < ntot; ++s2) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();  // stage s2 landed everywhere; stage s2-1 fully read
      asm volatile("" ::: "memory");
      if (s2 + 1 < ntot) issue_stage(s2 + 1, lds + ((s2 + 1) & 1) * K_STAGE);
      const double* as = lds + (s2 & 1) * K_STAGE;
      const int32_t kt = s2 - ncs;
      const double* bs = as + K_SA;
      // the last stage of a dpad that is not a multiple of 16 has k_rem k4 steps
      const int nks = kt < nk_full ? K_BK / 4 : k_rem;
#pragma unroll
      for (int ks = 0; ks < K_BK / 4; ++ks) {
        if (ks >= nks) break;
        const int kr = ks * 4 + (lane >> 4);
        double af[4], bf[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) af[i] = as[kr * K_BM + wm * 64 + i * 16 + arow];
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) bf[jj] = bs[kr * K_BN + wn * 64 + jj * 16 + (lane & 15)];
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int jj = 0; jj < 4; ++jj)
            acc[i][jj] = __builtin_amdgcn_mfma_f64_16x16x4f64(af[i], bf[jj], acc[i][jj], 0, 0, 0);
      }
    }
    if (ntot == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the epilogue operands

    __syncthreads();  // ring free: reuse as the column reduction buffer (and the h3 image)
    if constexpr (I8) {
      // the rows' epilogue operands once per item instead of once per column
      // group: the half-norm with the padding rows' -1e300, alpha / kscale
      if (t < K_BM) {
        const double hv = (-0.5 * KSTAR_T_SCALE) * rowop[t];
        rowop[t] = row0 + t < n ? hv : -1e300;
        rowop[K_BM + t] = rowop[K_BM + t] * ikscale;
      }
      __syncthreads();
    }
    double* red = lds + RED_OFF;  // [2][128]
    // epilogue operands from the LDS copies (landed with the first K stage).
    // Padding rows / columns get a huge negative half-norm, so their k* is
    // exactly 0 without a select.
    // (every LDS read is unconditional and the padding goes in by a select:
    // a branch around a read splits the epilogue into basic blocks and each
    // read's wait then stalls the wave instead of overlapping other elements)
    double hc[4];
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) {
      const int cl = wn * 64 + jj * 16 + (lane & 15);
      const double hv = (-0.5 * KSTAR_T_SCALE) * rowop[2 * K_BM + cl];
      hc[jj] = col0 + cl < m ? hv : -1e300;
    }
    const bool want2 = !PERM && MU && part2 != nullptr;
    double s[4] = {0.0, 0.0, 0.0, 0.0}, s2[4] = {0.0, 0.0, 0.0, 0.0};
    if constexpr (H3) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        // the four rows of this lane in row group i: training rows 4 (l >> 4) + r
        const int rl0 = wm * 64 + i * 16 + 4 * (lane >> 4);
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
          const int64_t col = col0 + wn * 64 + jj * 16 + (lane & 15);
          uint32_t hpk[2] = {0u, 0u}, lpk[2] = {0u, 0u};   // the four rows' fp16 hi / lo, packed
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const double hv = (-0.5 * KSTAR_T_SCALE) * rowop[rl0 + r];
            const double hx = row0 + rl0 + r < n ? hv : -1e300;
            const double x = __builtin_fmax(__builtin_fmin((acc[i][jj][r] + hx) + hc[jj], 0.0), KSTAR_T_MIN);
            const double ks = sf2_exp2t_nonpos(x, etab);
            // ks = k* * kscale (< 2^15): hi = fp16(ks), lo = fp16 of the rest,
            // the rest taken in f32 (exact there: hi is within 2^-11 of xf)
            const float xf = (float)ks;
            const _Float16 hi = (_Float16)xf;
            const uint32_t hb = __builtin_bit_cast(uint16_t, hi);
            const uint32_t lb = __builtin_bit_cast(uint16_t, (_Float16)(xf - (float)hi));
            hpk[r >> 1] |= (r & 1) ? hb << 16 : hb;
            lpk[r >> 1] |= (r & 1) ? lb << 16 : lb;
            s[jj] += (rowop[K_BM + rl0 + r] * ikscale) * ks;
          }
          // rows 4 (l >> 4) .. + 3 of this column: 8 bytes per plane in the blocked layout
          const int64_t o = h3_blk_off(col, row0 + rl0, RT * K_BM);
          *reinterpret_cast<uint2*>(kst + o) = make_uint2(hpk[0], hpk[1]);
          *reinterpret_cast<uint2*>(kst + lo_off + o) = make_uint2(lpk[0], lpk[1]);
        }
      }
    } else if constexpr (I8) {
      // per column group: the four row groups' digit dwords (lane row R = l >> 4
      // holds rows 16 i + 4 R .. + 3 of its column for i = 0..3), transposed
      // over (R, i) by two v_permlane32_swap + two v_permlane16_swap per plane
      // so that lane row R holds rows 16 R .. 16 R + 15: one 16-byte store per
      // plane, the 32-byte pieces of 16 consecutive candidates written whole
      // (four 4-byte stores per plane left pieces half written per instruction:
      // 1.4x the planes' bytes reached HBM)
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) {
        const int64_t col = col0 + wn * 64 + jj * 16 + (lane & 15);
        uint32_t pw[I8_S][4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int rl0 = wm * 64 + i * 16 + 4 * (lane >> 4);   // this lane's training rows rl0 .. rl0 + 3
          uint32_t lo[4], hi[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const double x = __builtin_fmax(__builtin_fmin((acc[i][jj][r] + rowop[rl0 + r]) + hc[jj], 0.0), KSTAR_T_MIN);
            const double ks = sf2_exp2t_nonpos(x, etab);   // y = k* 2^-eb
            s[jj] = __builtin_fma(rowop[K_BM + rl0 + r], ks, s[jj]);
            const uint64_t b = i8_biased(ks);
            lo[r] = (uint32_t)b;
            hi[r] = (uint32_t)(b >> 32);
          }
          uint32_t pl[I8_S];
          i8_planes(lo, hi, pl);
#pragma unroll
          for (int p = 0; p < I8_S; ++p) pw[p][i] = pl[p];
        }
#pragma unroll
        for (int p = 0; p < I8_S; ++p) {
          const auto a0 = __builtin_amdgcn_permlane32_swap(pw[p][0], pw[p][2], false, false);
          const auto a1 = __builtin_amdgcn_permlane32_swap(pw[p][1], pw[p][3], false, false);
          const auto b0 = __builtin_amdgcn_permlane16_swap(a0[0], a1[0], false, false);
          const auto b1 = __builtin_amdgcn_permlane16_swap(a0[1], a1[1], false, false);
          pw[p][0] = b0[0];
          pw[p][1] = b0[1];
          pw[p][2] = b1[0];
          pw[p][3] = b1[1];
        }
        // lo_off: bytes per plane
        int8_t* dst = reinterpret_cast<int8_t*>(kst) + i8_off(col, row0 + wm * 64 + 16 * (lane >> 4), ldk);
#pragma unroll
        for (int p = 0; p < I8_S; ++p)
          *reinterpret_cast<uint4*>(dst + p * lo_off) = make_uint4(pw[p][0], pw[p][1], pw[p][2], pw[p][3]);
      }
    } else {
      // STORE: this tile's rows are stored (pruned scoring stores the bound
      // rows only); decided once per item, so the element code has no branch
      auto epi = [&](auto store_c) {
        constexpr bool STORE = decltype(store_c)::value;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int rl = wm * 64 + i * 16 + (lane >> 4) + 4 * r;
            const int32_t row = row0 + rl;
            const double hv = (-0.5 * KSTAR_T_SCALE) * rowop[rl];
            const double hx = row < n ? hv : -1e300;
            double al = 0.0;
            if constexpr (MU) al = rowop[K_BM + rl];
            TS* kp = kst + (int64_t)row * ldk + col0 + wn * 64 + (lane & 15);
#pragma unroll
            for (int jj = 0; jj < 4; ++jj) {
              // t = (C - |x|^2/2 - |u|^2/2) * 256 / ln 2, clamped to [-1000 * 256 / ln 2, 0]
              const double x = __builtin_fmax(__builtin_fmin((acc[i][jj][r] + hx) + hc[jj], 0.0), KSTAR_T_MIN);
              const double ks = sf2_exp2t_nonpos(x, etab);
              if constexpr (STORE) kp[jj * 16] = (TS)ks;
              // (fused: the build contracts nothing by itself)
              if constexpr (MU) s[jj] = __builtin_fma(al, ks, s[jj]);
              if constexpr (MU) s2[jj] = __builtin_fma(ks, ks, s2[jj]);
            }
          }
        }
      };
      if (rt < store_rt) epi(std::integral_constant<bool, true>{});
      else epi(std::integral_constant<bool, false>{});
    }
    if constexpr (MU) {
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) {
        const int cl = wn * 64 + jj * 16 + (lane & 15);
        double a = s[jj];
        a += __shfl_xor(a, 16);
        a += __shfl_xor(a, 32);
        if ((lane >> 4) == 0) red[wm * K_BN + cl] = a;
        if (want2) {
          double b = s2[jj];
          b += __shfl_xor(b, 16);
          b += __shfl_xor(b, 32);
          if ((lane >> 4) == 0) red[2 * K_BN + wm * K_BN + cl] = b;
        }
      }
    }
    if constexpr (MU) __syncthreads();
    if constexpr (MU) {
      if (t < K_BN) {
        const int64_t col = col0 + t;
        if (col < m) {
          part[(int64_t)rt * ldk + col] = red[t] + red[K_BN + t];
          if (want2) part2[(int64_t)rt * ldk + col] = red[2 * K_BN + t] + red[3 * K_BN + t];
        }
      }
    }
  }
}

// ---------------------------------------------------------------------------
// Pruned scoring's bound pass in f32 (ut_gp_set_prune_pass 32, the default):
// row tiles rt0 .. RT-1 of K* (the bound rows before rt0 run through
// k_gp_kstar's fp64 epilogue), A = f32(Xs^T) and B = f32(U') on
// v_mfma_f32_16x16x4f32 (1.9x the f64 MFMA's rate; C/D: col = lane & 15, row =
// 4 (lane >> 4) + r, the i8 MFMA's map; scripts/exp/f32_mfma_probe.hip), then
// from the f32 accumulator t = C + hx + hc in f32 (t in units of 2^(1/256), the
// operands' KSTAR_T_SCALE), k* = sf2 2^(t/256) by v_exp_f32, and the tile
// partials of k* alpha, k* |alpha| and k*^2 as f32 sums: ~7 VALU ops per k*
// against the fp64 epilogue's ~15 DP ops, and the f32 MFMA, like the f64 one,
// does not issue beside them.  Error (k_prune_bound32):
// every partial sum of the contraction is at most |c0| + |x|^2/2 + |u|^2/2 in
// magnitude (|x . u| <= (|x|^2 + |u|^2) / 2), so |t^ - t| <= (K + 9) 2^-24
// (2 |c0| + |x|^2 + |u|^2) (units of t; K the contraction length: products
// and sums rounded to f32, hx / hc rounded once, two adds).
// ---------------------------------------------------------------------------
typedef float kf4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void kstar_issue_f32(const float* __restrict__ AT, int64_t lda, const float* __restrict__ B,
                                                int64_t ldb, int32_t row0, int64_t col0, int32_t k0, float* st, int w,
                                                int lane, int32_t dpad) {
  // 8 KiB of A and 8 KiB of B per 16-k stage: wave w loads k rows 4w .. 4w+3,
  // two 512-B rows per 1-KiB glds (lanes 0-31 row q, 32-63 row q + 1)
  if (k0 + 4 * w >= dpad) return;
  const int rr = lane >> 5, cc = (lane & 31) * 4;
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int q = 4 * w + 2 * u;
    __builtin_amdgcn_global_load_lds(AT + (int64_t)(k0 + q + rr) * lda + row0 + cc,
                                     (__attribute__((address_space(3))) void*)(st + q * 128), 16, 0, 0);
    __builtin_amdgcn_global_load_lds(B + (int64_t)(k0 + q + rr) * ldb + col0 + cc,
                                     (__attribute__((address_space(3))) void*)(st + K_SA + q * 128), 16, 0, 0);
  }
}

template <bool CAT>
__global__ __launch_bounds__(K_NT, 2) void k_gp_kstar_f32c(const float* __restrict__ AT, int64_t lda,
                                                           const float* __restrict__ B, int64_t ldb, int32_t dpad,
                                                           int32_t rt0, int32_t RT, int32_t CT,
                                                           const double* __restrict__ xnorm,
                                                           const double* __restrict__ cnorm,
                                                           const double* __restrict__ alpha, double sf2, int32_t n,
                                                           int64_t m, int32_t* __restrict__ ticket, int64_t ldk,
                                                           double* __restrict__ part, double* __restrict__ part2,
                                                           double* __restrict__ part3, const int8_t* __restrict__ acat,
                                                           const int8_t* __restrict__ bcat, int32_t nkc, float cat_c0,
                                                           float cat_c1) {
  // the ring (sized as k_gp_kstar's: the int8 stages fill it, the f32 ones half),
  // the ticket slot, the item's row / column operands
  __shared__ __attribute__((aligned(16))) double lds[2 * K_STAGE + 2 + 3 * K_BM];
  int32_t& s_item = *reinterpret_cast<int32_t*>(lds + 2 * K_STAGE);
  double* const rowop = lds + 2 * K_STAGE + 2;   // [xnorm 128][alpha 128][cnorm 128]
  const int t = threadIdx.x, lane = t & 63;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const int wm = w >> 1, wn = w & 1;
  const int32_t xcd = blockIdx.x & 7;
  const int32_t nk_full = dpad / K_BK, k_rem = (dpad % K_BK) / 4;
  const int32_t nk = nk_full + (k_rem ? 1 : 0);
  const int32_t ncs = CAT ? nkc : 0;
  const int32_t ntot = ncs + nk;
  const int npad_a = RT * K_BM;
  const int32_t RTe = RT - rt0;
  int32_t nxt = 0;
  if (t == 0) nxt = atomicAdd(&ticket[xcd], 1);
  for (;;) {
    if (t == 0) s_item = nxt;
    __syncthreads();
    const int32_t j = s_item;
    const int32_t ct = (j / RTe) * 8 + xcd;
    if (ct >= CT) break;
    if (t == 0) nxt = atomicAdd(&ticket[xcd], 1);
    const int32_t rt = rt0 + j % RTe;
    const int64_t col0 = (int64_t)ct * K_BN;
    const int32_t row0 = rt * K_BM;
    auto issue_stage = [&](int32_t s2, double* st) {
      if (CAT && s2 < ncs)
        kcat_issue(acat + ((int64_t)s2 * npad_a + row0) * 128, bcat + ((int64_t)s2 * ldb + col0) * 128, st, w, lane);
      else
        kstar_issue_f32(AT, lda, B, ldb, row0, col0, (s2 - ncs) * K_BK, reinterpret_cast<float*>(st), w, lane, dpad);
    };
    if (ntot > 0) issue_stage(0, lds);
    {
      const double* src = w == 0 ? xnorm + row0 : (w == 1 ? alpha + row0 : cnorm + col0);
      if (w < 3)
        __builtin_amdgcn_global_load_lds(src + lane * 2, (__attribute__((address_space(3))) void*)(rowop + w * K_BM),
                                         16, 0, 0);
    }
    kf4 acc[4][4];
    if constexpr (CAT) {
      ki4 iacc[4][4];
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) iacc[i][jj] = (ki4){0, 0, 0, 0};
      for (int32_t s2 = 0; s2 < ncs; ++s2) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        if (s2 + 1 < ntot) issue_stage(s2 + 1, lds + ((s2 + 1) & 1) * K_STAGE);
        const int8_t* as8 = reinterpret_cast<const int8_t*>(lds + (s2 & 1) * K_STAGE);
        const int8_t* bs8 = as8 + K_SA * 8;
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
          const int c16 = (lane >> 4) + 4 * kk;
          ki4 af[4], bf[4];
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int row = wm * 64 + i * 16 + (lane & 15);   // the f32 MFMA's rows are the i8 one's
            af[i] = *reinterpret_cast<const ki4*>(as8 + row * 128 + ((c16 ^ (row & 7)) << 4));
          }
#pragma unroll
          for (int jj = 0; jj < 4; ++jj) {
            const int col = wn * 64 + jj * 16 + (lane & 15);
            bf[jj] = *reinterpret_cast<const ki4*>(bs8 + col * 128 + ((c16 ^ (col & 7)) << 4));
          }
#pragma unroll
          for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int jj = 0; jj < 4; ++jj)
              iacc[i][jj] = __builtin_amdgcn_mfma_i32_16x16x64_i8(af[i], bf[jj], iacc[i][jj], 0, 0, 0);
        }
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int jj = 0; jj < 4; ++jj)
#pragma unroll
          for (int r = 0; r < 4; ++r) acc[i][jj][r] = __builtin_fmaf((float)iacc[i][jj][r], cat_c1, cat_c0);
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) acc[i][jj] = (kf4){0.f, 0.f, 0.f, 0.f};
    }
    for (int32_t s2 = ncs; s2 < ntot; ++s2) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      if (s2 + 1 < ntot) issue_stage(s2 + 1, lds + ((s2 + 1) & 1) * K_STAGE);
      const float* as = reinterpret_cast<const float*>(lds + (s2 & 1) * K_STAGE);
      const float* bs = as + K_SA;
      const int32_t kt = s2 - ncs;
      const int nks = kt < nk_full ? K_BK / 4 : k_rem;
#pragma unroll
      for (int ks = 0; ks < K_BK / 4; ++ks) {
        if (ks >= nks) break;
        const int kr = ks * 4 + (lane >> 4);
        float af[4], bf[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) af[i] = as[kr * K_BM + wm * 64 + i * 16 + (lane & 15)];
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) bf[jj] = bs[kr * K_BN + wn * 64 + jj * 16 + (lane & 15)];
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int jj = 0; jj < 4; ++jj)
            acc[i][jj] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[i], bf[jj], acc[i][jj], 0, 0, 0);
      }
    }
    if (ntot == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();   // ring free: the column reduction buffer
    double* red = lds;   // [6][128]
    float hc[4];
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) {
      const int cl = wn * 64 + jj * 16 + (lane & 15);
      hc[jj] = col0 + cl < m ? (float)((-0.5 * KSTAR_T_SCALE) * rowop[2 * K_BM + cl]) : -1.0f / 0.0f;
    }
    float fs[4] = {0.f, 0.f, 0.f, 0.f}, fa[4] = {0.f, 0.f, 0.f, 0.f}, f2[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int rl = wm * 64 + i * 16 + 4 * (lane >> 4) + r;
        const float hx = row0 + rl < n ? (float)((-0.5 * KSTAR_T_SCALE) * rowop[rl]) : -1.0f / 0.0f;
        const float al = (float)(rowop[K_BM + rl] * sf2);
        const float aa = __builtin_fabsf(al);
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
          const float kf = __builtin_amdgcn_exp2f(((acc[i][jj][r] + hx) + hc[jj]) * 0x1p-8f);
          fs[jj] = __builtin_fmaf(al, kf, fs[jj]);
          fa[jj] = __builtin_fmaf(aa, kf, fa[jj]);
          f2[jj] = __builtin_fmaf(kf, kf, f2[jj]);
        }
      }
    }
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) {
      const int cl = wn * 64 + jj * 16 + (lane & 15);
      double a = fs[jj], b = f2[jj], q = fa[jj];
      a += __shfl_xor(a, 16);
      a += __shfl_xor(a, 32);
      b += __shfl_xor(b, 16);
      b += __shfl_xor(b, 32);
      q += __shfl_xor(q, 16);
      q += __shfl_xor(q, 32);
      if ((lane >> 4) == 0) {
        red[wm * K_BN + cl] = a;
        red[2 * K_BN + wm * K_BN + cl] = b;
        red[4 * K_BN + wm * K_BN + cl] = q;
      }
    }
    __syncthreads();
    if (t < K_BN) {
      const int64_t col = col0 + t;
      if (col < m) {
        part[(int64_t)rt * ldk + col] = red[t] + red[K_BN + t];
        part2[(int64_t)rt * ldk + col] = (red[2 * K_BN + t] + red[3 * K_BN + t]) * (sf2 * sf2);
        part3[(int64_t)rt * ldk + col] = red[4 * K_BN + t] + red[5 * K_BN + t];
      }
    }
  }
}

int launch_gemm_kstar_f32c(ut_ctx* c, const float* XsT_f, int32_t npad, const float* ucand_f, int32_t dpad,
                           int64_t m, int64_t ldk, int32_t rt0, double* part, double* part2, double* part3,
                           const KstarCat& cat, const double* xn, const double* cn) {
  const bool has_cat = cat.nkc > 0;
  UT_CHECK(c, npad % K_BM == 0 && dpad % 4 == 0 && (dpad >= 4 || has_cat) && ldk % K_BN == 0 && ldk >= m, UT_EINVAL,
           "gemm_kstar_f32c: bad padding");
  UT_CHECK(c, !has_cat || (cat.acat && cat.bcat), UT_EINVAL, "gemm_kstar_f32c: categorical operands missing");
  UT_CHECK(c, part && part2 && part3, UT_EINVAL, "gemm_kstar_f32c: partial outputs missing");
  const int32_t RT = npad / K_BM;
  UT_CHECK(c, rt0 >= 0 && rt0 < RT, UT_EINVAL, "gemm_kstar_f32c: bad first row tile");
  const int32_t CT = (int32_t)(ldk / K_BN);
  const int64_t items = (int64_t)(RT - rt0) * CT;
  int32_t nb = 2 * (c->n_cu / 8) * 8;
  if (items < nb) nb = (int32_t)(((items + 7) / 8) * 8);
  UT_HIP(c, hipMemsetAsync(c->gp_ctr + 8, 0, sizeof(int32_t) * 8, c->stream));
  const float c0 = (float)(cat.c0 * KSTAR_T_SCALE), c1 = (float)(cat.c1 * KSTAR_T_SCALE);
  if (has_cat)
    hipLaunchKernelGGL(k_gp_kstar_f32c<true>, dim3(nb), dim3(K_NT), 0, c->stream, XsT_f, (int64_t)npad, ucand_f, ldk,
                       dpad, rt0, RT, CT, xn, cn, c->gp_alpha, c->gp_sf2, c->gp_n, m, c->gp_ctr + 8, ldk, part, part2,
                       part3, cat.acat, cat.bcat, cat.nkc, c0, c1);
  else
    hipLaunchKernelGGL(k_gp_kstar_f32c<false>, dim3(nb), dim3(K_NT), 0, c->stream, XsT_f, (int64_t)npad, ucand_f, ldk,
                       dpad, rt0, RT, CT, xn, cn, c->gp_alpha, c->gp_sf2, c->gp_n, m, c->gp_ctr + 8, ldk, part, part2,
                       part3, cat.acat, cat.bcat, cat.nkc, c0, c1);
  UT_LAUNCH_CHECK(c);
  return 0;
}

int h3_kstar_exp(double sf2) { return H3_KSCALE_EXP - ilogb(sf2); }  // sf2 * 2^e < 2^15

int launch_gemm_kstar(ut_ctx* c, int prec, const double* XsT, int32_t npad, const double* ucand, int32_t dpad,
                      int64_t m, void* kst, int64_t ldk, double* part, int32_t store_rows, const double* cn,
                      double* part2, const KstarCat& cat, const double* xn, int32_t row_tiles) {
  const bool has_cat = cat.nkc > 0;
  UT_CHECK(c, npad % K_BM == 0 && dpad % 4 == 0 && (dpad >= 4 || has_cat) && ldk % K_BN == 0 && ldk >= m, UT_EINVAL,
           "gemm_kstar: bad padding");
  UT_CHECK(c, !has_cat || (cat.acat && cat.bcat), UT_EINVAL, "gemm_kstar: categorical operands missing");
  UT_CHECK(c, prec == 64 || prec == 32 || prec == 16 || prec == 8, UT_EINVAL, "gemm_kstar: bad precision");
  UT_CHECK(c, part != nullptr || prec == 64 || prec == 8, UT_EINVAL,
           "gemm_kstar: fp32 / h3 mode takes the mean partial here");
  const int32_t RT = npad / K_BM;
  // row_tiles: only the first row_tiles tiles (the f32-contraction bound pass's fp64 bound rows)
  const int32_t RTe = row_tiles > 0 && row_tiles < RT ? row_tiles : RT;
  const int32_t CT = (int32_t)(ldk / K_BN);  // every column of K* (zeros past m) is written
  // fp64: only the first store_rows rows of K* are written (the mean still
  // sums every row); the other precisions always store everything
  const int32_t store_rt = store_rows < 0 ? RT : (store_rows + K_BM - 1) / K_BM;
  const int64_t items = (int64_t)RTe * CT;
  // Two K* workgroups fill a CU's VGPRs, so a full persistent grid leaves no
  // slot for the GP fit running beside it on the fit stream, and the fit's
  // serial chain of small kernels then stalls the variance GEMM that waits for
  // it.  While a fit is in flight, 2 CUs per XCD are left to it (C2: the round
  // with a refit 30.2 -> 29.6 ms, the same as without a refit; K* alone 3% slower).
  const bool fit_in_flight = c->fit_pending && hipEventQuery(c->ev_fit) == hipErrorNotReady;
  const int32_t spare = fit_in_flight ? KSTAR_SPARE_PER_XCD : 0;
  int32_t nb = 2 * (c->n_cu / 8 - spare) * 8;
  if (items < nb) nb = (int32_t)(((items + 7) / 8) * 8);
  UT_HIP(c, hipMemsetAsync(c->gp_ctr + 8, 0, sizeof(int32_t) * 8, c->stream));
  const double* xnorm = xn ? xn : c->gp_xnorm;
  const double* cnorm = cn ? cn : c->cnorm.p;
#define UT_KSTAR_LAUNCH(TS, MU, CAT, KST, PART, KSCALE, LOOFF, SRT, PART2)                                         \
  hipLaunchKernelGGL((k_gp_kstar<TS, MU, CAT>), dim3(nb), dim3(K_NT), 0, c->stream, XsT, (int64_t)npad, ucand, ldk, \
                     dpad, RT, CT, xnorm, cnorm, c->gp_alpha, c->gp_sf2, c->gp_n, m, c->gp_ctr + 8, KST, ldk, PART, \
                     KSCALE, LOOFF, SRT, PART2, cat.acat, cat.bcat, cat.nkc, cat.c0 * KSTAR_T_SCALE,        \
                     cat.c1 * KSTAR_T_SCALE, RTe)
#define UT_KSTAR_BOTH(TS, MU, ...)                   \
  do {                                               \
    if (has_cat) UT_KSTAR_LAUNCH(TS, MU, true, __VA_ARGS__); \
    else UT_KSTAR_LAUNCH(TS, MU, false, __VA_ARGS__);        \
  } while (0)
  if (prec == 16)
    UT_KSTAR_BOTH(_Float16, true, (_Float16*)kst, part, ldexp(1.0, h3_kstar_exp(c->gp_sf2)), ldk * (int64_t)npad, RT,
                  nullptr);
  else if (prec == 8)   // six digit planes of npad * ldk bytes (kst: [6][npad / 32][ldk][32]); the
                        // mean comes from the int8 variance epilogue (part == nullptr: K* needs no alpha)
    UT_KSTAR_BOTH(int8_t, false, (int8_t*)kst, part, ldexp(1.0, -i8_kstar_exp(c->gp_sf2)), ldk * (int64_t)npad, RT,
                  nullptr);
  else if (prec == 32)
    UT_KSTAR_BOTH(float, true, (float*)kst, part, 1.0, (int64_t)0, RT, nullptr);
  else if (part)   // fp64 with the mean k* . alpha in the epilogue (pruned scoring: needs the whole fit)
    UT_KSTAR_BOTH(double, true, (double*)kst, part, 1.0, (int64_t)0, store_rt, part2);
  else
    UT_KSTAR_BOTH(double, false, (double*)kst, part, 1.0, (int64_t)0, store_rt, nullptr);
#undef UT_KSTAR_BOTH
#undef UT_KSTAR_LAUNCH
  UT_LAUNCH_CHECK(c);
  return 0;
}

// U'[k][i] = feat[k][i] / ell_k (0 for k >= d or i >= m), cnorm[i] = |u'_i|^2
__global__ void k_gp_prep_cand(const double* __restrict__ feat, int64_t ld, int64_t m, int32_t d, int32_t dpad,
                               const double* __restrict__ inv_ell, double* __restrict__ u, int64_t ldu,
                               double* __restrict__ cn) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= ldu) return;
  double s = 0.0;
  for (int32_t k = 0; k < dpad; ++k) {
    const double v = (k < d && i < m) ? feat[(int64_t)k * ld + i] * inv_ell[k] : 0.0;
    u[(int64_t)k * ldu + i] = v;
    s += v * v;
  }
  cn[i] = s;
}

int launch_prep_cand(ut_ctx* c, const double* feat, int64_t ld, int64_t m, int32_t d, int32_t dpad, double* u,
                     int64_t ldu, double* cn) {
  hipLaunchKernelGGL(k_gp_prep_cand, dim3(grid1(ldu, 256)), dim3(256), 0, c->stream, feat, ld, m, d, dpad,
                     c->gp_inv_ell, u, ldu, cn);
  UT_LAUNCH_CHECK(c);
  return 0;
}

// k_gp_prep_cand for the categorical K*, from a feature matrix made by ut's own
// encoder (ENUM blocks one-hot, BOOL 0 / 1): numeric U' and norms as
// k_encode_scaled_cat writes them, codes from the blocks (the first 1.0 of an
// ENUM block; no 1.0: no code, as for an out-of-range value)
__global__ __launch_bounds__(256) void k_gp_prep_cand_cat(const DevParam* __restrict__ params, int32_t P,
                                                          const double* __restrict__ feat, int64_t ld, int64_t m,
                                                          const int32_t* __restrict__ num_feat, int32_t n_num,
                                                          int32_t dpad, const double* __restrict__ inv_ell,
                                                          const int32_t* __restrict__ cat_ccol, int32_t cat_k,
                                                          double* __restrict__ u, int64_t ldu,
                                                          double* __restrict__ cn, int8_t* __restrict__ bcat) {
  extern __shared__ uint32_t dyn[];
  const int32_t stride = cat_k / 32 + 1;
  uint32_t* bits = dyn;
  uint32_t* img = dyn + 256 * stride;
  const int t = threadIdx.x;
  const int64_t i0 = (int64_t)blockIdx.x * 256, i = i0 + t;
  for (int32_t w = 0; w < stride; ++w) bits[t * stride + w] = 0u;
  double s = 0.0;
  for (int32_t k = 0; k < dpad; ++k) {
    const int32_t f = k < n_num ? num_feat[k] : 0;
    const double v = (k < n_num && i < m) ? feat[(int64_t)f * ld + i] * inv_ell[f] : 0.0;
    u[(int64_t)k * ldu + i] = v;
    s += v * v;
  }
  cn[i] = s;
  if (i < m) {
    for (int32_t p = 0; p < P; ++p) {
      const int32_t cc = cat_ccol[p];
      if (cc < 0) continue;
      const DevParam pr = params[p];
      const double* x = feat + (int64_t)pr.feat_col * ld + i;
      int32_t o = -1;
      if (pr.kind == UT_BOOL) {
        o = x[0] != 0.0 ? 1 : 0;
      } else {
        for (int32_t k = 0; k < (int32_t)pr.n_opt; ++k)
          if (x[(int64_t)k * ld] == 1.0) { o = k; break; }
      }
      if (o < 0) continue;
      const int32_t q = cc + o;
      bits[t * stride + (q >> 5)] |= 1u << (q & 31);
    }
  }
  __syncthreads();
  store_code_rows(bits, stride, cat_k / 128, img, bcat, ldu, i0);
}

int launch_prep_cand_cat(ut_ctx* c, const double* feat, int64_t ld, int64_t m, double* u, int32_t dpad, int64_t ldu,
                         double* cn, int8_t* bcat) {
  const Space& s = c->space;
  UT_CHECK(c, ldu % 256 == 0 && s.cat_k % 128 == 0, UT_EINVAL, "prep_cand_cat: bad padding");
  hipLaunchKernelGGL(k_gp_prep_cand_cat, dim3((unsigned)(ldu / 256)), dim3(256), code_rows_lds(s.cat_k), c->stream,
                     s.d_params, s.P, feat, ld, m, s.d_num_feat, s.n_num, dpad, c->gp_inv_ell, s.d_cat_ccol, s.cat_k,
                     u, ldu, cn, bcat);
  UT_LAUNCH_CHECK(c);
  return 0;
}

// Xs^T [dpad][npad] from Xs [npad][d] (rows >= d zero)
__global__ void k_gp_xs_t(const double* __restrict__ Xs, int32_t npad, int32_t d, int32_t dpad,
                          double* __restrict__ XsT) {
  fit_prio_g();
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= (int64_t)dpad * npad) return;
  const int32_t k = (int32_t)(e / npad), r = (int32_t)(e % npad);
  XsT[e] = (k < d) ? Xs[(int64_t)r * d + k] * KSTAR_T_SCALE : 0.0;   // the K* operand, in 2^(1/256) units
}

int launch_xs_t(ut_ctx* c, const double* Xs, int32_t npad, int32_t d, int32_t dpad, double* XsT) {
  hipLaunchKernelGGL(k_gp_xs_t, dim3(grid1((int64_t)dpad * npad, 256)), dim3(256), 0, c->stream, Xs, npad, d, dpad,
                     XsT);
  UT_LAUNCH_CHECK(c);
  return 0;
}

// ---------------------------------------------------------------------------
// Variance contraction, persistent:  part[rt][col] = sum_{r in tile rt} (L^-1 K*^T)[r][col]^2
//
// fp32 (precision 32): one 512-thread workgroup per CU (8 waves as 2 x 4 of 64 x 64 outputs) walks
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
//   v_mfma_f32_32x32x2_f32, BK 32 (the fp64 tier's kernel is k_gp_var_pp below)
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

typedef double vd4 __attribute__((ext_vector_type(4)));
typedef float vf16 __attribute__((ext_vector_type(16)));

// one BK step of the fp32 variance contraction for row sub-tiles i >= imin
// (imin wave-uniform: scalar branches around each sub-tile's MFMAs)
__device__ __forceinline__ void var_step_f32(const float* as, const float* bs, int wm, int wn, int lane, int imin,
                                             vf16 (&acc)[2][2]) {
#pragma unroll
  for (int ks = 0; ks < 16; ++ks) {
    const int kr = ks * 2 + (lane >> 5);
    float af[2], bf[2];
#pragma unroll
    for (int jj = 0; jj < 2; ++jj) bf[jj] = bs[kr * VAR_BN + wn * 64 + jj * 32 + (lane & 31)];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      if (i < imin) continue;
      af[i] = as[kr * VAR_BM + wm * 64 + i * 32 + (lane & 31)];
#pragma unroll
      for (int jj = 0; jj < 2; ++jj) acc[i][jj] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[i], bf[jj], acc[i][jj], 0, 0, 0);
    }
  }
}

__global__ __launch_bounds__(V_NT, 1) void k_gp_var_f32(const float* __restrict__ AT, int64_t lda,
                                                         const float* __restrict__ B, int64_t ldb, int32_t K,
                                                         int32_t RT, int32_t CT, int64_t m,
                                                         int32_t* __restrict__ ticket, double* __restrict__ part,
                                                         int64_t ldp) {
  using C = VCfg<float>;
  constexpr int BK = C::BK;
  // ALL LDS in one object: a second __shared__ beside the glds ring makes
  // hipcc wait vmcnt(0) before every step's first ds_read (drains the ring)
  __shared__ __attribute__((aligned(16))) float lds[V_ST * C::STAGE + 4];
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

    vf16 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int jj = 0; jj < 2; ++jj)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[i][jj][r] = 0.0f;

    var_issue<float>(AT, lda, B, ldb, row0, col0, 0, lds, w, lane);
    if (nk > 1) var_issue<float>(AT, lda, B, ldb, row0, col0, BK, lds + C::STAGE, w, lane);
    // one pipeline step: retire stage kt (6 glds per wave per stage; stage kt+1
    // stays in flight), then refill the slot of stage kt-1 with stage kt+2
    auto pipe = [&](int32_t kt) -> const float* {
      if (kt + 1 < nk)
        asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
      else
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();  // all waves' stage kt landed; all reads of stage kt-1 done
      asm volatile("" ::: "memory");
      if (kt + 2 < nk)
        var_issue<float>(AT, lda, B, ldb, row0, col0, (kt + 2) * BK, lds + ((kt + 2) % V_ST) * C::STAGE, w, lane);
      return lds + (kt % V_ST) * C::STAGE;
    };
    // k blocks left of the diagonal block: every MFMA sub-tile
    const int32_t nfull = min(nk, row0 / BK);
    for (int32_t kt = 0; kt < nfull; ++kt) {
      const float* as = pipe(kt);
      var_step_f32(as, as + C::SA, wm, wn, lane, 0, acc);
    }
    // the diagonal block: (L^-1)^T is zero for k > row, so the MFMA sub-tiles
    // of rows below k are skipped (wave-uniform); skipped terms are exact
    // zeros, so the result is bit-identical
    for (int32_t kt = nfull; kt < nk; ++kt) {
      const float* as = pipe(kt);
      const int kd = kt - nfull - 2 * wm;
      const int imin = kd < 0 ? 0 : kd;
      if (imin < 2) var_step_f32(as, as + C::SA, wm, wn, lane, imin, acc);
    }

    // epilogue: column sums of squares over this tile's 128 rows
    __syncthreads();
    double* red = reinterpret_cast<double*>(lds);  // [2][256]
#pragma unroll
    for (int jj = 0; jj < 2; ++jj) {
      const int cl = wn * 64 + jj * 32 + (lane & 31);
      double s = 0.0;
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) s += (double)acc[i][jj][r] * (double)acc[i][jj][r];
      s += __shfl_xor(s, 32);
      if ((lane >> 5) == 0) red[wm * VAR_BN + cl] = s;
    }
    __syncthreads();
    if (t < VAR_BN) {
      const int64_t col = col0 + t;
      if (col < m) part[(int64_t)rt * ldp + col] = red[t] + red[VAR_BN + t];
    }
  }
}

// ---------------------------------------------------------------------------
// Variance contraction, fp64, "ping-pong": TWO 256-thread workgroups per CU
// (__launch_bounds__(256, 2), 68 KiB of LDS each), so every SIMD holds one wave
// of each and one workgroup's barrier wait, pipeline fill and epilogue overlap
// the other's MFMAs.  The one-512-thread-workgroup-per-CU form (k_gp_var_f32's
// shape in fp64, removed in round 5) put both waves of a SIMD behind the same
// barrier every 16 k.
//   tile: 128 rows of L^-1 x 128 candidates, 2 x 2 waves of 64 x 64 outputs;
//   rows interleaved by 16-row sub-tiles (wave wm owns sub-tiles 2i + wm), so
//   in the diagonal block -- where (L^-1)^T is zero for k > row and the
//   all-zero sub-tiles are skipped -- the two wave rows of a workgroup skip
//   about equally (with contiguous halves the upper waves idle half of it
//   while the barrier holds the lower ones);
//   ring: 2 stages of 16 k (32 KiB), global_load_lds_dwordx4, 8 per wave per
//   stage; stage kt+1 is issued right after the barrier of step kt.
// Measured on MI355X, C2 shape (scripts/exp/var_probe.hip): 16.9 ms (0.83 of
// the fp64 peak) against 18.1 ms for the one-workgroup form; 0.88 without any global
// loads, 0.93 without the triangle (full K, no loads).
// Tickets and the part / mpart layouts: [RT][ldk] column partials per 128-row tile.
// ---------------------------------------------------------------------------
constexpr int VP_NT = 256, VP_BN = 128, VP_BK = 16, VP_ST = 2;
constexpr int VP_SA = VP_BK * VAR_BM, VP_STAGE = VP_SA + VP_BK * VP_BN;

// SPLIT: few candidate strips (survivor and threshold-set passes of the pruned
// scoring): the item count RT x CT is far below the chip's workgroup slots and
// each item is a long serial k loop, so items are split into chunks of kcs
// k-steps.  Item g (over all XCDs) -> strip ct, row tile rt, chunk kc (chunks
// of a strip in row-tile order); the raw 128 x 128 tile of L^-1 K*^T partial
// sums goes to vbuf[g], and k_var_split_red sums the chunks in order, then
// squares (deterministic).
__device__ __forceinline__ int32_t var_nk(int32_t K, int32_t rt) { return min(K, (rt + 1) * VAR_BM) / VP_BK; }

template <bool SPLIT>
__global__ __launch_bounds__(VP_NT, 2) void k_gp_var_pp(const double* __restrict__ AT, int64_t lda,
                                                        const double* __restrict__ B, int64_t ldb, int32_t K,
                                                        int32_t RT, int32_t CT, int64_t m,
                                                        int32_t* __restrict__ ticket, double* __restrict__ part,
                                                        int64_t ldp, const double* __restrict__ beta,
                                                        double* __restrict__ mpart, int32_t kcs, int32_t per_strip,
                                                        double* __restrict__ vbuf, int32_t S) {
  // one __shared__ object (see k_gp_var): ring, reduction buffer, ticket slot
  __shared__ __attribute__((aligned(16))) double lds[VP_ST * VP_STAGE + 4 * VP_BN + VAR_BM + 2];
  double* red = lds + VP_ST * VP_STAGE;  // [2][128] squares, [2][128] mean
  double* sbeta = red + 4 * VP_BN;        // beta of the item's 128 rows
  int32_t& s_item = *reinterpret_cast<int32_t*>(sbeta + VAR_BM);
  const int t = threadIdx.x, lane = t & 63;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const int wm = w >> 1, wn = w & 1;
  const int32_t xcd = blockIdx.x & 7;
  // stage image: A [16 k][128 rows], B [16 k][128 cols]; one glds wave-instruction
  // moves one k row (128 doubles): wave w moves A rows 4w..4w+3 and B rows 4w..4w+3
  auto issue = [&](int32_t row0, int64_t col0, int32_t k0, double* st) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int q = 4 * w + u;
      __builtin_amdgcn_global_load_lds(AT + (int64_t)(k0 + q) * lda + row0 + lane * 2,
                                       (__attribute__((address_space(3))) void*)(st + q * VAR_BM), 16, 0, 0);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int q = 4 * w + u;
      __builtin_amdgcn_global_load_lds(B + (int64_t)(k0 + q) * ldb + col0 + lane * 2,
                                       (__attribute__((address_space(3))) void*)(st + VP_SA + q * VP_BN), 16, 0, 0);
    }
  };
  const int32_t P = (RT + 1) / 2;
  for (;;) {
    if (t == 0) s_item = atomicAdd(&ticket[xcd], 1);
    __syncthreads();  // also: the previous item's epilogue is done with `red`
    const int32_t j = s_item;
    int32_t ct, rt, kt0, kt1, g = 0;
    int32_t rt2 = -1;   // the pair's second (short) row tile
    if constexpr (SPLIT) {
      g = j * 8 + xcd;
      if (g >= CT * per_strip) break;
      ct = g / per_strip;
      int32_t rem = g - ct * per_strip;
      rt = 0;
      for (;;) {
        const int32_t nc = (var_nk(K, rt) + kcs - 1) / kcs;
        if (rem < nc) break;
        rem -= nc;
        ++rt;
      }
      kt0 = rem * kcs;
      kt1 = min(var_nk(K, rt), kt0 + kcs);
    } else {
      // paired groups (as k_gp_var_h3): item = row tiles (RT - 1 - p, p) of one
      // strip, every item the same length; an XCD's workgroups take P pairs x S
      // strips at once, so a group shares each L^-1 stage through L2 (C2: FETCH
      // 41.1 -> 24.3 GB per launch against strip-major items, round 26.10-26.15
      // -> 25.99 ms; round 4)
      const int32_t G = j / (P * S), q = j % (P * S), p = q % P;
      ct = (G * S + q / P) * 8 + xcd;
      if (ct >= CT) break;  // uniform: every wave of the block leaves together
      rt = RT - 1 - p;
      rt2 = p != rt ? p : -1;
      kt0 = 0;
      kt1 = var_nk(K, rt);
    }
    for (;;) {   // the item's row tiles (its pair)
    const int64_t col0 = (int64_t)ct * VP_BN;
    const int32_t row0 = rt * VAR_BM;
    vd4 acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) acc[i][jj] = (vd4){0.0, 0.0, 0.0, 0.0};
    // beta of this row tile, staged for the epilogue beside stage 0 (its load
    // retires with stage 0's vmcnt wait; the previous epilogue's reads of
    // sbeta ended before the ticket barrier)
    if (!SPLIT && w == 0)  // 128 doubles = one glds wave-instruction, asynchronous like the ring
      __builtin_amdgcn_global_load_lds(beta + row0 + lane * 2, (__attribute__((address_space(3))) void*)sbeta, 16, 0,
                                       0);
    issue(row0, col0, kt0 * VP_BK, lds + (kt0 & 1) * VP_STAGE);
    const int32_t nfull = min(var_nk(K, rt), row0 / VP_BK);
    for (int32_t kt = kt0; kt < kt1; ++kt) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();  // stage kt landed everywhere; stage kt-1 fully read
      asm volatile("" ::: "memory");
      if (kt + 1 < kt1) issue(row0, col0, (kt + 1) * VP_BK, lds + ((kt + 1) & 1) * VP_STAGE);
      const double* as = lds + (kt & 1) * VP_STAGE;
      const double* bs = as + VP_SA;
      // diagonal block: sub-tile i (rows (2i + wm) * 16 ..) is all zero once
      // 16 kd >= (2i + wm + 1) * 16, i.e. for i < ceil((kd - wm) / 2); skipped
      // terms are exact zeros
      int imin = 0;
      if (kt >= nfull) {
        const int z = kt - nfull - wm;
        imin = z <= 0 ? 0 : (z + 1) >> 1;
      }
      if (imin < 4) {
#pragma unroll
        for (int ks = 0; ks < VP_BK / 4; ++ks) {
          const int kr = ks * 4 + (lane >> 4);
          double af[4], bf[4];
#pragma unroll
          for (int jj = 0; jj < 4; ++jj) bf[jj] = bs[kr * VP_BN + wn * 64 + jj * 16 + (lane & 15)];
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            if (i < imin) continue;
            af[i] = as[kr * VAR_BM + (2 * i + wm) * 16 + (lane & 15)];
#pragma unroll
            for (int jj = 0; jj < 4; ++jj)
              acc[i][jj] = __builtin_amdgcn_mfma_f64_16x16x4f64(af[i], bf[jj], acc[i][jj], 0, 0, 0);
          }
        }
      }
    }
    if constexpr (SPLIT) {   // the raw partial tile; k_var_split_red squares the chunk sums
      double* vt = vbuf + (int64_t)g * (VAR_BM * VP_BN);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int jj = 0; jj < 4; ++jj)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            vt[((2 * i + wm) * 16 + (lane >> 4) + 4 * r) * VP_BN + wn * 64 + jj * 16 + (lane & 15)] = acc[i][jj][r];
      break;   // to the next ticket, whose barrier orders the LDS ring's reuse
    }
    // epilogue: column sums of squares over the tile's 128 rows and the mean
    // partial sum_r V[r][c] beta_r (beta = L^-1 y)
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) {
      const int cl = wn * 64 + jj * 16 + (lane & 15);
      double s = 0.0, u = 0.0;
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const double v = acc[i][jj][r];
          s += v * v;
          u += v * sbeta[(2 * i + wm) * 16 + (lane >> 4) + 4 * r];
        }
      s += __shfl_xor(s, 16);
      s += __shfl_xor(s, 32);
      u += __shfl_xor(u, 16);
      u += __shfl_xor(u, 32);
      if ((lane >> 4) == 0) {
        red[wm * VP_BN + cl] = s;
        red[2 * VP_BN + wm * VP_BN + cl] = u;
      }
    }
    __syncthreads();
    if (t < VP_BN) {
      const int64_t col = col0 + t;
      if (col < m) {
        part[(int64_t)rt * ldp + col] = red[t] + red[VP_BN + t];
        mpart[(int64_t)rt * ldp + col] = red[2 * VP_BN + t] + red[3 * VP_BN + t];
      }
    }
    if (SPLIT || rt2 < 0) break;
    rt = rt2;
    rt2 = -1;
    kt1 = var_nk(K, rt);
    __syncthreads();   // red / sbeta read; the ring is reused by the next tile
    }
  }
}

// chunk sums of the split partial tiles -> part / mpart (k_gp_var_pp's epilogue);
// one 1024-thread workgroup per (row tile, strip): thread = (column, 16-row group),
// four chunk loads in flight per thread
__global__ __launch_bounds__(1024) void k_var_split_red(const double* __restrict__ vbuf, int32_t K, int32_t kcs,
                                                        int32_t per_strip, int64_t m, const double* __restrict__ beta,
                                                        double* __restrict__ part, double* __restrict__ mpart,
                                                        int64_t ldp) {
  __shared__ double red[2][8][VP_BN];
  const int32_t rt = blockIdx.x, ct = blockIdx.y;
  int32_t first = ct * per_strip;
  for (int32_t r = 0; r < rt; ++r) first += (var_nk(K, r) + kcs - 1) / kcs;
  const int32_t nc = (var_nk(K, rt) + kcs - 1) / kcs;
  const int t = threadIdx.x, c = t & (VP_BN - 1), h = t >> 7;   // column, 16-row group
  const double* vb = vbuf + (int64_t)first * VAR_BM * VP_BN + c;
  double s = 0.0, u = 0.0;
  for (int r = h * 16; r < h * 16 + 16; ++r) {
    const double* p = vb + r * VP_BN;
    double v0 = 0.0, v1 = 0.0, v2 = 0.0, v3 = 0.0;
    int32_t q = 0;
    for (; q + 4 <= nc; q += 4) {
      v0 += p[(int64_t)q * VAR_BM * VP_BN];
      v1 += p[(int64_t)(q + 1) * VAR_BM * VP_BN];
      v2 += p[(int64_t)(q + 2) * VAR_BM * VP_BN];
      v3 += p[(int64_t)(q + 3) * VAR_BM * VP_BN];
    }
    for (; q < nc; ++q) v0 += p[(int64_t)q * VAR_BM * VP_BN];
    const double v = (v0 + v1) + (v2 + v3);
    s += v * v;
    u += v * beta[rt * VAR_BM + r];
  }
  red[0][h][c] = s;
  red[1][h][c] = u;
  __syncthreads();
  const int64_t col = (int64_t)ct * VP_BN + c;
  if (h < 2 && col < m) {
    double a = 0.0;
#pragma unroll
    for (int g = 0; g < 8; ++g) a += red[h][g][c];
    (h == 0 ? part : mpart)[(int64_t)rt * ldp + col] = a;
  }
}

// ---------------------------------------------------------------------------
// Variance contraction, f16x3 ("h3"): fp32-class accuracy at the fp16 MFMA rate.
// Both operands are split once into fp16 planes, x * 2^e = hi + lo (hi = fp16(x 2^e),
// lo = fp16(x 2^e - hi): 22 significant bits), and each product is taken as
// hi*hi + hi*lo + lo*hi (lo*lo, ~2^-22 relative, dropped) by three
// v_mfma_f32_32x32x16_f16 into one f32 accumulator: 3 x 16 = 48 fp16-MFMA flops
// per algorithmic pair against 16 at the fp32 MFMA's 1/16 rate, i.e. 5.3x the
// fp32 MFMA's arithmetic rate.  The scales keep both operands inside fp16's
// normal range: K* (<= sf2) by 2^h3_kstar_exp(sf2), L^-1 by 2^(14 - ilogb max|L^-1|)
// (from the device-side max), so hi < 2^15 and lo's subnormal floor sits ~2^-40
// below the largest element.  The epilogue unscales the f32 column sums.
//
// Operands in HBM, "blocked" (round 3): each plane is cut into 256-row x 32-k
// blocks of 16 KiB, block (rb, kb) at element (rb * K/32 + kb) * 8192, and
// inside a block row r's 16-B chunk c sits at r * 32 + ((c ^ ((r >> 2) & 3)) << 3)
// -- exactly the LDS image the MFMA fragments read conflict-free
// (ds_read_b128 lane groups of the 32x32x16 layout), so a ring stage is two
// contiguous 16-KiB copies per operand, 1 KiB per global_load_lds.
//   A = L^-1 [row][k]: rows padded with zeros to a multiple of 256 (k_split_h3)
//   B = K*   [cand][k]: written blocked by k_gp_kstar<_Float16> (ldk % 256 == 0)
// Measured against the row-major 128 x 256-tile kernel it replaces
// (scripts/exp/h3_probe.hip, random operands, one MI355X): C3 shape 100.5 ->
// 89.6 ms, C2 shape 3.61 -> 3.13 ms.
// ---------------------------------------------------------------------------

// s_waitcnt vmcnt(N) (N < 64), lgkmcnt / expcnt left alone
template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
}

// one stage: this wave's two 1-KiB pieces of each 16-KiB block.  PART: 1 = A
// planes, 2 = B planes, 3 = both
template <int PART>
__device__ __forceinline__ void h3_issue(const _Float16* __restrict__ Ab, int64_t a_lo, const _Float16* __restrict__ Bb,
                                         int64_t b_lo, _Float16* st, int w, int lane) {
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int off = w * 1024 + u * 512;
    if constexpr (PART & 1) {
      __builtin_amdgcn_global_load_lds(Ab + off + lane * 8, (__attribute__((address_space(3))) void*)(st + off), 16,
                                       0, 0);
      __builtin_amdgcn_global_load_lds(Ab + a_lo + off + lane * 8,
                                       (__attribute__((address_space(3))) void*)(st + H3_BLK + off), 16, 0, 0);
    }
    if constexpr (PART & 2) {
      __builtin_amdgcn_global_load_lds(Bb + off + lane * 8,
                                       (__attribute__((address_space(3))) void*)(st + 2 * H3_BLK + off), 16, 0, 0);
      __builtin_amdgcn_global_load_lds(Bb + b_lo + off + lane * 8,
                                       (__attribute__((address_space(3))) void*)(st + 3 * H3_BLK + off), 16, 0, 0);
    }
  }
}

__device__ __forceinline__ vh8 h3_frag(const _Float16* plane, int r, int c) {
  return *reinterpret_cast<const vh8*>(plane + r * H3_BK + ((c ^ ((r >> 2) & 3)) << 3));
}

// one 32-k stage of a wave's 64 x 128 sub-tile (2 x 4 blocks of 32 x 32); mid()
// runs between the two k16 sub-steps (the B half of the next stage's refill
// goes there, behind this stage's first MFMAs)
template <class Mid>
__device__ __forceinline__ void var_step_h3(const _Float16* st, int wm, int wn, int lane, int imin, vf16 (&acc)[2][4],
                                            Mid&& mid) {
  const _Float16* ah = st;
  const _Float16* al = st + H3_BLK;
  const _Float16* bh = st + 2 * H3_BLK;
  const _Float16* bl = st + 3 * H3_BLK;
#pragma unroll
  for (int s = 0; s < H3_BK / 16; ++s) {
    if (s == 1) {
      __builtin_amdgcn_sched_barrier(0);
      mid();
      __builtin_amdgcn_sched_barrier(0);
    }
    const int c = 2 * s + (lane >> 5);
    vh8 fbh[4], fbl[4];
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) {
      const int r = wn * 128 + jj * 32 + (lane & 31);
      fbh[jj] = h3_frag(bh, r, c);
      fbl[jj] = h3_frag(bl, r, c);
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      if (i < imin) continue;
      const int r = wm * 64 + i * 32 + (lane & 31);
      const vh8 fah = h3_frag(ah, r, c), fal = h3_frag(al, r, c);
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) {
        acc[i][jj] = __builtin_amdgcn_mfma_f32_32x32x16_f16(fal, fbh[jj], acc[i][jj], 0, 0, 0);
        acc[i][jj] = __builtin_amdgcn_mfma_f32_32x32x16_f16(fah, fbl[jj], acc[i][jj], 0, 0, 0);
        acc[i][jj] = __builtin_amdgcn_mfma_f32_32x32x16_f16(fah, fbh[jj], acc[i][jj], 0, 0, 0);
      }
    }
  }
}

__device__ __forceinline__ int h3_linv_exp(const unsigned long long* amax_bits) {
  return H3_KSCALE_EXP - ilogb(__longlong_as_double((long long)*amax_bits));
}

// Persistent, one 512-thread workgroup per CU (the 128 KiB ring allows no
// more), per-XCD work tickets, 256 x 256 tiles: item (rt, ct) = rows
// [256 rt, +256) of L^-1 against candidates [256 ct, +256); its k loop stops
// at the diagonal.  Waves are 4 row groups x 2 column halves of 64 x 128; waves
// w and w + 4 share a SIMD and get row groups wm and 3 - wm, so the diagonal
// block's skipped 32-row blocks balance per SIMD.  A 2-slot ring: stage kt + 1
// is issued right after the barrier that retires stage kt - 1 (its A planes)
// and between stage kt's two k16 sub-steps (its B planes), and lands while
// stage kt's 48 MFMAs per wave run.  part[rt][col] gets the column partial
// sum_{r in tile} V[r][col]^2 (RT2 = rows / 256 of them).
//
// Item order ("paired groups"): an item is the row-tile pair (RT2 - 1 - p, p)
// of one strip (every pair the same length, RT2 + 1 tiles of k), and an XCD's
// W workgroups take W items at once as P pairs x S strips (P = ceil(RT2 / 2),
// S = W / P).  Equal lengths keep a group in step, so the S workgroups of a
// pair read each L^-1 stage at about the same time (one fetch from the
// Infinity Cache, S - 1 L2 hits) and the P workgroups of a strip share its
// long-tile K* stages -- where strip-major items (round 3) read the whole
// L^-1 triangle per strip from the Infinity Cache.
__global__ __launch_bounds__(512, 2) void k_gp_var_h3(const _Float16* __restrict__ A, int64_t a_lo,
                                                      const _Float16* __restrict__ B, int64_t b_lo, int32_t K,
                                                      int32_t RT2, int32_t CT, int64_t m, int32_t* __restrict__ ticket,
                                                      double* __restrict__ part, int64_t ldp,
                                                      const unsigned long long* __restrict__ amax_bits, int32_t kexp,
                                                      int32_t S) {
  __shared__ __attribute__((aligned(16))) _Float16 lds[H3_NS * H3_STAGE + 8];
  int32_t& s_item = *reinterpret_cast<int32_t*>(lds + H3_NS * H3_STAGE);
  const int t = threadIdx.x, lane = t & 63;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const int wm = w < 4 ? w : 7 - w, wn = w < 4 ? 0 : 1;
  const int32_t xcd = blockIdx.x & 7;
  const int32_t KB = K / H3_BK;
  const double unscale2 = __builtin_ldexp(1.0, -2 * (h3_linv_exp(amax_bits) + kexp));

  const int32_t P = (RT2 + 1) / 2;
  for (;;) {
    if (t == 0) s_item = atomicAdd(&ticket[xcd], 1);
    __syncthreads();
    const int32_t j = s_item;
    const int32_t G = j / (P * S), q = j % (P * S), p = q % P;
    const int32_t ct = (G * S + q / P) * 8 + xcd;
    const int32_t rts[2] = {RT2 - 1 - p, p};
    const int32_t nrt = rts[1] == rts[0] ? 1 : 2;
    if (ct >= CT) break;
    for (int32_t ri = 0; ri < nrt; ++ri) {
    if (ri > 0) __syncthreads();   // the previous tile's reduction buffer (LDS ring) fully read
    const int32_t rt = rts[ri];
    const int32_t row0 = rt * H3_BM;
    const int32_t nk = min(K, row0 + H3_BM) / H3_BK;
    const _Float16* Ab = A + (int64_t)rt * KB * H3_BLK;
    const _Float16* Bb = B + (int64_t)ct * KB * H3_BLK;

    vf16 acc[2][4];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int jj = 0; jj < 4; ++jj)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[i][jj][r] = 0.0f;

    // rev (the pair's second, short tile): its k stages in descending
    // order.  The strip's P workgroups then read K* stage t (long tiles) or
    // RT2 - t (short tiles, reversed) at step t of their items -- two stages
    // per step across the strip instead of up to P -- so the L2 serves the
    // rest.  (Ascending, each second tile restarted at stage 0 while the
    // others were far ahead: 344 GB fetched per C3 launch for 32 GB of K*.)
    const bool rev = ri > 0;
    auto ktof = [&](int32_t u) -> int32_t { return rev ? nk - 1 - u : u; };
    h3_issue<3>(Ab + (int64_t)ktof(0) * H3_BLK, a_lo, Bb + (int64_t)ktof(0) * H3_BLK, b_lo, lds, w, lane);
    auto pipe = [&](int32_t u) -> const _Float16* {
      wait_vmcnt<0>();
      __builtin_amdgcn_s_barrier();   // step u landed everywhere; step u - 1 fully read
      asm volatile("" ::: "memory");
      if (u + 1 < nk)
        h3_issue<1>(Ab + (int64_t)ktof(u + 1) * H3_BLK, a_lo, nullptr, 0, lds + ((u + 1) & 1) * H3_STAGE, w, lane);
      return lds + (u & 1) * H3_STAGE;
    };
    auto refill_b = [&](int32_t u) {
      return [&, u]() {
        if (u + 1 < nk)
          h3_issue<2>(nullptr, 0, Bb + (int64_t)ktof(u + 1) * H3_BLK, b_lo, lds + ((u + 1) & 1) * H3_STAGE, w, lane);
      };
    };
    const int32_t nfull = min(nk, row0 / H3_BK);
    // (two plain loops per order: one loop with the full / diagonal test inside
    // spilled 236 VGPRs and ran 3x slower)
    auto diag_step = [&](int32_t u) {
      const _Float16* st = pipe(u);
      const int kd = ktof(u) - nfull - 2 * wm;   // 32-row blocks of this wave entirely above the diagonal
      const int imin = kd < 0 ? 0 : kd;
      if (imin < 2) var_step_h3(st, wm, wn, lane, imin, acc, refill_b(u));
      else refill_b(u)();
    };
    if (!rev) {
      for (int32_t u = 0; u < nfull; ++u) var_step_h3(pipe(u), wm, wn, lane, 0, acc, refill_b(u));
      for (int32_t u = nfull; u < nk; ++u) diag_step(u);
    } else {
      for (int32_t u = 0; u < nk - nfull; ++u) diag_step(u);
      for (int32_t u = nk - nfull; u < nk; ++u) var_step_h3(pipe(u), wm, wn, lane, 0, acc, refill_b(u));
    }

    __syncthreads();
    double* red = reinterpret_cast<double*>(lds);  // [4][256]
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) {
      const int cl = wn * 128 + jj * 32 + (lane & 31);
      double s = 0.0;
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) s += (double)acc[i][jj][r] * (double)acc[i][jj][r];
      s += __shfl_xor(s, 32);
      if ((lane >> 5) == 0) red[wm * H3_BN + cl] = s;
    }
    __syncthreads();
    if (t < H3_BN) {
      const int64_t col = (int64_t)ct * H3_BN + t;
      if (col < m)
        part[(int64_t)rt * ldp + col] = ((red[t] + red[H3_BN + t]) + (red[2 * H3_BN + t] + red[3 * H3_BN + t])) * unscale2;
    }
    }
  }
}

// max |x| over cnt doubles into *out (as bits: non-negative doubles order like their bits)
__global__ __launch_bounds__(256) void k_absmax(const double* __restrict__ x, int64_t cnt,
                                                unsigned long long* __restrict__ out) {
  fit_prio_g();
  double v = 0.0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < cnt; i += (int64_t)gridDim.x * blockDim.x)
    v = fmax(v, fabs(x[i]));
  for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o));
  __shared__ double red[4];
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    v = fmax(fmax(red[0], red[1]), fmax(red[2], red[3]));
    atomicMax(out, (unsigned long long)__double_as_longlong(v));
  }
}

// L^-1 [row][k] (n x n fp64) -> scaled hi / lo planes in the blocked layout,
// rows padded with zeros to n256 = n rounded up to 256 (one element per thread;
// the lo plane n256 * n elements after the hi plane)
__global__ void k_split_h3(const double* __restrict__ x, int32_t n, int32_t n256,
                           const unsigned long long* __restrict__ amax_bits, _Float16* __restrict__ dst) {
  fit_prio_g();
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)n256 * n) return;
  const int64_t r = i / n;
  const int32_t k = (int32_t)(i - r * n);
  const double xs = r < n ? __builtin_ldexp(x[i], h3_linv_exp(amax_bits)) : 0.0;
  const _Float16 hi = (_Float16)(float)xs;
  const int64_t o = h3_blk_off(r, k, n);
  dst[o] = hi;
  dst[(int64_t)n256 * n + o] = (_Float16)(float)(xs - (double)hi);
}

int launch_split_h3(ut_ctx* c, const double* Linv, int32_t n, _Float16* dst) {
  const int64_t cnt = (int64_t)n * n;
  const int32_t n256 = ((n + H3_BM - 1) / H3_BM) * H3_BM;
  unsigned long long* amax = reinterpret_cast<unsigned long long*>(c->gp_ctr + 16);
  UT_HIP(c, hipMemsetAsync(amax, 0, sizeof(unsigned long long), c->stream));
  hipLaunchKernelGGL(k_absmax, dim3(1024), dim3(256), 0, c->stream, Linv, cnt, amax);
  hipLaunchKernelGGL(k_split_h3, dim3(grid1((int64_t)n256 * n, 256)), dim3(256), 0, c->stream, Linv, n, n256, amax,
                     dst);
  UT_LAUNCH_CHECK(c);
  return 0;
}

int launch_gemm_var(ut_ctx* c, int prec, const void* LinvT, int64_t lda, const void* kst, int64_t ldk, int32_t npad,
                    int64_t m, double* part, const double* beta, double* mpart) {
  const bool fp32 = prec != 64;
  UT_CHECK(c, prec == 64 || prec == 32 || prec == 16, UT_EINVAL, "gemm_var: bad precision");
  UT_CHECK(c, (beta != nullptr) == !fp32 && (mpart != nullptr) == !fp32, UT_EINVAL,
           "gemm_var: the mean partial is taken here in fp64 mode (only)");
  UT_CHECK(c, npad % VAR_BM == 0 && ldk % VAR_BN == 0 && ldk >= m, UT_EINVAL, "gemm_var: bad padding");
  const int32_t RT = npad / VAR_BM;
  const int32_t CT = (int32_t)((m + VAR_BN - 1) / VAR_BN);
  const int64_t items = (int64_t)RT * CT;
  // one block per CU (the 144 KiB LDS ring allows no more), a multiple of 8 so
  // every XCD group has workers; never more blocks than work items
  int32_t nb = (c->n_cu / 8) * 8;
  if (items < nb) nb = (int32_t)(((items + 7) / 8) * 8);
  UT_HIP(c, hipMemsetAsync(c->gp_ctr, 0, sizeof(int32_t) * 8, c->stream));
  if (prec == 16) {  // LinvT / kst: the blocked hi / lo planes of L^-1 and K* (see k_gp_var_h3)
    UT_CHECK(c, ldk % H3_BN == 0, UT_EINVAL, "gemm_var: h3 needs 256-candidate padding");
    const int32_t n256 = ((npad + H3_BM - 1) / H3_BM) * H3_BM;
    const int32_t RT2 = n256 / H3_BM, CT2 = (int32_t)(ldk / H3_BN);
    const int64_t items2 = (int64_t)RT2 * CT2;
    int32_t nb2 = (c->n_cu / 8) * 8;
    if (items2 < nb2) nb2 = (int32_t)(((items2 + 7) / 8) * 8);
    const unsigned long long* amax = reinterpret_cast<const unsigned long long*>(c->gp_ctr + 16);
    // paired groups: S strips per group so that P x S items fill an XCD's workgroups
    const int32_t P2 = (RT2 + 1) / 2, W = nb2 / 8;
    const int32_t S2 = W / P2 > 1 ? W / P2 : 1;
    hipLaunchKernelGGL(k_gp_var_h3, dim3(nb2), dim3(512), 0, c->stream, (const _Float16*)LinvT, (int64_t)n256 * npad,
                       (const _Float16*)kst, ldk * (int64_t)npad, npad, RT2, (int32_t)((m + H3_BN - 1) / H3_BN), m,
                       c->gp_ctr, part, ldk, amax, h3_kstar_exp(c->gp_sf2), S2);
  }
  else if (fp32)
    hipLaunchKernelGGL(k_gp_var_f32, dim3(nb), dim3(V_NT), 0, c->stream, (const float*)LinvT, lda,
                       (const float*)kst, ldk, npad, RT, CT, m, c->gp_ctr, part, ldk);
  else {
    // two workgroups per CU on 128-candidate column tiles
    const int32_t CTp = (int32_t)((m + VP_BN - 1) / VP_BN);
    const int64_t items_p = (int64_t)RT * CTp;
    const int32_t slots = 2 * (c->n_cu / 8) * 8;
    int32_t nbp = slots;
    // few strips (pruned scoring's survivor / threshold passes): split the k loops
    int64_t steps = 0;   // k-steps per strip
    for (int32_t r = 0; r < RT; ++r) steps += min(npad, (r + 1) * VAR_BM) / VP_BK;
    if (c->var_split && items_p < slots && steps >= 64) {
      int32_t kcs = (int32_t)((steps * CTp + 2 * slots - 1) / (2 * slots));   // ~2 items per workgroup slot
      kcs = kcs < 8 ? 8 : kcs;
      int32_t per_strip = 0;
      for (int32_t r = 0; r < RT; ++r) per_strip += (min(npad, (r + 1) * VAR_BM) / VP_BK + kcs - 1) / kcs;
      const int64_t items_s = (int64_t)per_strip * CTp;
      int rc;
      if ((rc = ensure(c, c->var_vbuf, (size_t)items_s * VAR_BM * VP_BN))) return rc;
      if (items_s < nbp) nbp = (int32_t)(((items_s + 7) / 8) * 8);
      hipLaunchKernelGGL(k_gp_var_pp<true>, dim3(nbp), dim3(VP_NT), 0, c->stream, (const double*)LinvT, lda,
                         (const double*)kst, ldk, npad, RT, CTp, m, c->gp_ctr, part, ldk, beta, mpart, kcs, per_strip,
                         c->var_vbuf.p, 1);
      hipLaunchKernelGGL(k_var_split_red, dim3(RT, CTp), dim3(1024), 0, c->stream, c->var_vbuf.p, npad, kcs, per_strip,
                         m, beta, part, mpart, ldk);
    } else {
      if (items_p < nbp) nbp = (int32_t)(((items_p + 7) / 8) * 8);
      const int32_t Pp = (RT + 1) / 2, Wp = nbp / 8;
      const int32_t Sp = Wp / Pp > 1 ? Wp / Pp : 1;
      hipLaunchKernelGGL(k_gp_var_pp<false>, dim3(nbp), dim3(VP_NT), 0, c->stream, (const double*)LinvT, lda,
                         (const double*)kst, ldk, npad, RT, CTp, m, c->gp_ctr, part, ldk, beta, mpart, 0, 0, nullptr,
                         Sp);
    }
  }
  UT_LAUNCH_CHECK(c);
  return 0;
}

// dst[c][r] = src[r][c] (n x n, n % 64 == 0), optionally also as fp32
__global__ __launch_bounds__(256) void k_transpose(const double* __restrict__ src, int32_t n, double* __restrict__ dst,
                                                   float* __restrict__ dst_f) {
  fit_prio_g();
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
