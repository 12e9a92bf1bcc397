// gp_kq.hip -- K* for precision-8 fits: the distance contraction on the int8
// MFMA ("Ozaki" digits, exact int32 sums), the exp epilogue on the VALU beside it.
// (Round 5 measured it alone: 2.6-2.7 + 0.33 ms against 3.1-3.3 for
// k_gp_kstar<int8_t>, and did not keep it; round 6 runs it beside the round's
// hash, which is integer VALU work the int8 MFMA issues beside, where the f64
// MFMA does not: C2 ~1 % per round.  Numeric fits only -- at C3's categorical
// HPL-64 fit it was 43 against 28.5 ms of K* -- and only the digit-plane
// variant without the mean (the variance epilogue has it) is instantiated.
// UT_KSTAR_Q=0 keeps k_gp_kstar<int8_t>.)
//
// k_gp_kstar (gp_gemm.hip) contracts C = Xs U' on the fp64 MFMA, and on gfx950
// an f64 MFMA holds its SIMD's VALU issue for its whole duration: the exp
// epilogue of one workgroup cannot run under the MFMAs of the other, so that
// kernel costs MFMA + epilogue (scripts/exp/coissue_roles.hip: f64 MFMA 4.29 ms
// and f64 VALU 1.28 ms alone, 5.56 together; i8 MFMA 1.17 ms beside the same
// VALU stream 1.59).  Here both operands are cut into six balanced 8-bit digit
// planes, as the int8 variance contraction does (gp_i8.hip), and the products
// run on v_mfma_i32_32x32x32_i8, whose waves leave the VALU to the other
// workgroup's epilogue:
//
//   x_rk = Xs^T[k][r] (t units: times 256 / ln 2) 2^-ea     (one ea for the fit)
//   u_kc = U'[k][c] 2^-eb_c                                   (one eb per candidate)
//   T_g  = sum_k sum_{p+q=g} a_p b_q   (g = 2..7, exact int32 for K < 2^14 / 6)
//   C_rc = 2^(ea + eb_c - 16) (T_2 + 2^-8 (T_3 + ... + 2^-8 T_7))
//
// (K <= 96: the pairs 256 T_2 + T_3, 256 T_4 + T_5, 256 T_6 + T_7 are exact
// int32 too, and C = 2^(ea + eb_c - 24) (U_23 + 2^-16 (U_45 + 2^-16 U_67)):
// three conversions instead of six.)  The digits' rounding (2^-49 of each
// operand's scale) and the dropped pairs p + q >= 8 leave |C - C^| below
// 2^-46 K 2^(ea + eb_c) -- the size of the fp64 contraction's own rounding
// (K 2^-53 |x| |u|), so k* = sf2 exp2((C - |x|^2/2 - |u|^2/2) / 256) keeps the
// fp64 tier's accuracy.  The epilogue is k_gp_kstar's: exp and K* as six
// digit planes for the int8 variance (TS = int8_t).  The template also holds
// the round-5 variants (MU: the mean partial sum_r alpha_r k*_r; TS = double:
// fp64 rows; CAT: the ENUM / BOOL one-hot blocks through the same MFMA as an
// int32 match count), which the library no longer instantiates.
//
// Tiles: 64 training rows x 64 candidates per 256-thread workgroup, two per
// CU; waves 2 x 2 of 32 x 32 (one MFMA output tile, six group accumulators);
// stages of 32 k: 6 A + 6 B planes of 2 KiB each in a 3-slot glds ring; each
// XCD's items dealt round-robin to its workgroups (no ticket atomics).
#include "ut_internal.h"

namespace ut {

constexpr int Q_BM = 64, Q_BN = 64, Q_NT = 256;
constexpr int Q_PL = Q_BM * 32;              // one plane's 32-k piece of a tile (2 KiB)
constexpr int Q_STAGE = 2 * I8_S * Q_PL;     // 24 KiB (a categorical stage: 2 x 8 KiB)
constexpr int Q_PAIR_MAX_K = 96;             // 256 |T_6| + |T_7| < 2^31 (5 and 6 pairs of 2^14)

// ---------------------------------------------------------------------------
// operands: digit planes [6][K32][rows][32 B] (i8_off layout), K32 = ceil(K / 32)
// ---------------------------------------------------------------------------
// max |x| of the K* training operand -> amax (u64 bit pattern; |x| >= 0 orders as an integer)
__global__ __launch_bounds__(256) void k_q_absmax(const double* __restrict__ x, int64_t cnt,
                                                  unsigned long long* __restrict__ amax) {
  double mx = 0.0;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < cnt; e += (int64_t)gridDim.x * 256)
    mx = fmax(mx, fabs(x[e]));
  for (int o = 32; o > 0; o >>= 1) mx = fmax(mx, __shfl_xor(mx, o));
  if ((threadIdx.x & 63) == 0 && mx > 0.0) atomicMax(amax, (unsigned long long)__double_as_longlong(mx));
}

__device__ __forceinline__ int32_t q_exp(double mx) { return mx > 0.0 ? ilogb(mx / 0.49) + 1 : 0; }

// the digits of 32 consecutive k of one row / candidate (v[k] * 2^-e): six
// planes x 32 bytes, stored as two 16-byte chunks each (swizzled by row bit 3)
__device__ __forceinline__ void q_store_piece(const double (&v)[32], int32_t e, int8_t* __restrict__ base,
                                              int64_t plane, int64_t r) {
  uint32_t pw[I8_S][8];
#pragma unroll
  for (int g = 0; g < 8; ++g) {
    uint32_t lo[4], hi[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const uint64_t b = i8_biased(__builtin_ldexp(v[4 * g + u], -e));
      lo[u] = (uint32_t)b;
      hi[u] = (uint32_t)(b >> 32);
    }
    uint32_t pl[I8_S];
    i8_planes(lo, hi, pl);
#pragma unroll
    for (int p = 0; p < I8_S; ++p) pw[p][g] = pl[p];
  }
  const int sw = (int)((r >> 3) & 1);
#pragma unroll
  for (int p = 0; p < I8_S; ++p) {
    int8_t* d = base + p * plane;
    *reinterpret_cast<uint4*>(d + (sw << 4)) = make_uint4(pw[p][0], pw[p][1], pw[p][2], pw[p][3]);
    *reinterpret_cast<uint4*>(d + ((sw ^ 1) << 4)) = make_uint4(pw[p][4], pw[p][5], pw[p][6], pw[p][7]);
  }
}

// training rows: XsT [K][npad] -> Xd; ea from amax (stored in *ea_out)
__global__ __launch_bounds__(256) void k_q_split_x(const double* __restrict__ XsT, int32_t K, int32_t npad,
                                                   int32_t K32, const unsigned long long* __restrict__ amax,
                                                   int8_t* __restrict__ Xd, int64_t* __restrict__ ea_out) {
  const int32_t r = blockIdx.x * 256 + threadIdx.x;
  const int32_t ea = q_exp(__longlong_as_double((long long)*amax));
  if (r == 0) ea_out[0] = ea;
  if (r >= npad) return;
  const int64_t plane = (int64_t)K32 * 32 * npad;
  for (int32_t kb = 0; kb < K32; ++kb) {
    double v[32];
#pragma unroll
    for (int u = 0; u < 32; ++u) {
      const int32_t k = kb * 32 + u;
      v[u] = k < K ? XsT[(int64_t)k * npad + r] : 0.0;
    }
    q_store_piece(v, ea, Xd + ((int64_t)kb * npad + r) * 32, plane, r);
  }
}

// candidates: U' [K][ldk] -> Ud; per-candidate eb and the column scale
// 2^(ea + eb + shift) (shift -24 with the paired groups, -16 without)
__global__ __launch_bounds__(256) void k_q_split_u(const double* __restrict__ U, int32_t K, int64_t ldk, int32_t K32,
                                                   const int64_t* __restrict__ ea_in, int32_t shift,
                                                   int8_t* __restrict__ Ud, double* __restrict__ scol) {
  const int64_t c = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (c >= ldk) return;
  double mx = 0.0;
  for (int32_t k = 0; k < K; ++k) mx = fmax(mx, fabs(U[(int64_t)k * ldk + c]));
  const int32_t eb = q_exp(mx);
  scol[c] = __builtin_ldexp(1.0, (int32_t)ea_in[0] + eb + shift);
  const int64_t plane = (int64_t)K32 * 32 * ldk;
  for (int32_t kb = 0; kb < K32; ++kb) {
    double v[32];
#pragma unroll
    for (int u = 0; u < 32; ++u) {
      const int32_t k = kb * 32 + u;
      v[u] = k < K ? U[(int64_t)k * ldk + c] : 0.0;
    }
    q_store_piece(v, eb, Ud + ((int64_t)kb * ldk + c) * 32, plane, c);
  }
}

// s_waitcnt vmcnt(n) lgkmcnt(0) for a run-time n (uniform), clamped to 63
__device__ __forceinline__ void vm_wait_n(int32_t n) {
  n = n < 0 ? 0 : (n > 63 ? 63 : n);
  switch (n) {
#define UT_VMW(N) \
  case N: asm volatile("s_waitcnt vmcnt(" #N ") lgkmcnt(0)" ::: "memory"); break;
    UT_VMW(0) UT_VMW(1) UT_VMW(2) UT_VMW(3) UT_VMW(4) UT_VMW(5) UT_VMW(6) UT_VMW(7) UT_VMW(8) UT_VMW(9) UT_VMW(10)
    UT_VMW(11) UT_VMW(12) UT_VMW(13) UT_VMW(14) UT_VMW(15) UT_VMW(16) UT_VMW(17) UT_VMW(18) UT_VMW(19) UT_VMW(20)
    UT_VMW(21) UT_VMW(22) UT_VMW(23) UT_VMW(24) UT_VMW(25) UT_VMW(26) UT_VMW(27) UT_VMW(28) UT_VMW(29) UT_VMW(30)
    UT_VMW(31) UT_VMW(32) UT_VMW(33) UT_VMW(34) UT_VMW(35) UT_VMW(36) UT_VMW(37) UT_VMW(38) UT_VMW(39) UT_VMW(40)
    UT_VMW(41) UT_VMW(42) UT_VMW(43) UT_VMW(44) UT_VMW(45) UT_VMW(46) UT_VMW(47) UT_VMW(48) UT_VMW(49) UT_VMW(50)
    UT_VMW(51) UT_VMW(52) UT_VMW(53) UT_VMW(54) UT_VMW(55) UT_VMW(56) UT_VMW(57) UT_VMW(58) UT_VMW(59) UT_VMW(60)
    UT_VMW(61) UT_VMW(62) UT_VMW(63)
#undef UT_VMW
  }
}

// a categorical stage's loads into an LDS ring slot: 64 code rows of 128 B for
// A and B, 8 pieces of 1 KiB each; wave w moves pieces w + 4u (u < 4)
__device__ __forceinline__ void q_issue_cat(const int8_t* __restrict__ acat, const int8_t* __restrict__ bcat,
                                            int32_t npad, int64_t ldk, int w, int lane, int32_t row0, int64_t col0,
                                            int32_t s2, int8_t* st) {
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int q = w + 4 * u;        // 0..15: A pieces 0..7, B pieces 8..15
    const bool isb = q >= 8;
    const int qq = q & 7;
    const int r = 8 * qq + (lane >> 3);
    const int cch = (lane & 7) ^ (r & 7);   // the source chunk that lands at position lane & 7
    const int8_t* src = isb ? bcat + ((int64_t)s2 * ldk + col0 + r) * 128 + cch * 16
                            : acat + ((int64_t)s2 * npad + row0 + r) * 128 + cch * 16;
    __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)(st + (isb ? 8192 : 0) + qq * 1024),
                                     16, 0, 0);
  }
}

// an item's epilogue operands (512 B each: waves 0..3 load xnorm, alpha, cnorm, scol)
template <bool MU>
__device__ __forceinline__ void q_issue_ops(const double* __restrict__ xnorm, const double* __restrict__ alpha,
                                            const double* __restrict__ cnorm, const double* __restrict__ scol, int w,
                                            int lane, int32_t row0, int64_t col0, double* ops) {
  if (lane < 32 && (MU || w != 1)) {
    const double* src = w == 0 ? xnorm + row0 : (w == 1 ? alpha + row0 : (w == 2 ? cnorm + col0 : scol + col0));
    __builtin_amdgcn_global_load_lds(src + lane * 2, (__attribute__((address_space(3))) void*)(ops + w * Q_BM), 16, 0,
                                     0);
  }
}

// ---------------------------------------------------------------------------
// the contraction + epilogue
// ---------------------------------------------------------------------------
template <typename TS, bool MU, bool CAT, bool PAIR>
__global__ __launch_bounds__(Q_NT, 2) void k_gp_kstar_q(
    const int8_t* __restrict__ Xd, int32_t npad, const int8_t* __restrict__ Ud, int64_t ldk, int32_t K32,
    const double* __restrict__ scol, int32_t RT, int32_t CT, const double* __restrict__ xnorm,
    const double* __restrict__ cnorm, const double* __restrict__ alpha, double sf2, int32_t n, int64_t m,
    TS* __restrict__ kst, double* __restrict__ part, double kscale, int64_t lo_off,
    int32_t store_rt, double* __restrict__ part2, const int8_t* __restrict__ acat, const int8_t* __restrict__ bcat,
    int32_t nkc, double cat_c0, double cat_c1) {
  constexpr bool I8 = sizeof(TS) == 1;
  constexpr int OPS = 2 * Q_BM + 2 * Q_BN;              // one item's epilogue operands (doubles)
  // a 3-slot ring (80 KiB in all: two workgroups per CU)
  __shared__ __attribute__((aligned(16))) int8_t lds[3 * Q_STAGE + 8 * (EXP_TAB + 3 * OPS)];
  double* etab = reinterpret_cast<double*>(lds + 3 * Q_STAGE);
  // three buffers (items k mod 3) of [rx 64 | ra 64 | cn 64 | cs 64]:
  //   rx training half-norms (t units; -1e300 past n), ra alpha (I8: / kscale),
  //   cn candidate half-norms (-1e300 past m), cs column scales
  double* ops0 = etab + EXP_TAB;
  const int t = threadIdx.x, lane = t & 63;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const int wm = w >> 1, wn = w & 1;
  const int32_t xcd = blockIdx.x & 7;
  if (t < EXP_TAB) etab[t] = (sf2 * exp2((double)t / EXP_TAB)) * (I8 ? kscale : 1.0);
  const double ikscale = 1.0 / kscale;
  const int64_t xplane = (int64_t)K32 * 32 * npad, uplane = (int64_t)K32 * 32 * ldk;
  const int32_t ncs = CAT ? nkc : 0;
  const int32_t ntot = ncs + K32;
  const bool want2 = !I8 && MU && part2 != nullptr;
  // fragment offsets: A row ra_ = wm*32 + (l & 31), B column cb = wn*32 + (l & 31), 16-B chunk l >> 5
  const int c = lane >> 5;
  const int ra_ = wm * 32 + (lane & 31), cb = wn * 32 + (lane & 31);
  const int aoff = ra_ * 32 + ((c ^ ((ra_ >> 3) & 1)) << 4);
  const int boff = I8_S * Q_PL + cb * 32 + ((c ^ ((cb >> 3) & 1)) << 4);

  // Items: XCD x's strips (ct = x mod 8), each strip's row tiles in turn, dealt
  // round-robin to the XCD's W workgroups (equal items: no ticket atomic, whose
  // return would drain this wave's stores every item).  The items' stages form
  // one stream, g = k ntot + s for item k, issued two stages ahead into a
  // 3-slot ring (the next items' first stages and epilogue operands load under
  // the current item's MFMAs and epilogue).  s_waitcnt vmcnt counts loads,
  // stores and LDS-DMA together in issue order (MI355X_MICROARCH.md), so stage
  // g waits for all but the vector-memory instructions this wave issued after
  // g's loads (counted below; the uncounted MU partial stores only add to the
  // younger ones: the wait is then longer, never short).
  const int32_t W = gridDim.x >> 3, b0 = blockIdx.x >> 3;
  const int32_t Wq = W / RT, Wr = W % RT;    // an item's successor: W items on
  const int ops_n = (MU || w != 1) ? 1 : 0;   // this wave's epilogue-operand load per item
  int32_t cnt = 0;                           // vector-memory instructions issued (counted ones)
  int32_t at0 = 0, at1 = 0, at2 = 0;         // cnt just after stage g's loads, slot g mod 3
  // this wave's digit-stage pieces u = 0..5: piece q = w + 4u is half q & 1 of
  // plane (q >> 1) of A (u < 3) or of B (plane (q >> 1) - 6): the plane and
  // half offsets of the source and of the LDS image, fixed per wave
  int64_t so[6];
  int32_t ldo[6];
#pragma unroll
  for (int u = 0; u < 6; ++u) {
    const int q = w + 4 * u, h = q & 1;
    so[u] = (int64_t)((q >> 1) % I8_S) * (u < 3 ? xplane : uplane) + h * 1024 + lane * 16;
    ldo[u] = (q >> 1) * Q_PL + h * 1024;
  }
  // the issue cursor: stage is_ of item (row tile irt, column tile ict), ring
  // slot isl, operand buffer iob; iok false past the last item
  int32_t irt = b0 % RT, ictq = b0 / RT, is_ = 0, isl = 0, iob = 0;
  bool iok = ictq * 8 + xcd < CT;
#define UT_KQ_ISSUE()                                                                                            \
  do {                                                                                                          \
    if (iok) {                                                                                                  \
      const int32_t r0_ = irt * Q_BM;                                                                            \
      const int64_t c0_ = (int64_t)(ictq * 8 + xcd) * Q_BN;                                                      \
      int8_t* st_ = lds + isl * Q_STAGE;                                                                         \
      if (CAT && is_ < ncs) {                                                                                    \
        q_issue_cat(acat, bcat, npad, ldk, w, lane, r0_, c0_, is_, st_);                                         \
        cnt += 4;                                                                                               \
      } else {                                                                                                  \
        const int32_t kb_ = is_ - ncs;                                                                           \
        const int8_t* ab_ = Xd + ((int64_t)kb_ * npad + r0_) * 32;                                              \
        const int8_t* bb_ = Ud + ((int64_t)kb_ * ldk + c0_) * 32;                                               \
        _Pragma("unroll") for (int u = 0; u < 6; ++u)                                                           \
          __builtin_amdgcn_global_load_lds((u < 3 ? ab_ : bb_) + so[u],                                         \
                                           (__attribute__((address_space(3))) void*)(st_ + ldo[u]), 16, 0, 0);  \
        cnt += 6;                                                                                               \
      }                                                                                                         \
      if (is_ == 0) {                                                                                           \
        q_issue_ops<MU>(xnorm, alpha, cnorm, scol, w, lane, r0_, c0_, ops0 + iob * OPS);                        \
        cnt += ops_n;                                                                                           \
      }                                                                                                         \
      if (isl == 0) at0 = cnt;                                                                                  \
      else if (isl == 1) at1 = cnt;                                                                             \
      else at2 = cnt;                                                                                           \
      isl = isl == 2 ? 0 : isl + 1;                                                                             \
      if (++is_ == ntot) {                                                                                      \
        is_ = 0;                                                                                                \
        iob = iob == 2 ? 0 : iob + 1;                                                                           \
        irt += Wr;                                                                                              \
        ictq += Wq;                                                                                             \
        if (irt >= RT) {                                                                                        \
          irt -= RT;                                                                                            \
          ++ictq;                                                                                               \
        }                                                                                                       \
        iok = ictq * 8 + xcd < CT;                                                                              \
      }                                                                                                         \
    }                                                                                                           \
  } while (0)
  __syncthreads();   // (the exp table)
  if (!iok) return;   // (uniform: no item)
  UT_KQ_ISSUE();
  UT_KQ_ISSUE();
  // the consumer: item (row tile crt, column tile cctq), stage slot csl, operand buffer cob
  int32_t crt = b0 % RT, cctq = b0 / RT, csl = 0, cob = 0;
  for (;;) {
    const int32_t row0 = crt * Q_BM;
    const int64_t col0 = (int64_t)(cctq * 8 + xcd) * Q_BN;
    double* ops = ops0 + cob * OPS;
    double* rx = ops;
    double* ra = ops + Q_BM;
    double* cn = ops + 2 * Q_BM;
    double* cs = cn + Q_BN;
    const int32_t rt = crt;
    i8v16 acc[I8_S], iacc;
    if (K32 == 0) {
#pragma unroll
      for (int g = 0; g < I8_S; ++g)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[g][r] = 0;
    }
    // the epilogue operands in place, once they landed (after the item's first
    // stage barrier; the next barrier publishes them): row / column half-norms
    // with the padding's -1e300 (its k* is then exactly 0), alpha / kscale
#define UT_KQ_OPS_IN()                                                 \
  if (t < Q_BM) {                                                      \
    const double hv = (-0.5 * KSTAR_T_SCALE) * rx[t];                  \
    rx[t] = row0 + t < n ? hv : -1e300;                                \
    if (MU) ra[t] = ra[t] * ikscale;                                   \
  } else if (t < Q_BM + Q_BN) {                                        \
    const int u = t - Q_BM;                                            \
    const double hv = (-0.5 * KSTAR_T_SCALE) * cn[u];                  \
    cn[u] = col0 + u < m ? hv : -1e300;                                \
  }
    // the categorical stages first (the match count), then the digit stages
#define UT_KQ_STAGE_IN()                                                                               \
  vm_wait_n(cnt - (csl == 0 ? at0 : (csl == 1 ? at1 : at2)));   /* this stage (+ the item's operands) */ \
  __builtin_amdgcn_s_barrier();   /* ... landed in every wave; the slot two ahead fully read */       \
  asm volatile("" ::: "memory");                                                                      \
  UT_KQ_ISSUE();                                                                                      \
  const int8_t* st = lds + csl * Q_STAGE;                                                             \
  csl = csl == 2 ? 0 : csl + 1
    for (int32_t s2 = 0; s2 < ncs; ++s2) {
      UT_KQ_STAGE_IN();
      if (s2 == 0) UT_KQ_OPS_IN();
      // four 32-code steps (the first stage's first from zero)
      auto cbody = [&](auto first_c) {
        constexpr bool FIRST = decltype(first_c)::value;
#pragma unroll
        for (int kk = 0; kk < 4; ++kk) {
          const int c16 = 2 * kk + c;
          const i8v4 af = *reinterpret_cast<const i8v4*>(st + ra_ * 128 + ((c16 ^ (ra_ & 7)) << 4));
          const i8v4 bf = *reinterpret_cast<const i8v4*>(st + 8192 + cb * 128 + ((c16 ^ (cb & 7)) << 4));
          iacc = __builtin_amdgcn_mfma_i32_32x32x32_i8(af, bf, (FIRST && kk == 0) ? (i8v16){} : iacc, 0, 0, 0);
        }
      };
      if (s2 == 0) cbody(std::integral_constant<bool, true>{});
      else cbody(std::integral_constant<bool, false>{});
    }
    for (int32_t s2 = ncs; s2 < ntot; ++s2) {
      UT_KQ_STAGE_IN();
      if (s2 == 0) UT_KQ_OPS_IN();
      i8v4 af[I8_S];
#pragma unroll
      for (int p = 0; p < I8_S; ++p) af[p] = *reinterpret_cast<const i8v4*>(st + p * Q_PL + aoff);
      // digit products of group g = pa + qb (0-based: p + q <= 7 1-based); the
      // first stage starts each group from zero (its qb = 0 product)
      auto body = [&](auto first_c) {
        constexpr bool FIRST = decltype(first_c)::value;
#pragma unroll
        for (int qb = 0; qb < I8_S; ++qb) {
          const i8v4 bf = *reinterpret_cast<const i8v4*>(st + qb * Q_PL + boff);
#pragma unroll
          for (int pa = 0; pa + qb < I8_S; ++pa) {
            if (FIRST && qb == 0) acc[pa] = __builtin_amdgcn_mfma_i32_32x32x32_i8(af[pa], bf, (i8v16){}, 0, 0, 0);
            else acc[pa + qb] = __builtin_amdgcn_mfma_i32_32x32x32_i8(af[pa], bf, acc[pa + qb], 0, 0, 0);
          }
        }
      };
      if (s2 == ncs) body(std::integral_constant<bool, true>{});
      else body(std::integral_constant<bool, false>{});
    }
#undef UT_KQ_STAGE_IN
#undef UT_KQ_OPS_IN
#undef UT_KQ_ISSUE
    if (ntot == 1) {   // (no stage barrier after the first: publish the operands)
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
    }
    // lane: column cb of the tile, rows wm*32 + (q & 3) + 8 (q >> 2) + 4 (l >> 5)
    const double hc = cn[cb], sc = cs[cb];
    const int64_t col = col0 + cb;
    double s = 0.0, s2v = 0.0;
    uint32_t pw[I8_S][4];
    const bool store = !I8 && rt < store_rt;
#pragma unroll
    for (int G = 0; G < 4; ++G) {
      uint32_t lo[4], hi[4];
#pragma unroll
      for (int q4 = 0; q4 < 4; ++q4) {
        const int q = 4 * G + q4;
        const int rl = wm * 32 + q4 + 8 * G + 4 * c;
        double v;
        if constexpr (PAIR) {
          const int32_t u23 = (acc[0][q] << 8) + acc[1][q];
          const int32_t u45 = (acc[2][q] << 8) + acc[3][q];
          const int32_t u67 = (acc[4][q] << 8) + acc[5][q];
          v = __builtin_fma(__builtin_fma((double)u67, 0x1p-16, (double)u45), 0x1p-16, (double)u23);
        } else {
          v = (double)acc[5][q];
#pragma unroll
          for (int g = 4; g >= 0; --g) v = __builtin_fma(v, 0x1p-8, (double)acc[g][q]);
        }
        double base = rx[rl];
        if constexpr (CAT) base = __builtin_fma((double)iacc[q], cat_c1, cat_c0) + base;
        const double x = __builtin_fmax(__builtin_fmin(__builtin_fma(v, sc, base) + hc, 0.0), KSTAR_T_MIN);
        const double ks = sf2_exp2t_nonpos(x, etab);
        if constexpr (MU) s = __builtin_fma(ra[rl], ks, s);
        if (want2) s2v = __builtin_fma(ks, ks, s2v);
        if constexpr (I8) {
          const uint64_t b = i8_biased(ks);   // y = k* 2^-eb
          lo[q4] = (uint32_t)b;
          hi[q4] = (uint32_t)(b >> 32);
        } else {
          if (store) kst[(int64_t)(row0 + rl) * ldk + col] = (TS)ks;
        }
      }
      if constexpr (I8) {
        uint32_t pl[I8_S];
        i8_planes(lo, hi, pl);
#pragma unroll
        for (int p = 0; p < I8_S; ++p) pw[p][G] = pl[p];
      }
    }
    if constexpr (I8) {
      // lane l holds rows 8G .. 8G + 3 (l < 32) or 8G + 4 .. 8G + 7 of its column
      // for G = 0..3: two permlane32 swaps give l rows 0..15 and l + 32 rows
      // 16..31 of the wave's 32, one 32-byte piece of the column per plane
#pragma unroll
      for (int p = 0; p < I8_S; ++p) {
        const auto a0 = __builtin_amdgcn_permlane32_swap(pw[p][0], pw[p][2], false, false);
        const auto a1 = __builtin_amdgcn_permlane32_swap(pw[p][1], pw[p][3], false, false);
        int8_t* dst = reinterpret_cast<int8_t*>(kst) + p * lo_off + i8_off(col, row0 + wm * 32 + 16 * c, ldk);
        *reinterpret_cast<uint4*>(dst) = make_uint4(a0[0], a0[1], a1[0], a1[1]);
      }
    }
    if constexpr (MU) {
      // each wave's 32 rows: one partial per 32-row half tile (no cross-wave
      // reduction, so no barrier; the scoring sums npad / 32 partials)
      s += __shfl_xor(s, 32);
      if (want2) s2v += __shfl_xor(s2v, 32);
      if (lane < 32 && col < m) {
        const int64_t o = (int64_t)(2 * rt + wm) * ldk + col;
        part[o] = s;
        if (want2) part2[o] = s2v;
      }
    }
    if constexpr (I8) cnt += I8_S;   // the plane stores
    else if (store) cnt += 16;        // the rows' stores
    cob = cob == 2 ? 0 : cob + 1;
    crt += Wr;
    cctq += Wq;
    if (crt >= RT) {
      crt -= RT;
      ++cctq;
    }
    if (cctq * 8 + xcd >= CT) break;   // (uniform: no next item)
  }
}

// ---------------------------------------------------------------------------
int alloc_split_x8(ut_ctx* c, int32_t npad, int32_t K) {
  int rc;
  const int32_t K32 = (K + 31) / 32;
  if ((rc = ensure(c, c->gp_x8, (size_t)I8_S * (K32 > 0 ? K32 : 1) * 32 * npad))) return rc;
  return ensure(c, c->gp_q8, 2);
}

int launch_split_x8(ut_ctx* c, const double* XsT, int32_t K, int32_t npad) {
  const int32_t K32 = (K + 31) / 32;
  DevBuf<int8_t>& xd = c->gp_x8;
  UT_CHECK(c, xd.n >= (size_t)I8_S * K32 * 32 * npad && c->gp_q8.n >= 2, UT_EINVAL,
           "split_x8: planes not allocated (alloc_split_x8)");
  unsigned long long* amax = reinterpret_cast<unsigned long long*>(c->gp_q8.p);
  UT_HIP(c, hipMemsetAsync(amax, 0, sizeof(unsigned long long), c->stream));
  if (K > 0)
    hipLaunchKernelGGL(k_q_absmax, dim3(256), dim3(256), 0, c->stream, XsT, (int64_t)K * npad, amax);
  hipLaunchKernelGGL(k_q_split_x, dim3(grid1(npad, 256)), dim3(256), 0, c->stream, XsT, K, npad, K32, amax, xd.p,
                     c->gp_q8.p + 1);
  UT_LAUNCH_CHECK(c);
  return 0;
}

int launch_gemm_kstar_q(ut_ctx* c, bool planes, const double* XsT, int32_t npad, const double* ucand, int32_t dpad,
                        int64_t m, void* kst, int64_t ldk, double* part, int32_t store_rows, const double* cn,
                        double* part2, const KstarCat& cat, const double* xn, DevBuf<int8_t>& u8,
                        DevBuf<double>& scol) {
  const DevBuf<int8_t>& xd = c->gp_x8;
  const int32_t K32 = (dpad + 31) / 32;
  const bool pair = K32 * 32 <= Q_PAIR_MAX_K;
  const bool has_cat = cat.nkc > 0;
  // exact int32 group sums: K 6 2^14 < 2^31
  UT_CHECK(c, npad % Q_BM == 0 && ldk % Q_BN == 0 && ldk >= m && (int64_t)K32 * 32 * 6 * 16384 < (1LL << 31),
           UT_EINVAL, "gemm_kstar_q: bad padding or too many features");
  UT_CHECK(c, xd.p && xd.n >= (size_t)I8_S * K32 * 32 * npad, UT_EINVAL,
           "gemm_kstar_q: the fit has no training digit planes");
  UT_CHECK(c, !has_cat || (cat.acat && cat.bcat), UT_EINVAL, "gemm_kstar_q: categorical operands missing");
  UT_CHECK(c, K32 + cat.nkc >= 1, UT_EINVAL, "gemm_kstar_q: no features");
  // the library runs it for the variance's digit planes of numeric fits (the
  // mean from the variance epilogue, no one-hot codes: gp.hip gp_score_impl)
  UT_CHECK(c, planes && !part && !part2 && !has_cat && XsT == c->gp_XsT, UT_EINVAL,
           "gemm_kstar_q: digit planes of a numeric fit only");
  int rc;
  if ((rc = ensure(c, u8, (size_t)I8_S * (K32 > 0 ? K32 : 1) * 32 * ldk))) return rc;
  if ((rc = ensure(c, scol, (size_t)ldk))) return rc;
  hipLaunchKernelGGL(k_q_split_u, dim3(grid1(ldk, 256)), dim3(256), 0, c->stream, ucand, dpad, ldk, K32,
                     c->gp_q8.p + 1, pair ? -24 : -16, u8.p, scol.p);
  UT_LAUNCH_CHECK(c);
  const int32_t RT = npad / Q_BM;
  const int32_t CT = (int32_t)(ldk / Q_BN);
  const int32_t store_rt = store_rows < 0 ? RT : (store_rows + Q_BM - 1) / Q_BM;
  const int64_t items = (int64_t)RT * CT;
  const bool fit_in_flight = c->fit_pending && hipEventQuery(c->ev_fit) == hipErrorNotReady;
  const int32_t spare = fit_in_flight ? 2 : 0;   // as launch_gemm_kstar
  int32_t nb = 2 * (c->n_cu / 8 - spare) * 8;
  if (items < nb) nb = (int32_t)(((items + 7) / 8) * 8);
  const double* xnorm = xn ? xn : c->gp_xnorm;
  const double* cnorm = cn ? cn : c->cnorm.p;
  const double kscale = planes ? ldexp(1.0, -i8_kstar_exp(c->gp_sf2)) : 1.0;
#define UT_KQ_LAUNCH(PAIR)                                                                                     \
  hipLaunchKernelGGL((k_gp_kstar_q<int8_t, false, false, PAIR>), dim3(nb), dim3(Q_NT), 0, c->stream, xd.p, npad,    \
                     u8.p, ldk, K32, scol.p, RT, CT, xnorm, cnorm, c->gp_alpha, c->gp_sf2, c->gp_n, m, (int8_t*)kst, \
                     nullptr, kscale, (int64_t)npad * ldk, store_rt, nullptr, cat.acat, cat.bcat, cat.nkc,         \
                     cat.c0 * KSTAR_T_SCALE, cat.c1 * KSTAR_T_SCALE)
  if (pair) UT_KQ_LAUNCH(true);
  else UT_KQ_LAUNCH(false);
#undef UT_KQ_LAUNCH
  UT_LAUNCH_CHECK(c);
  return 0;
}

}  // namespace ut
