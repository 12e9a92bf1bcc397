// propose.hip -- population initialisation and batched proposal operators.
//
// One lane = one candidate; the parameter loop is wave-uniform (every lane
// of a wave works on the same parameter, so the DevParam record is a scalar
// load and there is no divergence on the parameter kind).  Values are SoA
// columns ([P][ld] f64), so each per-parameter load/store of a wave is one
// fully coalesced 512-byte access.  Bound: HBM (40*P bytes per DE trial).
//
// Arithmetic is compiled with -ffp-contract=off and follows Python's
// evaluation order so the results are bit-identical to the reference
// operators given the same random draws:
//   op1_randomize       manipulator.py:596-606 (numeric), :940-949 (bool), :1033-1042 (enum)
//   get_unit_value      manipulator.py:473-488
//   set_unit_value      manipulator.py:490-503
//   op4_set_linear      manipulator.py:523-542 (primitive), :866-914 (complex)
//   DE trial            differentialevolution.py:105-129
//   PERM operators      manipulator.py:1048-1356 (ut_perm.h)
//
// Column model: param p's values start at SoA column params[p].col; a PERM
// of size S owns S columns (item indices).  Per-param random draws are keyed
// by the PARAM index, so spaces without PERMs (col == p) are unchanged.
#include "ut_param.h"
#include "ut_perm.h"

namespace ut {

__global__ __launch_bounds__(256) void k_population_init(const DevParam* __restrict__ params, int32_t P,
                                                         double* __restrict__ pop, int64_t ld, int64_t npop,
                                                         uint64_t seed, uint32_t round_) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= npop) return;
  for (int32_t p = 0; p < P; ++p) {
    const DevParam pr = params[p];
    if (pr.kind == UT_PERM) {
      // seed_value() = list(items), then op1_randomize = shuffle
      WRow x{pop + (int64_t)pr.col * ld + i, ld};
      perm_identity(x, pr.psize);
      PermRng R(seed, (uint64_t)i, (uint32_t)p, round_, OP_INIT);
      perm_shuffle(x, pr.psize, R);
      continue;
    }
    const u32x4 r = draw(seed, (uint64_t)i, (uint32_t)p, round_, OP_INIT);
    pop[(int64_t)pr.col * ld + i] = randomize(pr, r);
  }
}

// x1, x2, x3 = the first 3 of shuffle(list(set(population) - {target}) +
// [best] * information_sharing) (differentialevolution.py:109-118): three
// distinct positions of a pool of Q = (npop - 1) + share entries.  Position
// q < npop - 1 is the q-th member other than t (q + (q >= t)); positions
// >= npop - 1 are copies of the best config, returned as -1.  With share = 0
// this is exactly 3 distinct members != t.
__device__ __forceinline__ int64_t pool_member(int64_t q, int64_t npop, int64_t t) {
  return q < npop - 1 ? q + (q >= t ? 1 : 0) : -1;
}
__device__ __forceinline__ void pick_donors(uint32_t w0, uint32_t w1, uint32_t w2, int64_t npop, int64_t share,
                                            int64_t t, int64_t& d1, int64_t& d2, int64_t& d3) {
  const int64_t Q = npop - 1 + share;
  const int64_t a = (int64_t)umulhi32(w0, (uint32_t)Q);
  int64_t b = (int64_t)umulhi32(w1, (uint32_t)(Q - 1));
  b += (b >= a ? 1 : 0);
  const int64_t s0 = a < b ? a : b, s1 = a < b ? b : a;
  int64_t c = (int64_t)umulhi32(w2, (uint32_t)(Q - 2));
  if (c >= s0) ++c;
  if (c >= s1) ++c;
  d1 = pool_member(a, npop, t);
  d2 = pool_member(b, npop, t);
  d3 = pool_member(c, npop, t);
}

// Fused DE-diff outputs (DE scoring rounds, ut_score_round_de): which
// computed-digest values of the trial differ bitwise from the target's, as the
// mask [ceil(n_comp/32)][ldo] and compacted (candidate << 20 | cslot) pairs --
// what k_de_diff derives by re-reading both rows, taken here from registers.
struct DeDiffOut {
  uint32_t* mask;
  uint64_t* pairs;
  unsigned long long* npairs;
  int32_t n_comp;
};

// One DE trial per candidate.  Candidate g (global) targets member g % npop.
// Forced crossover set = a uniform n_cross-subset of the params (the first
// n_cross names of a uniform shuffle, differentialevolution.py:122-125), drawn
// by skip-rank from one block; the `random() < cr` tests are 32-bit uniforms,
// four params per Philox block (ut_core.h de_forced_set / DE_CR_STREAM).  The
// first pass keeps the tests' outcomes as one bit per param in LDS
// ([ceil(P/32)][blockDim] words, each lane its own column), so the second pass
// draws nothing for the crossover decision.
// AOS (the default): block = one wave; the donors' values come from the
// member-major donor copy (pop_aos, [npop + 1][lda], row npop = the best
// config; primitive params as unit values, so no unit_of is left here), staged
// DE_GW columns at a time into LDS by global_load_lds row gathers of 64-B
// pieces: 3 x 64 pieces per wave and group instead of one 8-B gather (a cache
// line each) per crossing (param, donor).  The first group's loads are issued
// before pass 1, so the Philox work hides them.  The target's raw values are
// read column-major one param ahead.
// LDS image per donor k: [64 candidates][DE_CH chunks of 16 B], chunk ch of
// candidate c at position ch ^ ((c >> DE_SW) & (DE_CH - 1)) (the swizzle goes on
// the source address: a glds writes lane-linear), so a wave's ds_read_b64 of
// one column is at worst 2-way bank-conflicted.
// Measured at C2 (k_de alone, m = 2^20): 0.99 ms column-major gathers; staged
// whole lines with the target row too (32 KiB per wave, 4 waves per CU) 1.12 ms;
// 64-B pieces (16 KiB, 9 waves per CU) 0.82 ms; 32-B pieces 1.32 ms.
#ifndef UT_DE_GW
#define UT_DE_GW 8
#endif
constexpr int DE_GW = UT_DE_GW;                  // columns per staged group (8: 64-B half lines, 16: whole lines)
constexpr int DE_CH = DE_GW / 2;                 // 16-B chunks per row and group
constexpr int DE_SW = DE_CH == 8 ? 1 : (DE_CH == 4 ? 2 : 3);  // swizzle: chunk ^ ((candidate >> DE_SW) & (DE_CH - 1))
#ifndef UT_DE_DB
#define UT_DE_DB 0
#endif
constexpr int DE_NBUF = UT_DE_DB ? 2 : 1;        // 2: group g + 1 is in flight while group g is processed
constexpr int DE_AOS_BUF = 3 * 64 * DE_GW;       // the donor rows of one group per wave
constexpr int DE_AOS_LDS_DBL = DE_NBUF * DE_AOS_BUF;

template <bool DIFF, bool AOS>
__global__ __launch_bounds__(AOS ? 64 : 256) void k_de(const DevParam* __restrict__ params, int32_t P,
                                            const double* __restrict__ vtab, const double* __restrict__ pop, int64_t ldp, int64_t npop,
                                            const double* __restrict__ best, int64_t share,
                                            double cr, int32_t n_cross, uint64_t seed, uint32_t round_,
                                            int64_t cand_base, int64_t m, double* __restrict__ out,
                                            int64_t ldo, DeDiffOut dd, uint32_t* __restrict__ xglob,
                                            const double* __restrict__ aos, int64_t lda) {
  extern __shared__ __attribute__((aligned(16))) uint32_t dyn_lds[];
  double* const stg = reinterpret_cast<double*>(dyn_lds);                    // AOS: the donor lines
  uint32_t* const xlds = AOS ? dyn_lds + 2 * DE_AOS_LDS_DBL : dyn_lds;       // [ceil(P/32)][blockDim]
  const int tid = threadIdx.x, lane = tid & 63;
  const int64_t i0 = (int64_t)blockIdx.x * blockDim.x + tid;
  // the bits live in LDS, or (spaces of more than 2048 params) in a global
  // [ceil(P/32)][grid * blockDim] scratch
  uint32_t* const xb = xglob ? xglob + i0 : xlds + tid;
  const int64_t xs = xglob ? (int64_t)gridDim.x * blockDim.x : (int64_t)blockDim.x;
  // out-of-range lanes of the last block run along (on candidate m-1) and
  // write nothing: the DIFF epilogue takes one atomic per whole wave, and the
  // AOS gathers load the rows of every lane's donors
  const bool valid = i0 < m;
  if (!DIFF && !AOS && !valid) return;
  const int64_t i = valid ? i0 : m - 1;
  const uint64_t g = (uint64_t)(cand_base + i);
  const int64_t t = (int64_t)(g % (uint64_t)npop);
  const u32x4 rc = draw(seed, g, STREAM_CAND | 0u, round_, OP_DE);
  int64_t d1, d2, d3;
  pick_donors(rc.x, rc.y, rc.z, npop, share, t, d1, d2, d3);
  const u32x4 rf = draw(seed, g, STREAM_CAND | 1u, round_, OP_DE);
  // use_f = old_div(random.random(), 2.0) + 0.5
  const double F = __dadd_rn(__ddiv_rn(u01_from(rf.x, rf.y), 2.0), 0.5);
  const double nF = -F;

  // AOS: the donor rows of the 8 candidates each of this lane's 24 gather
  // pieces ((donor k, candidate block q): candidate 8q + lane / 8, 16-B chunk
  // lane % 8 of its line)
  uint32_t srow[3][DE_CH];
  int32_t cur_grp = -1;
  int32_t staged[2] = {-1, -1};   // the group held by each LDS buffer
  auto issue_group = [&](int32_t gi) {
    staged[gi % DE_NBUF] = gi;
    double* const buf = stg + (gi % DE_NBUF) * DE_AOS_BUF;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // the previous group's LDS reads are done
#pragma unroll
    for (int k = 0; k < 3; ++k)
#pragma unroll
      for (int q = 0; q < DE_CH; ++q) {
        const int cnd = (64 / DE_CH) * q + lane / DE_CH;
        const int ch = (lane % DE_CH) ^ ((cnd >> DE_SW) & (DE_CH - 1));
        const double* src = aos + (int64_t)srow[k][q] * lda + gi * DE_GW + ch * 2;
        __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)(buf + k * 64 * DE_GW + q * 128), 16,
                                         0, 0);
      }
  };
  if constexpr (AOS) {
    const uint32_t r1 = d1 >= 0 ? (uint32_t)d1 : (uint32_t)npop, r2 = d2 >= 0 ? (uint32_t)d2 : (uint32_t)npop,
                   r3 = d3 >= 0 ? (uint32_t)d3 : (uint32_t)npop;
#pragma unroll
    for (int q = 0; q < DE_CH; ++q) {
      const int src_lane = (64 / DE_CH) * q + lane / DE_CH;
      srow[0][q] = (uint32_t)__shfl((int)r1, src_lane, 64);
      srow[1][q] = (uint32_t)__shfl((int)r2, src_lane, 64);
      srow[2][q] = (uint32_t)__shfl((int)r3, src_lane, 64);
    }
    // the first group with a non-PERM column, issued ahead of the Philox pass
    for (int32_t p = 0; p < P; ++p) {
      const DevParam pr = params[p];
      if (pr.kind != UT_PERM) {
        cur_grp = pr.col / DE_GW;
        break;
      }
    }
    if (cur_grp >= 0) {
      issue_group(cur_grp);
      if (DE_NBUF == 2 && (cur_grp + 1) * DE_GW < lda) issue_group(cur_grp + 1);
    }
  }
  // AOS: the target's value of param p, loaded one param ahead
  auto load_vt = [&](int32_t p) -> double {
    const DevParam q = params[p];
    return q.kind != UT_PERM ? pop[(int64_t)q.col * ldp + t] : 0.0;
  };
  double vt_next = 0.0;
  if constexpr (AOS) vt_next = load_vt(0);
  // donor k's value of column col (AOS: from the staged group of col)
  auto donor = [&](int k, int32_t col) -> double {
    const int cc = col % DE_GW;
    return stg[(cur_grp % DE_NBUF) * DE_AOS_BUF + k * 64 * DE_GW + lane * DE_GW +
               ((((cc >> 1) ^ ((lane >> DE_SW) & (DE_CH - 1))) << 1) | (cc & 1))];
  };

  // pass 1: the forced set and the cr-test bits (four params per Philox block)
  int32_t fset[4];
  de_forced_set(draw(seed, g, STREAM_CAND | 2u, round_, OP_DE), P, n_cross, fset);
  {
    uint32_t acc = 0;
    for (int32_t p0 = 0; p0 < P; p0 += 4) {
      const u32x4 r = draw(seed, g, STREAM_CAND | (DE_CR_STREAM + (uint32_t)(p0 >> 2)), round_, OP_DE);
      const uint32_t ws[4] = {r.x, r.y, r.z, r.w};
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int32_t p = p0 + q;
        if (p < P && de_cr_pass(ws[q], cr)) acc |= 1u << (p & 31);
      }
      if ((p0 & 31) == 28 || p0 + 4 >= P) {   // a 32-param word is complete
        xb[(p0 >> 5) * xs] = acc;
        acc = 0;
      }
    }
  }

  uint32_t xw = 0;                  // the cr-test bits of params [32 (p>>5), +32)
  uint32_t dw = 0;                  // DIFF: mask bits of the current word
  int32_t dwi = 0;                  // DIFF: its word index
  uint32_t dcnt = 0;                // DIFF: changed computed-digest values
  if constexpr (AOS) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the first group landed
  }
  for (int32_t p = 0; p < P; ++p) {
    const DevParam pr = params[p];
    if ((p & 31) == 0) xw = xb[(p >> 5) * xs];
    if constexpr (AOS) {
      // wave-uniform: columns grow with p, so the groups are staged in order
      if (pr.kind != UT_PERM && pr.col / DE_GW != cur_grp) {
        cur_grp = pr.col / DE_GW;
        if (staged[cur_grp % DE_NBUF] != cur_grp) issue_group(cur_grp);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        // the next group into the other buffer (its previous group is consumed)
        if (DE_NBUF == 2 && (cur_grp + 1) * DE_GW < lda) issue_group(cur_grp + 1);
      }
    }
    double vt_pf = 0.0;
    if constexpr (AOS) {
      vt_pf = vt_next;
      if (p + 1 < P) vt_next = load_vt(p + 1);
    }
    const bool forced = p == fset[0] || p == fset[1] || p == fset[2] || p == fset[3];
    const double* col = pop + (int64_t)pr.col * ldp;
    // `i < n_cross or random() < cr` (short-circuit: the draw is only
    // consulted for non-forced params, which is what selecting on it does)
    const bool cross = forced || ((xw >> (p & 31)) & 1u);
    if (pr.kind == UT_PERM) {
      if (!valid) continue;  // no computed digest (cslot -1): nothing for the DIFF epilogue
      // ComplexParameter.op4_set_linear: copy x1, shuffle it iff x2 != x3
      const int32_t S = pr.psize;
      WRow o{out + (int64_t)pr.col * ldo + i, ldo};
      if (cross) {
        // donor -1 = the best config's row (stride 1 over its columns)
        const double* bcol = best + pr.col;
        const PRow r1 = d1 >= 0 ? PRow{col + d1, ldp} : PRow{bcol, 1};
        const PRow r2 = d2 >= 0 ? PRow{col + d2, ldp} : PRow{bcol, 1};
        const PRow r3 = d3 >= 0 ? PRow{col + d3, ldp} : PRow{bcol, 1};
        perm_copy(o, r1, S);
        if (!perm_equal(r2, r3, S)) {
          PermRng R(seed, g, (uint32_t)p | (1u << STREAM_SUB_SHIFT), round_, OP_DE);
          perm_shuffle(o, S, R);
        }
      } else {
        perm_copy(o, PRow{col + t, ldp}, S);
      }
      continue;
    }
    double vt;
    if constexpr (AOS) vt = vt_pf;
    else vt = col[t];
    double v = vt;
    if (cross) {
      double x1, x2, x3;
      if constexpr (AOS) {
        x1 = donor(0, pr.col);
        x2 = donor(1, pr.col);
        x3 = donor(2, pr.col);
      } else {
        const double xb = share ? best[pr.col] : 0.0;
        x1 = d1 >= 0 ? col[d1] : xb;
        x2 = d2 >= 0 ? col[d2] : xb;
        x3 = d3 >= 0 ? col[d3] : xb;
      }
      if (is_primitive(pr.kind)) {
        double va = x1, vb = x2, vc = x3;   // AOS: the donor copy holds unit values
        if constexpr (!AOS) {
          va = unit_of(pr, x1, vtab);
          vb = unit_of(pr, x2, vtab);
          vc = unit_of(pr, x3, vtab);
        }
        // v = a*va + b*vb + c*vc with a = 1.0, b = F, c = -F
        double u = __dadd_rn(__dadd_rn(__dmul_rn(1.0, va), __dmul_rn(F, vb)), __dmul_rn(nF, vc));
        u = py_max(0.0, py_min(u, 1.0));
        v = from_unit(pr, u, vt);
      } else {
        // ComplexParameter.op4_set_linear with a=1, b=F, c=-F reduces to
        // copy_value(x1) then add_difference: randomize iff x2 != x3.
        v = x1;
        if (x2 != x3) {
          const u32x4 rq = draw(seed, g, (uint32_t)p | (1u << STREAM_SUB_SHIFT), round_, OP_DE);
          v = randomize(pr, rq);
        }
      }
    }
    if (valid) out[(int64_t)pr.col * ldo + i] = v;
    if constexpr (DIFF) {
      // cslots are assigned in param order, so the mask words fill in order
      const int32_t cs = pr.cslot;
      if (cs >= 0) {
        if ((cs >> 5) != dwi) {
          if (valid) dd.mask[(int64_t)dwi * ldo + i] = dw;
          dw = 0;
          dwi = cs >> 5;
        }
        if (__double_as_longlong(v) != __double_as_longlong(vt)) {
          dw |= 1u << (cs & 31);
          ++dcnt;
        }
      }
    }
  }
  if constexpr (DIFF) {
    if (dd.n_comp <= 0) return;
    if (valid) dd.mask[(int64_t)dwi * ldo + i] = dw;
    if (!valid) dcnt = 0;
    // one atomic per wave for the wave's pair count, then the pairs slot-major
    // within the wave (ballot + mbcnt: each store instruction writes one
    // contiguous run, and k_inner_pairs sees mostly one param per wave)
    uint32_t tot = dcnt;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) tot += __shfl_xor(tot, d, 64);
    unsigned long long base = 0;
    if (lane == 0 && tot) base = atomicAdd(dd.npairs, (unsigned long long)tot);
    base = __shfl(base, 0, 64);
    if (!tot) return;
    const uint64_t lt = (1ull << lane) - 1ull;   // lanes below this one
    for (int32_t w = 0; w * 32 < dd.n_comp; ++w) {
      const uint32_t bits = valid ? dd.mask[(int64_t)w * ldo + i] : 0u;
      const int32_t hi = dd.n_comp - w * 32 < 32 ? dd.n_comp - w * 32 : 32;
      for (int32_t b = 0; b < hi; ++b) {
        const bool on = (bits >> b) & 1u;
        const uint64_t bal = __ballot(on);
        if (on) dd.pairs[base + __popcll(bal & lt)] = ((uint64_t)i << 20) | (uint64_t)(w * 32 + b);
        base += __popcll(bal);
      }
    }
  }
}

// GP features of a configuration: emit(feature column, value) for each feature
// of param pr at candidate i (every column of the param is emitted)
// (encode_param_v: the same with the param's first value column already loaded)
template <class Emit>
__device__ __forceinline__ void encode_param_v(const DevParam& pr, double v, const double* __restrict__ values,
                                               int64_t ld, int64_t i, const double* __restrict__ vtab, Emit&& emit) {
  if (is_primitive(pr.kind)) {
    emit(pr.feat_col, unit_of(pr, v, vtab));
  } else if (pr.kind == UT_BOOL) {
    emit(pr.feat_col, v);
  } else if (pr.kind == UT_PERM) {
    // position of each item, normalised: feature[item] = k / (S - 1)
    const int32_t S = pr.psize;
    for (int32_t k = 0; k < S; ++k) {
      int32_t item = (int32_t)values[(int64_t)(pr.col + k) * ld + i];
      item = item < 0 ? 0 : (item >= S ? S - 1 : item);  // never fault on garbage input
      emit(pr.feat_col + item, S > 1 ? (double)k / (double)(S - 1) : 0.0);
    }
  } else {
    const int64_t o = (int64_t)v;
    for (int64_t k = 0; k < pr.n_opt; ++k) emit(pr.feat_col + (int32_t)k, (k == o) ? 1.0 : 0.0);
  }
}

template <class Emit>
__device__ __forceinline__ void encode_param(const DevParam& pr, const double* __restrict__ values, int64_t ld,
                                             int64_t i, const double* __restrict__ vtab, Emit&& emit) {
  encode_param_v(pr, values[(int64_t)pr.col * ld + i], values, ld, i, vtab, emit);
}

__global__ __launch_bounds__(256) void k_encode(const DevParam* __restrict__ params, int32_t P,
                                                const double* __restrict__ vtab, const double* __restrict__ values, int64_t ld, int64_t m,
                                                double* __restrict__ feat, int64_t ldf) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= m) return;
  constexpr int ENC_PF = 8;   // value columns loaded ahead (see k_encode_scaled_cat)
  for (int32_t p0 = 0; p0 < P; p0 += ENC_PF) {
    double vv[ENC_PF];
#pragma unroll
    for (int q = 0; q < ENC_PF; ++q) vv[q] = p0 + q < P ? values[(int64_t)params[p0 + q].col * ld + i] : 0.0;
#pragma unroll
    for (int q = 0; q < ENC_PF; ++q) {
      if (p0 + q >= P) break;
      encode_param_v(params[p0 + q], vv[q], values, ld, i, vtab,
                     [&](int32_t c, double f) { feat[(int64_t)c * ldf + i] = f; });
    }
  }
}

// k_encode and k_gp_prep_cand in one pass (dense scoring rounds): the K* B
// operand U'[k][i] = feature_k / ell_k straight from the values (0 for k >= F
// and for the padding columns i >= m) and cnorm[i] = |u'_i|^2, summed in
// feature order as k_gp_prep_cand sums (a PERM's items in position order).
// Saves the feature matrix's write and re-read (2 x 8 F bytes per candidate).
__global__ __launch_bounds__(256) void k_encode_scaled(const DevParam* __restrict__ params, int32_t P,
                                                       const double* __restrict__ vtab,
                                                       const double* __restrict__ values, int64_t ld, int64_t m,
                                                       int32_t F, const double* __restrict__ inv_ell, int32_t dpad,
                                                       double* __restrict__ u, int64_t ldu, double* __restrict__ cn) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= ldu) return;
  double s = 0.0;
  if (i < m) {
    constexpr int ENC_PF = 8;   // value columns loaded ahead (see k_encode_scaled_cat)
    for (int32_t p0 = 0; p0 < P; p0 += ENC_PF) {
      double vv[ENC_PF];
#pragma unroll
      for (int q = 0; q < ENC_PF; ++q) vv[q] = p0 + q < P ? values[(int64_t)params[p0 + q].col * ld + i] : 0.0;
#pragma unroll
      for (int q = 0; q < ENC_PF; ++q) {
        if (p0 + q >= P) break;
        encode_param_v(params[p0 + q], vv[q], values, ld, i, vtab, [&](int32_t c, double f) {
          const double v = f * inv_ell[c];
          u[(int64_t)c * ldu + i] = v;
          s += v * v;
        });
      }
    }
  } else {
    for (int32_t k = 0; k < F; ++k) u[(int64_t)k * ldu + i] = 0.0;
  }
  for (int32_t k = F; k < dpad; ++k) u[(int64_t)k * ldu + i] = 0.0;
  cn[i] = s;
}

// the categorical K*'s candidate operands in one pass (gp_gemm.hip
// "Categorical K*"): U'[k][i] = numeric feature k / ell (0 past n_num and for
// the padding columns), cnorm[i] = |u'_i|^2 over the numeric features in
// feature order, and the one-hot codes bcat[(q >> 7)][i][q & 127] = 1 at code
// column q = ccol + option (ENUM), ccol + (value != 0) (BOOL); every code byte
// of the candidate is written.  One thread per candidate, 256 per workgroup
// (ldu % 256 == 0): each numeric feature of U' is written once (the padding
// rows >= n_num zero) and |u'|^2 summed in feature order on the way; the codes
// are set as bits in LDS and stored as whole 128-byte rows (store_code_rows:
// the byte stores per candidate row made this kernel 18 ms at C4)
__global__ __launch_bounds__(256) void k_encode_scaled_cat(const DevParam* __restrict__ params, int32_t P,
                                                           const double* __restrict__ vtab,
                                                           const double* __restrict__ values, int64_t ld, int64_t m,
                                                           const int32_t* __restrict__ feat_num, int32_t n_num,
                                                           int32_t dpad, const double* __restrict__ inv_ell,
                                                           const int32_t* __restrict__ cat_ccol, int32_t cat_k,
                                                           double* __restrict__ u, int64_t ldu, double* __restrict__ cn,
                                                           int8_t* __restrict__ bcat) {
  extern __shared__ uint32_t dyn[];
  const int32_t stride = cat_k / 32 + 1;
  uint32_t* bits = dyn;
  uint32_t* img = dyn + 256 * stride;
  const int t = threadIdx.x;
  const int64_t i0 = (int64_t)blockIdx.x * 256, i = i0 + t;
  for (int32_t w = 0; w < stride; ++w) bits[t * stride + w] = 0u;
  double s = 0.0;
  if (i < m) {
    // the params' value columns loaded ENC_PF at a time ahead of their use: one
    // load in flight per param left the kernel latency-bound (two workgroups per
    // CU for the LDS; C4: 339 params, ~10 ms at 2^22 candidates)
    constexpr int ENC_PF = 8;
    for (int32_t p0 = 0; p0 < P; p0 += ENC_PF) {
      double vv[ENC_PF];
#pragma unroll
      for (int q = 0; q < ENC_PF; ++q)
        vv[q] = p0 + q < P ? values[(int64_t)params[p0 + q].col * ld + i] : 0.0;
#pragma unroll
      for (int q = 0; q < ENC_PF; ++q) {
        const int32_t p = p0 + q;
        if (p >= P) break;
        const int32_t cc = cat_ccol[p];
        const DevParam pr = params[p];
        const double v = vv[q];
        if (cc >= 0) {
          const int64_t o = pr.kind == UT_BOOL ? (v != 0.0 ? 1 : 0) : (int64_t)v;
          if (o < 0 || o >= (pr.kind == UT_BOOL ? 2 : pr.n_opt)) continue;   // no option: no match
          const int32_t qb = cc + (int32_t)o;
          bits[t * stride + (qb >> 5)] |= 1u << (qb & 31);
          continue;
        }
        encode_param_v(pr, v, values, ld, i, vtab, [&](int32_t c, double f) {
          const double x = f * inv_ell[c];
          u[(int64_t)feat_num[c] * ldu + i] = x;
          s += x * x;
        });
      }
    }
  }
  for (int32_t k = i < m ? n_num : 0; k < dpad; ++k) u[(int64_t)k * ldu + i] = 0.0;
  cn[i] = s;
  __syncthreads();
  store_code_rows(bits, stride, cat_k / 128, img, bcat, ldu, i0);
}

__global__ void k_gather_rows(int32_t NC, const double* __restrict__ values, int64_t ld,
                              const int64_t* __restrict__ idx, int64_t cand_base, int32_t k,
                              double* __restrict__ out, int64_t ldo, const uint32_t* __restrict__ dig,
                              uint32_t* __restrict__ out_dig) {
  const int32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= k) return;
  const int64_t g = idx[j];
  const int64_t i = g - cand_base;
  for (int32_t p = 0; p < NC; ++p) out[(int64_t)p * ldo + j] = (g >= 0) ? values[(int64_t)p * ld + i] : 0.0;
  if (out_dig) {
    for (int w = 0; w < 8; ++w) out_dig[(int64_t)j * 8 + w] = (g >= 0) ? dig[i * 8 + w] : 0u;
  }
}

__global__ void k_pop_replace(int32_t NC, double* __restrict__ pop, int64_t ldp, const double* __restrict__ trial,
                              int64_t ld, const int64_t* __restrict__ idx, int64_t n) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  const int64_t dst = idx[j];
  for (int32_t p = 0; p < NC; ++p) pop[(int64_t)p * ldp + dst] = trial[(int64_t)p * ld + j];
}

// ---------------------------------------------------------------------------
// PSO: HybridParticle.move (pso.py:70-77) with the per-kind op3_swarm
// (manipulator.py:660-700 Int, :709-744 Float, :962-996 Bool, :409-443 Enum,
// :1115-1140 Permutation).  Candidate g moves particle g % npop:  cfg = x,
// cfg1 = gbest, cfg2 = pbest, c = omega, c1 = phi_g, c2 = phi_l.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_pso(const DevParam* __restrict__ params, int32_t P,
                                             const double* __restrict__ vtab, const double* __restrict__ pos, const double* __restrict__ vel,
                                             const double* __restrict__ pbest, int64_t ldp, int64_t npop,
                                             const double* __restrict__ gbest, double c, double c1, double c2,
                                             double sigma, int32_t enum_mode, int32_t xop, uint64_t seed,
                                             uint32_t round_, int64_t cand_base, int64_t m, double* __restrict__ out_x,
                                             double* __restrict__ out_v, int64_t ldo, double* __restrict__ ws,
                                             int64_t ldw, int32_t scr_col) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= m) return;
  const uint64_t g = (uint64_t)(cand_base + i);
  const int64_t t = (int64_t)(g % (uint64_t)npop);
  for (int32_t p = 0; p < P; ++p) {
    const DevParam pr = params[p];
    const int64_t o = (int64_t)pr.col * ldp + t;
    const u32x4 r = draw(seed, g, (uint32_t)p, round_, OP_PSO);
    if (pr.kind == UT_PERM) {
      // op3_swarm: if uniform(0,1) > c: op3_cross(cfg, cfg, g if uniform(0,1) < c1 else l)
      const int32_t S = pr.psize;
      const PRow x{pos + o, ldp};
      WRow ox{out_x + (int64_t)pr.col * ldo + i, ldo};
      if (u01_from(r.x, r.y) > c) {
        const PRow other = (u01_from(r.z, r.w) < c1) ? PRow{gbest + pr.col, 1} : PRow{pbest + o, ldp};
        PermRng R(seed, g, (uint32_t)p | (1u << STREAM_SUB_SHIFT), round_, OP_PSO);
        perm_cross(xop, ox, x, other, S, (int32_t)rint((double)S * 0.3), WRow{ws + (int64_t)scr_col * ldw + i, ldw},
                   R);
      } else {
        perm_copy(ox, x, S);
      }
      if (out_v)  // op3_swarm returns None: the particle keeps no velocity for it
        for (int32_t k = 0; k < S; ++k) out_v[(int64_t)(pr.col + k) * ldo + i] = 0.0;
      continue;
    }
    // scaled kinds move in their search scale (get_value / set_value):
    // LOGINT by the Float rule on log values, POW2 by the Int rule on exponents
    const double xr = pos[o], v = vel[o];
    const double x = scaled_of(pr, xr, vtab), l = scaled_of(pr, pbest[o], vtab), gb = scaled_of(pr, gbest[pr.col], vtab);
    const double r1 = u01_from(r.x, r.y), r2 = u01_from(r.z, r.w);
    double nx, nv;
    if (pr.kind == UT_ENUM) {
      nv = v;
      nx = xr;  // reference: opn_stochastic_mix copies the particle INTO the parent (manipulator.py:442)
      if (enum_mode == 1) {
        const u32x4 q = draw(seed, g, (uint32_t)p | (1u << STREAM_SUB_SHIFT), round_, OP_PSO);
        const double rr = u01_from(q.x, q.y);
        const double tot = (c + c1) + c2;
        const double w0 = c / tot, w1 = c1 / tot;
        nx = rr < w0 ? xr : (rr < w0 + w1 ? gbest[pr.col] : pbest[o]);
      }
    } else {
      nv = ((v * c) + (((gb - x) * c1) * r1)) + (((l - x) * c2) * r2);
      if (pr.kind == UT_FLOAT || pr.kind == UT_LOGINT) {
        // legal_range: FLOAT (lo, hi); LOGINT its scaled range (u_lo, u_hi)
        const double vmin = pr.kind == UT_FLOAT ? pr.lo : pr.u_lo, vmax = pr.kind == UT_FLOAT ? pr.hi : pr.u_hi;
        double y = x + nv;
        y = (vmin > y) ? vmin : y;              // max(p, vmin)
        nx = unscale(pr, (y < vmax) ? y : vmax);  // min(vmax, .); set_value
      } else if (pr.kind == UT_INT || pr.kind == UT_POW2) {
        const double k = pr.hi - pr.lo;
        const double s = k / (1.0 + ut_exp(-nv)) + pr.lo;
        const double z = normal_draw(seed, g, (uint32_t)p | (2u << STREAM_SUB_SHIFT), round_, OP_PSO);
        double pp = rint(s + z * (sigma * k));
        pp = (pr.lo > pp) ? pr.lo : pp;
        nx = unscale(pr, (pp < pr.hi) ? pp : pr.hi);
      } else {  // BOOL
        const double s = 1.0 / (1.0 + ut_exp(-nv));
        const u32x4 q = draw(seed, g, (uint32_t)p | (1u << STREAM_SUB_SHIFT), round_, OP_PSO);
        nx = ((s - u01_from(q.x, q.y)) > 0.0) ? 1.0 : 0.0;
      }
    }
    out_x[(int64_t)pr.col * ldo + i] = nx;
    if (out_v) out_v[(int64_t)pr.col * ldo + i] = nv;
  }
}

// ---------------------------------------------------------------------------
// GA family: EvolutionaryTechnique.desired_configuration
// (evolutionarytechniques.py:29-61), NormalMutationMixin (:98-114),
// CrossoverMixin (:117-134, PERM params of size > 6), GGA crossover
// (globalGA.py:68-76).  Random d-subsets ("first d of a shuffle") by
// selection sampling, one uniform per parameter (oracle/ga.py).
// ---------------------------------------------------------------------------
__device__ __forceinline__ double parent_value(const DevParam& pr, const double* parent, int32_t p, uint32_t sub,
                                               uint64_t seed, uint64_t g, uint32_t round_, uint32_t op) {
  if (parent) return parent[pr.col];
  return randomize(pr, draw(seed, g, (uint32_t)p | (sub << STREAM_SUB_SHIFT), round_, op));
}

// the permutation of a parent: its row (broadcast), or a random one
// materialised in the workspace (manipulator.random() = seed + shuffle)
__device__ __forceinline__ PRow parent_perm(const DevParam& pr, const double* parent, int32_t p, uint32_t sub,
                                            uint64_t seed, uint64_t g, uint32_t round_, uint32_t op, double* wsc,
                                            int64_t ldw, bool build) {
  if (parent) return PRow{parent + pr.col, 1};  // a host-supplied row: contiguous
  WRow w{wsc, ldw};
  if (build) {
    perm_identity(w, pr.psize);
    PermRng R(seed, g, (uint32_t)p | (sub << STREAM_SUB_SHIFT), round_, op);
    perm_shuffle(w, pr.psize, R);
  }
  return w.ro();
}

__global__ __launch_bounds__(256) void k_ga(const DevParam* __restrict__ params, int32_t P,
                                            const double* __restrict__ vtab, const double* __restrict__ parent1, const double* __restrict__ parent2,
                                            double mutation_rate, double sigma, double crossover_rate, int32_t d_cross,
                                            int32_t must, int32_t normal, int32_t max_retries, uint32_t op, int32_t xop,
                                            uint64_t seed, uint32_t round_, int64_t cand_base, int64_t m,
                                            double* __restrict__ out, int64_t ldo, uint8_t* __restrict__ invalid,
                                            double* __restrict__ ws, int64_t ldw, int32_t perm_cols) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= m) return;
  const uint64_t g = (uint64_t)(cand_base + i);
  const u32x4 rc = draw(seed, g, STREAM_CAND | 0u, round_, op);
  const bool two = u01_from(rc.x, rc.y) < crossover_rate;
  const double* p2row = parent2 ? parent2 : parent1;  // select() twice returns the same best config
  const uint32_t sub2 = 3u;  // random second parent (both parents NULL)
  const int32_t scr_col = 2 * perm_cols;
  double chosen = 0.0, sel = 0.0;
  bool diff1 = false, diff2 = false;
  // one parameter of mutation attempt r: PERM in place in `out`, the other
  // kinds on v, stored when mutated or when `fresh` (attempt 0 runs fused with
  // the parent copy, so the copy is stored once and never read back)
  auto attempt = [&](const DevParam& pr, int32_t p, int32_t r, double v, bool fresh) {
    const uint32_t sp = (uint32_t)p | ((uint32_t)r << STREAM_RETRY_SHIFT);
    const u32x4 q = draw(seed, g, sp, round_, op);
    bool mut = false;
    if ((double)(P - p) * u01_from(q.x, q.y) < (double)must - sel) {
      sel += 1.0;
      mut = true;
    }
    mut = mut || (u01_from(q.z, q.w) < mutation_rate);
    if (pr.kind == UT_PERM) {
      const int32_t S = pr.psize;
      WRow o{out + (int64_t)pr.col * ldo + i, ldo};
      if (mut) {
        // uniform: op1_randomize; normal: random.choice(manipulators) =
        // [op1_randomize, op1_small_random_change]
        PermRng R(seed, g, sp | (1u << STREAM_SUB_SHIFT), round_, op);
        bool small = false;
        if (normal) {
          const u32x4 qc = draw(seed, g, sp | (1u << STREAM_SUB_SHIFT), round_, op);
          small = below64(u64_from(qc.z, qc.w), 2) == 1;
        }
        if (small) perm_small_change(o, S, R);
        else perm_shuffle(o, S, R);
      }
      const PRow a = parent_perm(pr, parent1, p, 2u, seed, g, round_, op, ws + (int64_t)pr.wcol * ldw + i, ldw, false);
      const PRow b = parent_perm(pr, p2row, p, sub2, seed, g, round_, op,
                                 ws + (int64_t)(perm_cols + pr.wcol) * ldw + i, ldw, false);
      diff1 |= !perm_equal(o.ro(), a, S);
      diff2 |= !perm_equal(o.ro(), b, S);
      return;
    }
    if (mut) {
      if (normal && is_primitive(pr.kind)) {
        // op1_normal_mutation (manipulator.py:505-521)
        double u = unit_of(pr, v, vtab);
        const double z = normal_draw(seed, g, sp | (2u << STREAM_SUB_SHIFT), round_, op);
        u = u + (0.0 + z * sigma);
        if (u < 0.0) u = u * -1.0;
        if (u > 1.0) u = 1.0 - fmod(u, 1.0);
        v = from_unit(pr, u, v);
      } else if (normal && pr.kind == UT_BOOL) {
        v = 1.0 - v;  // op1_flip
      } else {
        v = randomize(pr, draw(seed, g, sp | (1u << STREAM_SUB_SHIFT), round_, op));
      }
    }
    if (mut || fresh) out[(int64_t)pr.col * ldo + i] = v;
    const double a = parent_value(pr, parent1, p, 2u, seed, g, round_, op);
    const double b = parent_value(pr, p2row, p, sub2, seed, g, round_, op);
    diff1 |= d_to_bits(v) != d_to_bits(a);
    diff2 |= d_to_bits(v) != d_to_bits(b);
  };
  // the child (parent 1, the GGA crossover from parent 2, the GA crossover of
  // permutations) and, in the same pass, mutation attempt 0
  for (int32_t p = 0; p < P; ++p) {
    const DevParam pr = params[p];
    bool from2 = false;
    if (d_cross > 0 && two) {
      const u32x4 q = draw(seed, g, (uint32_t)p | (4u << STREAM_SUB_SHIFT), round_, op);
      if ((double)(P - p) * u01_from(q.x, q.y) < (double)d_cross - chosen) {
        chosen += 1.0;
        from2 = true;
      }
    }
    if (pr.kind == UT_PERM) {
      const int32_t S = pr.psize;
      const PRow a = parent_perm(pr, parent1, p, 2u, seed, g, round_, op, ws + (int64_t)pr.wcol * ldw + i, ldw, true);
      const PRow b = parent_perm(pr, p2row, p, sub2, seed, g, round_, op,
                                 ws + (int64_t)(perm_cols + pr.wcol) * ldw + i, ldw, true);
      WRow o{out + (int64_t)pr.col * ldo + i, ldo};
      if (from2) {
        perm_copy(o, b, S);
      } else if (two && xop != X_NONE && S > 6) {
        PermRng R(seed, g, (uint32_t)p | (5u << STREAM_SUB_SHIFT), round_, op);
        perm_cross(xop, o, a, b, S, S / 3, WRow{ws + (int64_t)scr_col * ldw + i, ldw}, R);
      } else {
        perm_copy(o, a, S);
      }
      attempt(pr, p, 0, 0.0, false);
      continue;
    }
    double v = parent_value(pr, parent1, p, 2u, seed, g, round_, op);
    if (from2) v = parent_value(pr, p2row, p, sub2, seed, g, round_, op);
    attempt(pr, p, 0, v, true);
  }
  bool accepted = diff1 && (!two || diff2);
  for (int32_t r = 1; r < max_retries && !accepted; ++r) {
    diff1 = diff2 = false;
    sel = 0.0;
    for (int32_t p = 0; p < P; ++p) {
      const DevParam pr = params[p];
      attempt(pr, p, r, pr.kind == UT_PERM ? 0.0 : out[(int64_t)pr.col * ldo + i], false);
    }
    accepted = diff1 && (!two || diff2);
  }
  if (invalid) invalid[i] = accepted ? 0 : 1;
}

// workspace of the PERM operators: GA parents + crossover scratch, [slot][ldw]
static int perm_workspace(ut_ctx* c, int64_t m, double** ws, int64_t* ldw) {
  const Space& s = c->space;
  *ws = nullptr;
  *ldw = 0;
  if (s.n_perm == 0) return 0;
  const int64_t l = ((m + 63) / 64) * 64;
  const int64_t slots = 2 * (int64_t)s.perm_cols + 3 * (int64_t)s.perm_smax;
  int rc = ensure(c, c->perm_ws, (size_t)(slots * l));
  if (rc) return rc;
  *ws = c->perm_ws.p;
  *ldw = l;
  return 0;
}

int launch_population_init(ut_ctx* c, uint32_t round_) {
  hipLaunchKernelGGL(k_population_init, dim3(grid1(c->npop, 256)), dim3(256), 0, c->stream, c->space.d_params,
                     c->space.P, c->pop, c->npop, c->npop, c->seed, round_);
  UT_LAUNCH_CHECK(c);
  return 0;
}

// the donor copy's value of column col: unit_of for a primitive param's
// column, the raw value otherwise (complex params, PERM item columns)
__device__ __forceinline__ double aos_value(const DevParam* __restrict__ params, const int32_t* __restrict__ col_param,
                                            const double* __restrict__ vtab, int32_t col, double v) {
  const int32_t pp = col_param[col];
  if (pp < 0) return v;
  const DevParam& pr = params[pp];
  return is_primitive(pr.kind) ? unit_of(pr, v, vtab) : v;
}

// pop (column-major [ncols][ldp]) -> aos (member-major [npop][lda], donor
// values): 64 members x 16 columns per 256-thread block through an LDS tile,
// coalesced on both sides (64-member runs read, 128-B member lines written)
__global__ __launch_bounds__(256) void k_pop_to_aos(const DevParam* __restrict__ params,
                                                    const int32_t* __restrict__ col_param,
                                                    const double* __restrict__ vtab, int32_t NC,
                                                    const double* __restrict__ pop, int64_t ldp, int64_t npop,
                                                    double* __restrict__ aos, int64_t lda) {
  __shared__ double tile[64][17];
  const int t = threadIdx.x;
  const int64_t m0 = (int64_t)blockIdx.x * 64;
  const int32_t c0 = blockIdx.y * 16;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int idx = t + 256 * r, cl = idx >> 6, ml = idx & 63;
    const int64_t mem = m0 + ml;
    const int32_t col = c0 + cl;
    tile[ml][cl] = (mem < npop && col < NC) ? aos_value(params, col_param, vtab, col, pop[(int64_t)col * ldp + mem])
                                            : 0.0;
  }
  __syncthreads();
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int idx = t + 256 * r, ml = idx >> 4, cl = idx & 15;
    const int64_t mem = m0 + ml;
    if (mem < npop) aos[mem * lda + c0 + cl] = tile[ml][cl];
  }
}

// aos rows idx[j] = donor values of trial column j (after ut_population_replace)
__global__ void k_pop_aos_rows(const DevParam* __restrict__ params, const int32_t* __restrict__ col_param,
                               const double* __restrict__ vtab, int32_t NC, double* __restrict__ aos, int64_t lda,
                               const double* __restrict__ trial, int64_t ld, const int64_t* __restrict__ idx,
                               int64_t n) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n * NC) return;
  const int64_t j = e / NC;
  const int32_t p = (int32_t)(e - j * NC);
  aos[idx[j] * lda + p] = aos_value(params, col_param, vtab, p, trial[(int64_t)p * ld + j]);
}

int ensure_pop_aos(ut_ctx* c) {
  if (c->pop_aos_valid) return 0;
  const int64_t lda = pop_aos_ld(c);
  const int64_t need = (c->npop + 1) * lda;   // + the best-config row
  if (c->pop_aos_cap < need) {
    if (c->pop_aos) {
      UT_HIP(c, sync_all(c));
      (void)ut::dfree(c->pop_aos);
      c->pop_aos = nullptr;
      c->pop_aos_cap = 0;
    }
    const hipError_t e = ut::dmalloc((void**)&c->pop_aos, sizeof(double) * need);
    if (e != hipSuccess) return set_err(c, UT_ENOMEM, std::string("ut::dmalloc(pop_aos): ") + hipGetErrorString(e));
    c->pop_aos_cap = need;
  }
  hipLaunchKernelGGL(k_pop_to_aos, dim3(grid1(c->npop, 64), (unsigned)(lda / 16)), dim3(256), 0, c->stream,
                     c->space.d_params, c->space.d_col_param, c->space.d_vtab, c->space.ncols, c->pop, c->npop,
                     c->npop, c->pop_aos, lda);
  UT_LAUNCH_CHECK(c);
  c->pop_aos_valid = true;
  return 0;
}

int launch_pop_aos_rows(ut_ctx* c, const double* trial, int64_t ld, const int64_t* idx, int64_t n) {
  const int64_t e = n * c->space.ncols;
  hipLaunchKernelGGL(k_pop_aos_rows, dim3(grid1(e, 256)), dim3(256), 0, c->stream, c->space.d_params,
                     c->space.d_col_param, c->space.d_vtab, c->space.ncols, c->pop_aos, pop_aos_ld(c), trial, ld, idx,
                     n);
  UT_LAUNCH_CHECK(c);
  return 0;
}

__global__ void k_aos_row(const DevParam* __restrict__ params, const int32_t* __restrict__ col_param,
                          const double* __restrict__ vtab, int32_t NC, const double* __restrict__ src,
                          double* __restrict__ dst) {
  const int32_t p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p < NC) dst[p] = aos_value(params, col_param, vtab, p, src[p]);
}

int launch_aos_row(ut_ctx* c, const double* src, int64_t row) {
  hipLaunchKernelGGL(k_aos_row, dim3(grid1(c->space.ncols, 64)), dim3(64), 0, c->stream, c->space.d_params,
                     c->space.d_col_param, c->space.d_vtab, c->space.ncols, src, c->pop_aos + row * pop_aos_ld(c));
  UT_LAUNCH_CHECK(c);
  return 0;
}

int launch_de(ut_ctx* c, const ut_de_params* p, uint32_t round_, int64_t cand_base, int64_t m, double* out,
              int64_t ld, bool diff) {
  const int32_t nw = (c->space.P + 31) / 32;
  // member-major donor gathers (k_de<., true>) up to 2048 params (cr-test bits in LDS)
  const bool aos = c->de_aos && nw <= 64;
  const int NT = aos ? 64 : 256;
  const unsigned grid = grid1(m, NT);
  size_t lds = sizeof(uint32_t) * (size_t)nw * NT + (aos ? sizeof(double) * DE_AOS_LDS_DBL : 0);
  uint32_t* xg = nullptr;
  if (nw > 64) {  // > 2048 params: the cr-test bits go to a global scratch
    const int rc = ensure(c, c->de_xbits, (size_t)nw * grid * NT);
    if (rc) return rc;
    xg = c->de_xbits.p;
    lds = 0;
  }
  const int64_t share = p->best ? (int64_t)p->information_sharing : (int64_t)0;
  int64_t lda = 0;
  if (aos) {
    const int rc = ensure_pop_aos(c);
    if (rc) return rc;
    lda = pop_aos_ld(c);
    if (share) {   // row npop: the best config, the donor of pool positions >= npop - 1
      const int rc = launch_aos_row(c, p->best, c->npop);
      if (rc) return rc;
    }
  }
  DeDiffOut dd{nullptr, nullptr, nullptr, 0};
  diff = diff && c->space.n_comp > 0;
  if (diff) {
    const int rc = ensure_de_diff(c, ld);
    if (rc) return rc;
    UT_HIP(c, hipMemsetAsync(c->r_npairs.p, 0, sizeof(int64_t), c->stream));
    dd = DeDiffOut{c->r_mask.p, c->r_pairs.p, reinterpret_cast<unsigned long long*>(c->r_npairs.p),
                   c->space.n_comp};
  }
  auto kern = aos ? (diff ? k_de<true, true> : k_de<false, true>) : (diff ? k_de<true, false> : k_de<false, false>);
  hipLaunchKernelGGL(kern, dim3(grid), dim3(NT), lds, c->stream, c->space.d_params, c->space.P, c->space.d_vtab,
                     c->pop, c->npop, c->npop, p->best, share, p->cr, p->n_cross, c->seed, round_, cand_base, m, out,
                     ld, dd, xg, c->pop_aos, lda);
  UT_LAUNCH_CHECK(c);
  return 0;
}

int launch_pso(ut_ctx* c, const ut_pso_params* a, const double* gbest, uint32_t round_, int64_t cand_base,
               int64_t m, double* out_x, double* out_v, int64_t ld) {
  const double* pb = a->alias_pbest ? c->pop : c->pso_best;
  double* ws;
  int64_t ldw;
  int rc = perm_workspace(c, m, &ws, &ldw);
  if (rc) return rc;
  hipLaunchKernelGGL(k_pso, dim3(grid1(m, 256)), dim3(256), 0, c->stream, c->space.d_params, c->space.P,
                     c->space.d_vtab, c->pop,
                     c->pso_vel, pb, c->npop, c->npop, gbest, a->omega, a->phi_g, a->phi_l, a->sigma, a->enum_mode,
                     a->crossover, c->seed, round_, cand_base, m, out_x, out_v, ld, ws, ldw, 2 * c->space.perm_cols);
  UT_LAUNCH_CHECK(c);
  return 0;
}

int launch_ga(ut_ctx* c, const ut_ga_params* a, const double* parent1, const double* parent2, uint32_t round_,
              int64_t cand_base, int64_t m, double* out, int64_t ld, uint8_t* invalid) {
  const int32_t d = (int32_t)(a->crossover_strength * (double)c->space.P);  // int(strength * len(params))
  double* ws;
  int64_t ldw;
  int rc = perm_workspace(c, m, &ws, &ldw);
  if (rc) return rc;
  hipLaunchKernelGGL(k_ga, dim3(grid1(m, 256)), dim3(256), 0, c->stream, c->space.d_params, c->space.P,
                     c->space.d_vtab, parent1,
                     parent2, a->mutation_rate, a->sigma, a->crossover_rate, d, a->must_mutate_count, a->normal,
                     a->max_retries, (uint32_t)a->op, a->crossover, c->seed, round_, cand_base, m, out, ld, invalid,
                     ws, ldw, c->space.perm_cols);
  UT_LAUNCH_CHECK(c);
  return 0;
}

int launch_encode(ut_ctx* c, const double* values, int64_t ld, int64_t m, double* feat, int64_t ldf) {
  hipLaunchKernelGGL(k_encode, dim3(grid1(m, 256)), dim3(256), 0, c->stream, c->space.d_params, c->space.P,
                     c->space.d_vtab, values, ld, m, feat, ldf);
  UT_LAUNCH_CHECK(c);
  return 0;
}

int launch_encode_scaled(ut_ctx* c, const double* values, int64_t ld, int64_t m, double* u, int32_t dpad, int64_t ldu,
                         double* cn) {
  hipLaunchKernelGGL(k_encode_scaled, dim3(grid1(ldu, 256)), dim3(256), 0, c->stream, c->space.d_params, c->space.P,
                     c->space.d_vtab, values, ld, m, c->space.n_feat, c->gp_inv_ell, dpad, u, ldu, cn);
  UT_LAUNCH_CHECK(c);
  return 0;
}

int launch_encode_scaled_cat(ut_ctx* c, const double* values, int64_t ld, int64_t m, double* u, int32_t dpad,
                             int64_t ldu, double* cn, int8_t* bcat) {
  const Space& s = c->space;
  UT_CHECK(c, ldu % 256 == 0 && s.cat_k % 128 == 0, UT_EINVAL, "encode_scaled_cat: bad padding");
  hipLaunchKernelGGL(k_encode_scaled_cat, dim3((unsigned)(ldu / 256)), dim3(256), code_rows_lds(s.cat_k), c->stream,
                     s.d_params, s.P, s.d_vtab, values, ld, m, s.d_feat_num, s.n_num, dpad, c->gp_inv_ell,
                     s.d_cat_ccol, s.cat_k, u, ldu, cn, bcat);
  UT_LAUNCH_CHECK(c);
  return 0;
}

int launch_gather_rows(ut_ctx* c, const double* values, int64_t ld, const int64_t* idx, int64_t cand_base,
                       int32_t k, double* out, int64_t ldo, const uint32_t* dig, uint32_t* out_dig) {
  hipLaunchKernelGGL(k_gather_rows, dim3(grid1(k, 64)), dim3(64), 0, c->stream, c->space.ncols, values, ld, idx,
                     cand_base, k, out, ldo, dig, out_dig);
  UT_LAUNCH_CHECK(c);
  return 0;
}

}  // namespace ut

extern "C" int ut_population_replace(ut_ctx* c, const double* trial, int64_t ld, const int64_t* idx, int64_t n) {
  if (!c) return UT_EINVAL;
  UT_CHECK(c, c->has_space, UT_ENOSPACE, "space not defined");
  UT_CHECK(c, c->pop != nullptr, UT_EINVAL, "population not initialised");
  if (n <= 0) return 0;
  hipLaunchKernelGGL(ut::k_pop_replace, dim3(ut::grid1(n, 64)), dim3(64), 0, c->stream, c->space.ncols, c->pop,
                     c->npop, trial, ld, idx, n);
  UT_LAUNCH_CHECK(c);
  if (c->pop_aos_valid) {
    const int rc = ut::launch_pop_aos_rows(c, trial, ld, idx, n);
    if (rc) return rc;
  }
  // keep the population's inner-digest cache current: only the replaced rows
  if (c->pop_dig_valid) return ut::launch_pop_digests(c, idx, n);
  return 0;
}

extern "C" int ut_pso_reset(ut_ctx* c) {
  if (!c) return UT_EINVAL;
  UT_CHECK(c, c->has_space && c->pop != nullptr, UT_EINVAL, "pso_reset: population not initialised");
  const int64_t need = c->npop * c->space.ncols;
  if (c->pso_cap < need) {
    if (c->pso_vel) {
      UT_HIP(c, ut::sync_all(c));
      ut::dfree(c->pso_vel);
      ut::dfree(c->pso_best);
    }
    UT_HIP(c, ut::dmalloc((void**)&c->pso_vel, sizeof(double) * need));
    UT_HIP(c, ut::dmalloc((void**)&c->pso_best, sizeof(double) * need));
    c->pso_cap = need;
  }
  UT_HIP(c, hipMemsetAsync(c->pso_vel, 0, sizeof(double) * need, c->stream));
  UT_HIP(c, hipMemcpyAsync(c->pso_best, c->pop, sizeof(double) * need, hipMemcpyDeviceToDevice, c->stream));
  return 0;
}

extern "C" int ut_propose_pso(ut_ctx* c, const ut_pso_params* a, const double* gbest, uint32_t round_,
                              int64_t cand_base, int64_t m, double* out_values, double* out_vel, int64_t ld) {
  if (!c) return UT_EINVAL;
  UT_CHECK(c, c->has_space && c->pop != nullptr, UT_EINVAL, "propose_pso: population not initialised");
  UT_CHECK(c, c->pso_vel != nullptr && c->pso_cap >= c->npop * c->space.ncols, UT_EINVAL,
           "propose_pso: call ut_pso_reset after (re)initialising the population");
  UT_CHECK(c, a && gbest && (out_values || m == 0) && m >= 0 && cand_base >= 0 && ld >= m, UT_EINVAL,
           "propose_pso: bad arguments");
  UT_CHECK(c, a->crossover >= UT_X_NONE && a->crossover <= UT_X_PMX, UT_EINVAL, "propose_pso: bad crossover");
  if (m == 0) return 0;
  // a staged fit is issued after the proposal (api.hip score_round_de_impl)
  int rc;
  if ((rc = ut::gp_fit_prefit(c))) return rc;
  if ((rc = ut::launch_pso(c, a, gbest, round_, cand_base, m, out_values, out_vel, ld))) return rc;
  return ut::gp_fit_flush(c);
}

extern "C" int ut_pso_commit(ut_ctx* c, const double* values, const double* vel, int64_t ld, int64_t cand_base,
                             int64_t m) {
  if (!c) return UT_EINVAL;
  UT_CHECK(c, c->pso_vel != nullptr && values && cand_base >= 0 && m >= 0 && cand_base + m <= c->npop && ld >= m,
           UT_EINVAL, "pso_commit: bad arguments");
  if (m == 0) return 0;
  c->pop_dig_valid = false;   // positions moved: the inner-digest cache is rebuilt when a DE round needs it
  c->pop_aos_valid = false;   // and so is the member-major copy
  UT_HIP(c, hipMemcpy2DAsync(c->pop + cand_base, sizeof(double) * c->npop, values, sizeof(double) * ld,
                             sizeof(double) * m, c->space.ncols, hipMemcpyDeviceToDevice, c->stream));
  if (vel)
    UT_HIP(c, hipMemcpy2DAsync(c->pso_vel + cand_base, sizeof(double) * c->npop, vel, sizeof(double) * ld,
                               sizeof(double) * m, c->space.ncols, hipMemcpyDeviceToDevice, c->stream));
  return 0;
}

extern "C" int ut_pso_update_best(ut_ctx* c, const double* values, int64_t ld, const int64_t* idx, int64_t n) {
  if (!c) return UT_EINVAL;
  UT_CHECK(c, c->pso_best != nullptr && values && idx && n >= 0, UT_EINVAL, "pso_update_best: bad arguments");
  if (n == 0) return 0;
  hipLaunchKernelGGL(ut::k_pop_replace, dim3(ut::grid1(n, 64)), dim3(64), 0, c->stream, c->space.ncols, c->pso_best,
                     c->npop, values, ld, idx, n);
  UT_LAUNCH_CHECK(c);
  return 0;
}

extern "C" int ut_propose_ga(ut_ctx* c, const ut_ga_params* a, const double* parent1, const double* parent2,
                             uint32_t round_, int64_t cand_base, int64_t m, double* out_values, int64_t ld,
                             uint8_t* out_invalid) {
  if (!c) return UT_EINVAL;
  UT_CHECK(c, c->has_space, UT_ENOSPACE, "space not defined");
  UT_CHECK(c, a && (out_values || m == 0) && m >= 0 && cand_base >= 0 && ld >= m, UT_EINVAL, "propose_ga: bad arguments");
  UT_CHECK(c, a->max_retries >= 1 && a->max_retries <= 15, UT_EINVAL, "propose_ga: max_retries must be in [1, 15]");
  UT_CHECK(c, a->must_mutate_count >= 0 && a->must_mutate_count <= c->space.P, UT_EINVAL,
           "propose_ga: must_mutate_count out of range");
  UT_CHECK(c, a->op >= 0 && a->op < 256, UT_EINVAL, "propose_ga: op must fit 8 bits");
  UT_CHECK(c, a->crossover >= UT_X_NONE && a->crossover <= UT_X_PMX, UT_EINVAL, "propose_ga: bad crossover");
  if (m == 0) return 0;
  int rc;
  if ((rc = ut::gp_fit_prefit(c))) return rc;
  if ((rc = ut::launch_ga(c, a, parent1, parent2, round_, cand_base, m, out_values, ld, out_invalid))) return rc;
  return ut::gp_fit_flush(c);
}
