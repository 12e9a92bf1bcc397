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
#include "ut_internal.h"

namespace ut {

__device__ __forceinline__ bool is_primitive(int kind) { return kind <= UT_POW2; }

// get_unit_value (manipulator.py:473-488)
__device__ __forceinline__ double unit_of(const DevParam& pr, double v) {
  if (pr.u_lo < pr.u_hi) return __ddiv_rn(__dsub_rn(v, pr.u_lo), pr.u_span);
  return 0.0;
}

// set_unit_value (manipulator.py:490-503); returns the new stored value, or
// `keep` when the range is a single point (the reference leaves it alone).
__device__ __forceinline__ double from_unit(const DevParam& pr, double u, double keep) {
  if (!(pr.u_lo < pr.u_hi)) return keep;
  double val = __dadd_rn(__dmul_rn(u, pr.u_span), pr.u_lo);
  if (pr.kind == UT_INT) val = rint(val);  // Python round(): half-to-even
  val = py_max(pr.u_lo, py_min(val, pr.u_hi));
  if (pr.kind == UT_INT) val = trunc(val);  // int(val)
  return val;
}

// op1_randomize for one parameter from one 4x32 draw
__device__ __forceinline__ double randomize(const DevParam& pr, u32x4 r) {
  switch (pr.kind) {
    case UT_FLOAT: {
      // random.uniform(a, b) = a + (b - a) * random()
      const double u = u01_from(r.x, r.y);
      return __dadd_rn(pr.lo, __dmul_rn(__dsub_rn(pr.hi, pr.lo), u));
    }
    case UT_INT: {
      // random.randint(lo, hi)
      const int64_t lo = (int64_t)pr.lo, hi = (int64_t)pr.hi;
      return (double)(lo + (int64_t)below64(u64_from(r.z, r.w), (uint64_t)(hi - lo + 1)));
    }
    case UT_BOOL:
      // random.choice((True, False))
      return below64(u64_from(r.z, r.w), 2) == 0 ? 1.0 : 0.0;
    case UT_ENUM:
      // random.choice(self.options) -> option index
      return (double)below64(u64_from(r.z, r.w), (uint64_t)pr.n_opt);
    default:
      return 0.0;
  }
}

__global__ __launch_bounds__(256) void k_population_init(const DevParam* __restrict__ params, int32_t P,
                                                         double* __restrict__ pop, int64_t ld, int64_t npop,
                                                         uint64_t seed, uint32_t round_) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= npop) return;
  for (int32_t p = 0; p < P; ++p) {
    const DevParam pr = params[p];
    const u32x4 r = draw(seed, (uint64_t)i, (uint32_t)p, round_, OP_INIT);
    pop[(int64_t)p * ld + i] = randomize(pr, r);
  }
}

// Sample 3 distinct population members other than `t` (the reference draws
// x1,x2,x3 from shuffle(set(population) - {target}),
// differentialevolution.py:109-118).
__device__ __forceinline__ void pick_donors(uint32_t w0, uint32_t w1, uint32_t w2, int64_t npop, int64_t t,
                                            int64_t& d1, int64_t& d2, int64_t& d3) {
  int64_t a = (int64_t)umulhi32(w0, (uint32_t)(npop - 1));
  d1 = a + (a >= t ? 1 : 0);
  int64_t e0 = t < d1 ? t : d1, e1 = t < d1 ? d1 : t;
  int64_t b = (int64_t)umulhi32(w1, (uint32_t)(npop - 2));
  if (b >= e0) ++b;
  if (b >= e1) ++b;
  d2 = b;
  // sort {t, d1, d2}
  int64_t s0 = e0, s1 = e1, s2 = d2;
  if (s2 < s1) { int64_t x = s1; s1 = s2; s2 = x; }
  if (s1 < s0) { int64_t x = s0; s0 = s1; s1 = x; }
  int64_t c = (int64_t)umulhi32(w2, (uint32_t)(npop - 3));
  if (c >= s0) ++c;
  if (c >= s1) ++c;
  if (c >= s2) ++c;
  d3 = c;
}

// One DE trial per candidate.  Candidate g (global) targets member g % npop.
// Forced crossover set = the n_cross parameters with the smallest per-param
// random keys (= the first n_cross names of a uniform shuffle,
// differentialevolution.py:122-125).
__global__ __launch_bounds__(256) void k_de(const DevParam* __restrict__ params, int32_t P,
                                            const double* __restrict__ pop, int64_t ldp, int64_t npop,
                                            double cr, int32_t n_cross, uint64_t seed, uint32_t round_,
                                            int64_t cand_base, int64_t m, double* __restrict__ out,
                                            int64_t ldo) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= m) return;
  const uint64_t g = (uint64_t)(cand_base + i);
  const int64_t t = (int64_t)(g % (uint64_t)npop);
  const u32x4 rc = draw(seed, g, STREAM_CAND | 0u, round_, OP_DE);
  int64_t d1, d2, d3;
  pick_donors(rc.x, rc.y, rc.z, npop, t, d1, d2, d3);
  const u32x4 rf = draw(seed, g, STREAM_CAND | 1u, round_, OP_DE);
  // use_f = old_div(random.random(), 2.0) + 0.5
  const double F = __dadd_rn(__ddiv_rn(u01_from(rf.x, rf.y), 2.0), 0.5);
  const double nF = -F;

  // forced set: up to 4 smallest (key, p)
  uint64_t fk[4] = {~0ull, ~0ull, ~0ull, ~0ull};
  if (n_cross > 0) {
    for (int32_t p = 0; p < P; ++p) {
      const u32x4 r = draw(seed, g, (uint32_t)p, round_, OP_DE);
      uint64_t key = ((uint64_t)r.z << 32) | (uint32_t)p;
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        if (s < n_cross && key < fk[s]) {
          uint64_t x = fk[s]; fk[s] = key; key = x;
        }
      }
    }
  }

  for (int32_t p = 0; p < P; ++p) {
    const DevParam pr = params[p];
    const u32x4 r = draw(seed, g, (uint32_t)p, round_, OP_DE);
    bool forced = false;
#pragma unroll
    for (int s = 0; s < 4; ++s) forced |= (s < n_cross) && ((uint32_t)fk[s] == (uint32_t)p) && (fk[s] != ~0ull);
    const double* col = pop + (int64_t)p * ldp;
    const double vt = col[t];
    double v = vt;
    // `i < n_cross or random() < cr` (short-circuit: the draw is only
    // consulted for non-forced params, which is what selecting on it does)
    if (forced || u01_from(r.x, r.y) < cr) {
      const double x1 = col[d1], x2 = col[d2], x3 = col[d3];
      if (is_primitive(pr.kind)) {
        const double va = unit_of(pr, x1), vb = unit_of(pr, x2), vc = unit_of(pr, x3);
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
    out[(int64_t)p * ldo + i] = v;
  }
}

// GP features of a configuration.
__global__ __launch_bounds__(256) void k_encode(const DevParam* __restrict__ params, int32_t P,
                                                const double* __restrict__ values, int64_t ld, int64_t m,
                                                double* __restrict__ feat, int64_t ldf) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= m) return;
  for (int32_t p = 0; p < P; ++p) {
    const DevParam pr = params[p];
    const double v = values[(int64_t)p * ld + i];
    if (is_primitive(pr.kind)) {
      feat[(int64_t)pr.feat_col * ldf + i] = unit_of(pr, v);
    } else if (pr.kind == UT_BOOL) {
      feat[(int64_t)pr.feat_col * ldf + i] = v;
    } else {
      const int64_t o = (int64_t)v;
      for (int64_t k = 0; k < pr.n_opt; ++k) feat[(int64_t)(pr.feat_col + k) * ldf + i] = (k == o) ? 1.0 : 0.0;
    }
  }
}

__global__ void k_gather_rows(int32_t P, const double* __restrict__ values, int64_t ld,
                              const int64_t* __restrict__ idx, int64_t cand_base, int32_t k,
                              double* __restrict__ out, int64_t ldo, const uint32_t* __restrict__ dig,
                              uint32_t* __restrict__ out_dig) {
  const int32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= k) return;
  const int64_t g = idx[j];
  const int64_t i = g - cand_base;
  for (int32_t p = 0; p < P; ++p) out[(int64_t)p * ldo + j] = (g >= 0) ? values[(int64_t)p * ld + i] : 0.0;
  if (out_dig) {
    for (int w = 0; w < 8; ++w) out_dig[(int64_t)j * 8 + w] = (g >= 0) ? dig[i * 8 + w] : 0u;
  }
}

__global__ void k_pop_replace(int32_t P, double* __restrict__ pop, int64_t ldp, const double* __restrict__ trial,
                              int64_t ld, const int64_t* __restrict__ idx, int64_t n) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  const int64_t dst = idx[j];
  for (int32_t p = 0; p < P; ++p) pop[(int64_t)p * ldp + dst] = trial[(int64_t)p * ld + j];
}

int launch_population_init(ut_ctx* c, uint32_t round_) {
  hipLaunchKernelGGL(k_population_init, dim3(grid1(c->npop, 256)), dim3(256), 0, c->stream, c->space.d_params,
                     c->space.P, c->pop, c->npop, c->npop, c->seed, round_);
  UT_LAUNCH_CHECK(c);
  return 0;
}

int launch_de(ut_ctx* c, const ut_de_params* p, uint32_t round_, int64_t cand_base, int64_t m, double* out,
              int64_t ld) {
  hipLaunchKernelGGL(k_de, dim3(grid1(m, 256)), dim3(256), 0, c->stream, c->space.d_params, c->space.P, c->pop,
                     c->npop, c->npop, p->cr, p->n_cross, c->seed, round_, cand_base, m, out, ld);
  UT_LAUNCH_CHECK(c);
  return 0;
}

int launch_encode(ut_ctx* c, const double* values, int64_t ld, int64_t m, double* feat, int64_t ldf) {
  hipLaunchKernelGGL(k_encode, dim3(grid1(m, 256)), dim3(256), 0, c->stream, c->space.d_params, c->space.P,
                     values, ld, m, feat, ldf);
  UT_LAUNCH_CHECK(c);
  return 0;
}

int launch_gather_rows(ut_ctx* c, const double* values, int64_t ld, const int64_t* idx, int64_t cand_base,
                       int32_t k, double* out, int64_t ldo, const uint32_t* dig, uint32_t* out_dig) {
  hipLaunchKernelGGL(k_gather_rows, dim3(grid1(k, 64)), dim3(64), 0, c->stream, c->space.P, values, ld, idx,
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
  hipLaunchKernelGGL(ut::k_pop_replace, dim3(ut::grid1(n, 64)), dim3(64), 0, c->stream, c->space.P, c->pop,
                     c->npop, trial, ld, idx, n);
  UT_LAUNCH_CHECK(c);
  return 0;
}
