// ut_param.h -- per-kind value arithmetic of the parameter kinds on the
// device: the searched value (get_value), its unit encoding and the inverse.
// Bit-exact restatement of
//   get_unit_value        manipulator.py:473-488
//   set_unit_value        manipulator.py:490-503
//   op1_randomize         manipulator.py:596-606 (numeric), :940-949 (bool), :1033-1042 (enum)
//   ScaledNumericParameter.get_value/set_value   manipulator.py:747-775
//     LogIntegerParameter _scale/_unscale/legal_range  :778-797
//     PowerOfTwoParameter _scale/_unscale/legal_range  :811-836
// compiled with -ffp-contract=off, in Python's evaluation order.
#pragma once
#include "ut_internal.h"

namespace ut {

__device__ __forceinline__ bool is_primitive(int kind) { return kind <= UT_POW2; }
__device__ __forceinline__ bool is_integer_type(int kind) { return kind == UT_INT || kind == UT_POW2; }

// exponent of a stored power of two (exact)
__device__ __forceinline__ double pow2_exponent(double v) {
  return (double)((int32_t)((d_to_bits(v) >> 52) & 0x7FF) - 1023);
}

// get_value: the searched value of a stored value
//   LOGINT  math.log(v + 1.0 - min, 2.0)   (host CPython table when present)
//   POW2    int(math.log(v, 2)) == the exponent (exact for every power of two)
__device__ __forceinline__ double scaled_of(const DevParam& pr, double v, const double* __restrict__ vtab) {
  if (pr.kind == UT_LOGINT) {
    if (pr.vtab_n > 0) {
      int64_t k = (int64_t)(v - pr.lo);
      k = k < 0 ? 0 : (k >= pr.vtab_n ? pr.vtab_n - 1 : k);  // never fault on garbage input
      return vtab[pr.vtab_base + k];
    }
    return py_log2(__dsub_rn(__dadd_rn(v, 1.0), pr.lo));
  }
  if (pr.kind == UT_POW2) return pow2_exponent(v);
  return v;
}

// set_value of a searched value: the stored value
//   LOGINT  int(round(2.0 ** s - 1.0 + min))
//   POW2    2 ** int(s)
__device__ __forceinline__ double unscale(const DevParam& pr, double s) {
  if (pr.kind == UT_LOGINT) return rint(__dadd_rn(__dsub_rn(exp2_cr(s), 1.0), pr.lo));
  if (pr.kind == UT_POW2) return bits_to_d((uint64_t)((int64_t)s + 1023) << 52);
  return s;
}

// get_unit_value (manipulator.py:473-488)
__device__ __forceinline__ double unit_of(const DevParam& pr, double v, const double* __restrict__ vtab) {
  if (pr.u_lo < pr.u_hi) return __ddiv_rn(__dsub_rn(scaled_of(pr, v, vtab), pr.u_lo), pr.u_span);
  return 0.0;
}

// set_unit_value (manipulator.py:490-503); returns the new stored value, or
// `keep` when the range is a single point (the reference leaves it alone).
__device__ __forceinline__ double from_unit(const DevParam& pr, double u, double keep) {
  if (!(pr.u_lo < pr.u_hi)) return keep;
  double val = __dadd_rn(__dmul_rn(u, pr.u_span), pr.u_lo);
  const bool it = is_integer_type(pr.kind);
  if (it) val = rint(val);  // Python round(): half-to-even
  val = py_max(pr.u_lo, py_min(val, pr.u_hi));
  if (it) val = trunc(val);  // value_type(val) = int(val)
  return unscale(pr, val);
}

// op1_randomize for one parameter from one 4x32 draw
__device__ __forceinline__ double randomize(const DevParam& pr, u32x4 r) {
  switch (pr.kind) {
    case UT_FLOAT: {
      // random.uniform(a, b) = a + (b - a) * random()
      const double u = u01_from(r.x, r.y);
      return __dadd_rn(pr.lo, __dmul_rn(__dsub_rn(pr.hi, pr.lo), u));
    }
    case UT_LOGINT: {
      // set_value(random.uniform(*legal_range)) (not integer-typed: value_type float)
      const double u = u01_from(r.x, r.y);
      return unscale(pr, __dadd_rn(pr.u_lo, __dmul_rn(__dsub_rn(pr.u_hi, pr.u_lo), u)));
    }
    case UT_INT:
    case UT_POW2: {
      // set_value(random.randint(*legal_range))
      const int64_t lo = (int64_t)pr.lo, hi = (int64_t)pr.hi;
      return unscale(pr, (double)(lo + (int64_t)below64(u64_from(r.z, r.w), (uint64_t)(hi - lo + 1))));
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

}  // namespace ut
