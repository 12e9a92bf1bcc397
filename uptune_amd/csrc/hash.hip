// hash.hip -- batched ConfigurationManipulator.hash_config on gfx950.
//
// Reference (manipulator.py:233-243, :456-459, :855-858):
//   m = sha256()
//   for i, p in enumerate(sorted(params, key=name)):
//     m.update(str(p.name)); m.update(str(p.hash_value(cfg))); m.update(str(i)); m.update(b"|")
// where hash_value is sha256(repr(value)).hexdigest() -- wrapped as "b'...'"
// for primitive params by uptune's Python-3 port (str() of a bytes object).
//
// For a given space the outer message has a FIXED length: only the 64 hex
// characters of each inner digest vary.  The host therefore compiles the
// message into a table of 32-bit words (constant template bits + which hex
// "hole" overlaps the word and at what byte shift); the kernel streams the
// outer SHA-256 blocks word by word, producing each parameter's inner digest
// just before its hole is first needed.
//
// Inner digests: discrete values (ENUM, BOOL, POW2 exponents, small-range
// INT and LOGINT) come from a host-built LUT; FLOAT values are formatted on
// the device with Python's shortest round-trip repr (ut_core.h) and hashed
// (one SHA-256 block); large-range INT values use repr(int), large-range
// LOGINT values repr of the device's correctly rounded log2.
//
// One lane = one candidate.  The repr byte string is assembled in LDS in
// [word][lane] layout (bank-conflict-free, no cross-lane traffic, so no
// barriers); the two live 64-char hex "holes" stay in one 32-register array
// indexed by the wave-uniform word-table entry (s_set_gpr_idx / v_movrels, no
// scratch, no per-word selects).  The word table is read with scalar loads;
// parameter values are prefetched one parameter ahead.  Bound: integer VALU
// (~1.45k ops per SHA-256 compression, Sigma/Ch/Maj as single v_bitop3_b32;
// the 3-source ops issue at half rate, so ~28.5 G compressions/s is the
// measured chip ceiling, scripts/exp/sha_rate.hip).
#include "ut_param.h"

namespace ut {

constexpr int HASH_NT = 128;
constexpr int SCR_WORDS = 7;                       // inner message bytes 0..27

typedef uint32_t hex32 __attribute__((ext_vector_type(32)));

struct LdsEmit {
  uint8_t* base;  // &lds[0] as bytes
  int lane;
  __device__ __forceinline__ void put(int pos, uint8_t ch) {
    base[(((pos >> 2) * HASH_NT + lane) << 2) + (pos & 3)] = ch;
  }
};

// sha256(repr(value)) for the non-LUT modes: the repr bytes are assembled in
// this lane's LDS column, then one SHA-256 block
__device__ __forceinline__ void repr_digest(const DevParam& pr, double v, uint32_t* lds, int lane, uint32_t D[8]) {
#pragma unroll
  for (int w = 0; w < SCR_WORDS; ++w) lds[w * HASH_NT + lane] = 0u;
  LdsEmit e{reinterpret_cast<uint8_t*>(lds), lane};
  int len;
  if (pr.hash_mode == HM_FLOAT) len = repr_double(v, e);
  else if (pr.hash_mode == HM_LOGINT) len = repr_double(py_log2(__dsub_rn(__dadd_rn(v, 1.0), pr.lo)), e);
  else len = repr_int64((int64_t)v, e);
  e.put(len, 0x80);
  uint32_t W[16];
#pragma unroll
  for (int w = 0; w < SCR_WORDS; ++w) W[w] = __builtin_bswap32(lds[w * HASH_NT + lane]);
#pragma unroll
  for (int w = SCR_WORDS; w < 15; ++w) W[w] = 0u;
  W[15] = (uint32_t)len * 8u;
  sha256_init(D);
  sha256_compress(D, W);
}

// LUT row of a discrete value (the host hashed repr(get_value) of every value)
__device__ __forceinline__ int64_t lut_row(const DevParam& pr, double v) {
  int64_t idx;
  if (pr.kind == UT_ENUM || pr.kind == UT_BOOL) idx = (int64_t)v;
  else if (pr.kind == UT_POW2) idx = (int64_t)(pow2_exponent(v) - pr.lo);  // repr(exponent)
  else idx = (int64_t)(v - pr.lo);                                       // INT, LOGINT
  idx = idx < 0 ? 0 : (idx >= pr.lut_n ? pr.lut_n - 1 : idx);  // never fault on garbage input
  return pr.lut_base + idx;
}

__global__ __launch_bounds__(HASH_NT) void k_hash(const DevParam* __restrict__ params,
                                                  const int32_t* __restrict__ order,
                                                  const uint2* __restrict__ words,
                                                  const int32_t* __restrict__ block_last, int32_t nblocks,
                                                  int32_t P, const uint4* __restrict__ lut,
                                                  const double* __restrict__ values, int64_t ld, int64_t m,
                                                  uint32_t* __restrict__ out) {
  __shared__ uint32_t lds[SCR_WORDS * HASH_NT];
  const int lane = threadIdx.x;
  const int64_t i0 = (int64_t)blockIdx.x * HASH_NT + lane;
  const bool valid = i0 < m;
  const int64_t i = valid ? i0 : (m - 1);
  hex32 HX = {};  // two 16-word hex slots: hole j in HX[16 (j % 2) .. 16 (j % 2) + 15]
  uint32_t H[8];
  sha256_init(H);
  int32_t next = 0;
  // the value of the next parameter to digest is loaded one parameter ahead
  double vnext = values[(int64_t)order[0] * ld + i];
  for (int32_t b = 0; b < nblocks; ++b) {
    const int32_t last = block_last[b];
    while (next <= last) {
      const int32_t p = order[next];
      const DevParam pr = params[p];
      const double v = vnext;
      uint32_t D[8];
      if (pr.hash_mode == HM_LUT) {
        const uint4* src = lut + 2 * lut_row(pr, v);
        const uint4 a = src[0], c = src[1];  // issued before the prefetch: waits leave it in flight
        if (next + 1 < P) vnext = values[(int64_t)order[next + 1] * ld + i];
        D[0] = a.x; D[1] = a.y; D[2] = a.z; D[3] = a.w;
        D[4] = c.x; D[5] = c.y; D[6] = c.z; D[7] = c.w;
      } else {
        if (next + 1 < P) vnext = values[(int64_t)order[next + 1] * ld + i];
        repr_digest(pr, v, lds, lane, D);
      }
      // 64 hex characters as 16 big-endian words into slot next % 2
      if (next & 1) {
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          HX[16 + 2 * k] = hex4(D[k] >> 16);
          HX[16 + 2 * k + 1] = hex4(D[k] & 0xFFFFu);
        }
      } else {
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          HX[2 * k] = hex4(D[k] >> 16);
          HX[2 * k + 1] = hex4(D[k] & 0xFFFFu);
        }
      }
      ++next;
    }
    uint32_t W[16];
    const uint2* hw = words + (int64_t)b * 16;
#pragma unroll
    for (int w = 0; w < 16; ++w) {
      const uint2 e = hw[w];  // scalar load: the same word for every lane
      uint32_t x = e.x;
      if (e.y) {
        const uint32_t lo = (e.y & HW_LO_VALID) ? HX[e.y & 31u] : 0u;
        const uint32_t hi = (e.y & HW_HI_VALID) ? HX[(e.y >> HW_HI_POS) & 31u] : 0u;
        const uint64_t cat = ((uint64_t)lo << 32) | hi;
        x |= (uint32_t)((cat << ((e.y >> HW_SHIFT_POS) & 31u)) >> 32);
      }
      W[w] = x;
    }
    sha256_compress(H, W);
  }
  if (valid) {
    uint4* dst = reinterpret_cast<uint4*>(out + i * 8);
    dst[0] = make_uint4(H[0], H[1], H[2], H[3]);
    dst[1] = make_uint4(H[4], H[5], H[6], H[7]);
  }
}

int launch_hash(ut_ctx* c, const double* values, int64_t ld, int64_t m, uint32_t* out) {
  if (m <= 0) return 0;
  const Space& s = c->space;
  hipLaunchKernelGGL(k_hash, dim3(grid1(m, HASH_NT)), dim3(HASH_NT), 0, c->stream, s.d_params, s.d_order,
                     reinterpret_cast<const uint2*>(s.d_words), s.d_block_last, (int32_t)s.outer_blocks, s.P,
                     reinterpret_cast<const uint4*>(s.d_lut), values, ld, m, out);
  UT_LAUNCH_CHECK(c);
  return 0;
}

}  // namespace ut
