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

// a digest as its 64 hex characters: 16 big-endian words, 4 x 16-B stores
__device__ __forceinline__ void store_hex(uint4* dst, const uint32_t D[8]) {
  uint32_t X[16];
  digest_hex(D, X);
  dst[0] = make_uint4(X[0], X[1], X[2], X[3]);
  dst[1] = make_uint4(X[4], X[5], X[6], X[7]);
  dst[2] = make_uint4(X[8], X[9], X[10], X[11]);
  dst[3] = make_uint4(X[12], X[13], X[14], X[15]);
}
constexpr int SCR_WORDS = 7;                       // inner message bytes 0..27

typedef uint32_t hex32 __attribute__((ext_vector_type(32)));

template <int NT>
struct LdsEmitN {
  uint8_t* base;  // &lds[0] as bytes
  int lane;
  __device__ __forceinline__ void put(int pos, uint8_t ch) {
    base[(((pos >> 2) * NT + lane) << 2) + (pos & 3)] = ch;
  }
};
using LdsEmit = LdsEmitN<HASH_NT>;

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

// sha256(repr(list of items)) of every PERM param: "[" + ", ".join(repr(item))
// + "]" streamed through a 64-byte block in this lane's LDS column.  The
// message length is constant per param (a permutation of fixed items).
constexpr int PD_NT = 128;

__global__ __launch_bounds__(PD_NT) void k_perm_digest(const DevParam* __restrict__ params,
                                                       const int32_t* __restrict__ perm_params, int32_t n_perm,
                                                       const uint8_t* __restrict__ bytes,
                                                       const int32_t* __restrict__ off,
                                                       const int32_t* __restrict__ offbase,
                                                       const int32_t* __restrict__ msg_len,
                                                       const double* __restrict__ values, int64_t ld, int64_t m,
                                                       uint32_t* __restrict__ out) {
  __shared__ uint32_t lds[16 * PD_NT];
  const int lane = threadIdx.x;
  const int64_t i = (int64_t)blockIdx.x * PD_NT + lane;
  if (i >= m) return;  // no barriers below: every lane owns its LDS column
  LdsEmitN<PD_NT> e{reinterpret_cast<uint8_t*>(lds), lane};
  for (int32_t q = 0; q < n_perm; ++q) {
    const DevParam pr = params[perm_params[q]];
    const int32_t S = pr.psize;
    const int32_t* o = off + offbase[q];
    uint32_t H[8];
    sha256_init(H);
#pragma unroll
    for (int w = 0; w < 16; ++w) lds[w * PD_NT + lane] = 0u;
    int32_t fill = 0;
    auto flush = [&]() {
      uint32_t W[16];
#pragma unroll
      for (int w = 0; w < 16; ++w) {
        W[w] = __builtin_bswap32(lds[w * PD_NT + lane]);
        lds[w * PD_NT + lane] = 0u;
      }
      sha256_compress(H, W);
      fill = 0;
    };
    auto emit = [&](uint8_t ch) {
      e.put(fill, ch);
      if (++fill == 64) flush();
    };
    emit('[');
    for (int32_t k = 0; k < S; ++k) {
      if (k > 0) { emit(','); emit(' '); }
      int32_t item = (int32_t)values[(int64_t)(pr.col + k) * ld + i];
      item = item < 0 ? 0 : (item >= S ? S - 1 : item);  // never fault on garbage input
      for (int32_t b = o[item]; b < o[item + 1]; ++b) emit(bytes[b]);
    }
    emit(']');
    emit(0x80);
    if (fill > 56) {
      while (fill != 0) emit(0);
    }
    while (fill < 56) emit(0);
    const uint64_t bits = (uint64_t)msg_len[q] * 8u;
    for (int b = 7; b >= 0; --b) emit((uint8_t)(bits >> (8 * b)));  // completes (and flushes) the block
    uint4* dst = reinterpret_cast<uint4*>(out + ((int64_t)q * m + i) * 8);
    dst[0] = make_uint4(H[0], H[1], H[2], H[3]);
    dst[1] = make_uint4(H[4], H[5], H[6], H[7]);
  }
}

// ---------------------------------------------------------------------------
// Inner-digest reuse for DE rounds.  A DE trial copies its target member's
// value for every parameter it does not cross (differentialevolution.py:122-127:
// with cr = 0.2 and n_cross = 1, ~80% of them), and hash_value depends on the
// value alone, so the target's inner digest sha256(repr(v)) is the trial's.
// The population keeps those digests ([n_comp][npop][8], rebuilt when the
// population is re-initialised, patched per replaced row); a round then
//   k_de_diff     marks which computed-digest values differ from the target
//                 (bitwise) and compacts them into (candidate, cslot) pairs,
//   k_inner_pairs computes repr + SHA-256 only for those pairs, densely (a
//                 wave of 64 lanes always has 64 digests to do -- skipping
//                 per lane inside k_hash would not save anything: almost every
//                 wave has a lane crossing every parameter),
//   k_hash        reads each inner digest from the cache or the fresh buffer.
// ---------------------------------------------------------------------------
// The cache covers the members [lo, lo + wn): a context caches the targets of
// its own candidates (a rank's shard), not the whole replicated population.
// rows == nullptr: rebuild every member of the window; else patch the members
// rows[0..nrows) that fall inside it.
__global__ __launch_bounds__(HASH_NT) void k_pop_digests(const DevParam* __restrict__ params,
                                                         const int32_t* __restrict__ comp, int32_t n_comp,
                                                         const double* __restrict__ pop, int64_t npop,
                                                         const int64_t* __restrict__ rows, int64_t nrows,
                                                         int64_t lo, int64_t wn, uint4* __restrict__ cache) {
  __shared__ uint32_t lds[SCR_WORDS * HASH_NT];
  const int lane = threadIdx.x;
  const int32_t s = blockIdx.y;
  const int64_t r = (int64_t)blockIdx.x * HASH_NT + lane;
  const int64_t n = rows ? nrows : wn;
  if (s >= n_comp || r >= n) return;   // no barriers below: every lane owns its LDS column
  const int64_t j = rows ? rows[r] : lo + r;
  if (j < lo || j >= lo + wn || j >= npop) return;   // outside the cached window
  const DevParam pr = params[comp[s]];
  uint32_t D[8];
  repr_digest(pr, pop[(int64_t)pr.col * npop + j], lds, lane, D);
  store_hex(cache + 4 * ((int64_t)s * wn + (j - lo)), D);
}

constexpr int DIFF_NT = 256;

__device__ __forceinline__ uint64_t d_bits(double x) { return (uint64_t)__double_as_longlong(x); }

// one lane per candidate: mask bits of the values that differ from the target
// member (g % npop) and their (candidate, cslot) pairs, appended with one
// atomic per wave (the pair order does not matter: each pair's digest has its
// own slot in the fresh buffer)
__global__ __launch_bounds__(DIFF_NT) void k_de_diff(const DevParam* __restrict__ params,
                                                     const int32_t* __restrict__ comp, int32_t n_comp,
                                                     const double* __restrict__ values, int64_t ld, int64_t m,
                                                     const double* __restrict__ pop, int64_t npop, int64_t cand_base,
                                                     uint32_t* __restrict__ mask, uint64_t* __restrict__ pairs,
                                                     unsigned long long* __restrict__ npairs) {
  const int64_t i = (int64_t)blockIdx.x * DIFF_NT + threadIdx.x;
  const int lane = threadIdx.x & 63;
  const bool valid = i < m;
  const int64_t t = valid ? (int64_t)((uint64_t)(cand_base + i) % (uint64_t)npop) : 0;
  uint32_t cnt = 0;
  for (int32_t w = 0; w * 32 < n_comp; ++w) {
    uint32_t bits = 0;
    const int32_t hi = n_comp - w * 32 < 32 ? n_comp - w * 32 : 32;
    for (int32_t b = 0; b < hi; ++b) {
      const int32_t col = params[comp[w * 32 + b]].col;
      if (valid && d_bits(values[(int64_t)col * ld + i]) != d_bits(pop[(int64_t)col * npop + t])) bits |= 1u << b;
    }
    if (valid) mask[(int64_t)w * ld + i] = bits;
    cnt += __builtin_popcount(bits);
  }
  // wave-inclusive prefix sum of the counts, one atomic per wave for its base
  uint32_t incl = cnt;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t o = __shfl_up(incl, d, 64);
    if (lane >= d) incl += o;
  }
  const uint32_t total = __shfl(incl, 63, 64);
  unsigned long long base = 0;
  if (lane == 63 && total) base = atomicAdd(npairs, (unsigned long long)total);
  base = __shfl(base, 63, 64);
  if (!cnt) return;
  uint64_t pos = base + (incl - cnt);
  for (int32_t w = 0; w * 32 < n_comp; ++w) {
    uint32_t bits = mask[(int64_t)w * ld + i];
    while (bits) {
      const int b = __builtin_ctz(bits);
      bits &= bits - 1;
      pairs[pos++] = ((uint64_t)i << 20) | (uint64_t)(w * 32 + b);
    }
  }
}

// repr + SHA-256 of the changed values, a dense grid-stride over the pairs
__global__ __launch_bounds__(HASH_NT) void k_inner_pairs(const DevParam* __restrict__ params,
                                                         const int32_t* __restrict__ comp,
                                                         const double* __restrict__ values, int64_t ld,
                                                         const uint64_t* __restrict__ pairs,
                                                         const unsigned long long* __restrict__ npairs,
                                                         uint4* __restrict__ fresh) {
  __shared__ uint32_t lds[SCR_WORDS * HASH_NT];
  const int lane = threadIdx.x;
  const int64_t n = (int64_t)*npairs;
  for (int64_t q = (int64_t)blockIdx.x * HASH_NT + lane; q < n; q += (int64_t)gridDim.x * HASH_NT) {
    const uint64_t e = pairs[q];
    const int64_t i = (int64_t)(e >> 20);
    const int32_t s = (int32_t)(e & 0xFFFFFu);
    const DevParam pr = params[comp[s]];
    uint32_t D[8];
    repr_digest(pr, values[(int64_t)pr.col * ld + i], lds, lane, D);
    store_hex(fresh + 4 * ((int64_t)s * ld + i), D);
  }
}

// every computed inner digest of m candidates, (param, candidate) pairs in
// parallel (small-m ut_hash: one thread per candidate would leave the chip idle)
__global__ __launch_bounds__(HASH_NT) void k_inner_all(const DevParam* __restrict__ params,
                                                       const int32_t* __restrict__ comp, int32_t n_comp,
                                                       const double* __restrict__ values, int64_t ld, int64_t m,
                                                       uint4* __restrict__ fresh) {
  __shared__ uint32_t lds[SCR_WORDS * HASH_NT];
  const int lane = threadIdx.x;
  const int64_t n = (int64_t)n_comp * m;
  for (int64_t q = (int64_t)blockIdx.x * HASH_NT + lane; q < n; q += (int64_t)gridDim.x * HASH_NT) {
    const int32_t s = (int32_t)(q / m);
    const int64_t i = q - (int64_t)s * m;
    const DevParam pr = params[comp[s]];
    uint32_t D[8];
    repr_digest(pr, values[(int64_t)pr.col * ld + i], lds, lane, D);
    store_hex(fresh + 4 * ((int64_t)s * m + i), D);
  }
}

// Inner digests of the computed-digest params, when k_hash reuses them (DE
// rounds), kept as their 64 hex characters (16 big-endian words: what the
// outer message holds), so k_hash moves them into its hex slot as they are
struct InnerRef {
  const uint32_t* mask;   // [ceil(n_comp / 32)][ldf]
  const uint4* fresh;     // [n_comp][ldf][16 hex words]
  const uint4* cache;     // [n_comp][wn][16 hex words] of members [wlo, wlo + wn); nullptr = compute every
                          // inner digest in k_hash
  int64_t npop, cand_base;
  int64_t wlo, wn;        // the cache's member window (every target (cand_base + i) % npop lies in it)
  int64_t ldf;            // leading dimension of mask / fresh
};

// REF: every computed inner digest comes from ref (cache / fresh) and the
// repr + SHA-256 path is not compiled in: 175 -> 135 VGPRs, and with a
// 4-waves/SIMD bound 128 (9 spilled), outer-message-only hashing 3.54 ->
// 3.42 ms at C2.  Tried and not kept: the two hex slots in LDS instead of 32
// VGPRs (104 VGPRs, still 4 waves: 3.59 ms, the ds_reads cost more than the
// registers), 5 or 6 waves/SIMD (107 / 137 VGPRs spilled: 4.53 / 6.87 ms).
// 16 hex words into hex slot `odd` (static register indices in both branches)
__device__ __forceinline__ void put_hex(hex32& HX, int odd, uint4 q0, uint4 q1, uint4 q2, uint4 q3) {
  const uint32_t q[16] = {q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, q1.z, q1.w,
                          q2.x, q2.y, q2.z, q2.w, q3.x, q3.y, q3.z, q3.w};
  if (odd) {
#pragma unroll
    for (int k = 0; k < 16; ++k) HX[16 + k] = q[k];
  } else {
#pragma unroll
    for (int k = 0; k < 16; ++k) HX[k] = q[k];
  }
}

template <bool REF, int MINW>
__global__ __launch_bounds__(HASH_NT, MINW) void k_hash(const DevParam* __restrict__ params,
                                                  const int32_t* __restrict__ order,
                                                  const int32_t* __restrict__ order_col,
                                                  const uint2* __restrict__ words,
                                                  const int32_t* __restrict__ block_last, int32_t nblocks,
                                                  int32_t P, const uint4* __restrict__ lut,
                                                  const double* __restrict__ values, int64_t ld, int64_t m,
                                                  const uint4* __restrict__ perm_dig,
                                                  uint32_t* __restrict__ out, InnerRef ref) {
  __shared__ uint32_t lds[REF ? 1 : SCR_WORDS * HASH_NT];
  const int lane = threadIdx.x;
  // grid-stride over candidate blocks (launch_hash gives one block per 128
  // candidates; a smaller grid stays correct)
  for (int64_t blk = blockIdx.x; blk * HASH_NT < m; blk += gridDim.x) {
    const int64_t i0 = blk * HASH_NT + lane;
    const bool valid = i0 < m;
    const int64_t i = valid ? i0 : (m - 1);
    const int64_t t = REF ? (int64_t)((uint64_t)(ref.cand_base + i) % (uint64_t)ref.npop) : 0;
    hex32 HX = {};  // two 16-word hex slots: hole j in HX[16 (j % 2) .. 16 (j % 2) + 15]
    uint32_t H[8];
    sha256_init(H);
    int32_t next = 0;
    // the value of the next parameter to digest is loaded one parameter ahead
    double vnext = values[(int64_t)order_col[0] * ld + i];
    for (int32_t b = 0; b < nblocks; ++b) {
      const int32_t last = block_last[b];
      while (next <= last) {
        const int32_t p = order[next];
        const DevParam pr = params[p];
        const double v = vnext;
        uint32_t D[8];
        if (pr.hash_mode == HM_LUT) {
          // the value's hex digest from the LUT, straight into the hex slot
          const uint4* src = lut + 4 * lut_row(pr, v);
          const uint4 q0 = src[0], q1 = src[1], q2 = src[2], q3 = src[3];  // issued before the prefetch
          if (next + 1 < P) vnext = values[(int64_t)order_col[next + 1] * ld + i];
          put_hex(HX, next & 1, q0, q1, q2, q3);
          ++next;
          continue;
        } else if (pr.hash_mode == HM_PERM) {
          const uint4* src = perm_dig + 2 * ((int64_t)pr.pslot * m + i);
          const uint4 a = src[0], c = src[1];
          if (next + 1 < P) vnext = values[(int64_t)order_col[next + 1] * ld + i];
          D[0] = a.x; D[1] = a.y; D[2] = a.z; D[3] = a.w;
          D[4] = c.x; D[5] = c.y; D[6] = c.z; D[7] = c.w;
        } else if constexpr (REF) {
          // the target's cached hex digest, or this trial's fresh one (k_inner_pairs),
          // straight into the hex slot
          const uint32_t mw = ref.mask[(int64_t)(pr.cslot >> 5) * ref.ldf + i];
          const uint4* src = ((mw >> (pr.cslot & 31)) & 1u)
                                 ? ref.fresh + 4 * ((int64_t)pr.cslot * ref.ldf + i)
                                 : ref.cache + 4 * ((int64_t)pr.cslot * ref.wn + (t - ref.wlo));
          const uint4 q0 = src[0], q1 = src[1], q2 = src[2], q3 = src[3];
          if (next + 1 < P) vnext = values[(int64_t)order_col[next + 1] * ld + i];
          put_hex(HX, next & 1, q0, q1, q2, q3);
          ++next;
          continue;
        } else {
          if (next + 1 < P) vnext = values[(int64_t)order_col[next + 1] * ld + i];
          repr_digest(pr, v, lds, lane, D);
        }
        (void)v;
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
}

// Workgroups per CU for the grid-stride hash grids (0 = uncapped).  A large
// refit (>= HASH_CAP_MIN_NPAD padded rows) still running when the hash is
// enqueued (and not waited for by the hash's stream first) is a chain of small
// latency-bound kernels the round's scoring waits for; a full hash grid takes
// every CU slot the chain frees, so the chain runs ~2.5x longer than alone.
// Capped (with the fit's waves at s_setprio 3), the chain keeps slots and the
// hash, off the critical path, takes ~2x longer.  Only for hashes small enough
// to stay off the critical path at half speed (m x components <=
// HASH_CAP_MAX_PAIRS for the inner digests, m x outer blocks <=
// HASH_CAP_MAX_BLOCKS for the outer hash).  Measured: C3 (n 4096, 2^21
// candidates) pruned 39.6 -> 36.7-37.5 ms, f16x3 119.7 -> 115.6 ms; capped,
// C2 (n 1024) went 26.2 -> 29.2 ms, C4 (2^22 x 472 blocks) 191 -> 247 ms, and
// C2 f16x3 with only its inner digests capped 11.44 -> 11.79 ms (its fit_wait
// 4.0 -> 1.5 ms, but the hash then overlapped K*: 3.4 -> 5.0 ms)
// (scripts/ab/r04s_fitprio.sh, r04t_capsweep.sh, r04x_innercap.sh).
// UT_HASH_WG_PER_CU: N > 0 always N, 0 never, -1 (default) as above.
constexpr int32_t HASH_CAP_MIN_NPAD = 2048, HASH_CAP_WG = 4;
constexpr double HASH_CAP_MAX_BLOCKS = 5e8, HASH_CAP_MAX_PAIRS = 268435456.0;

static int32_t hash_cap(ut_ctx* c, int64_t m, bool outer, bool after_fit) {
  if (c->hash_wg_per_cu >= 0) return c->hash_wg_per_cu;
  if (after_fit || !c->fit_pending) return 0;
  if (c->gp_npad_fit < HASH_CAP_MIN_NPAD) return 0;
  if (outer ? (double)m * (double)c->space.outer_blocks > HASH_CAP_MAX_BLOCKS
            : (double)m * (double)c->space.n_comp > HASH_CAP_MAX_PAIRS)
    return 0;
  return hipEventQuery(c->ev_fit) == hipErrorNotReady ? HASH_CAP_WG : 0;
}

static int launch_hash_impl(ut_ctx* c, const double* values, int64_t ld, int64_t m, uint32_t* out, InnerRef ref,
                            bool after_fit = false) {
  if (m <= 0) return 0;
  const Space& s = c->space;
  const uint32_t* pd = nullptr;
  if (s.n_perm > 0) {
    int rc = ensure(c, c->perm_dig, (size_t)s.n_perm * (size_t)m * 8);
    if (rc) return rc;
    hipLaunchKernelGGL(k_perm_digest, dim3(grid1(m, PD_NT)), dim3(PD_NT), 0, c->stream, s.d_params, s.d_perm_params,
                       s.n_perm, s.d_perm_bytes, s.d_perm_off, s.d_perm_offbase, s.d_perm_len, values, ld, m,
                       c->perm_dig.p);
    UT_LAUNCH_CHECK(c);
    pd = c->perm_dig.p;
  }
  // (grid-stride: a cap on the grid leaves CU slots to the fit stream's kernels)
  int64_t nb = (int64_t)grid1(m, HASH_NT);
  if (const int32_t cap = hash_cap(c, m, true, after_fit)) nb = std::min<int64_t>(nb, (int64_t)c->n_cu * cap);
#ifndef UT_HASH_REF_WAVES
#define UT_HASH_REF_WAVES 4
#endif
  auto kern = ref.cache ? k_hash<true, UT_HASH_REF_WAVES> : k_hash<false, 1>;
  hipLaunchKernelGGL(kern, dim3((unsigned)nb), dim3(HASH_NT), 0, c->stream, s.d_params, s.d_order,
                     s.d_order_col, reinterpret_cast<const uint2*>(s.d_words), s.d_block_last,
                     (int32_t)s.outer_blocks, s.P, reinterpret_cast<const uint4*>(s.d_lut), values, ld, m,
                     reinterpret_cast<const uint4*>(pd), out, ref);
  UT_LAUNCH_CHECK(c);
  return 0;
}

// up to this many candidates ut_hash computes the inner digests first, all
// (param, candidate) pairs in parallel, then the outer messages from them
constexpr int64_t HASH_SMALL_M = 16384;   // R64 0.66 -> 0.34-0.44 ms at 2^12-2^14; HPL-64 at 2^15 was 2% slower

int launch_hash(ut_ctx* c, const double* values, int64_t ld, int64_t m, uint32_t* out) {
  const Space& s = c->space;
  if (s.n_comp > 0 && m > 0 && m <= HASH_SMALL_M) {
    const int32_t nw = (s.n_comp + 31) / 32;
    int rc;
    // the fresh digests and the mask are indexed with leading dimension m, not
    // ld (a few columns of a wide SoA array must not size them by its ld)
    if ((rc = ensure(c, c->hs_mask, (size_t)nw * m))) return rc;
    if ((rc = ensure(c, c->hs_fresh, (size_t)s.n_comp * m * 16))) return rc;
    UT_HIP(c, hipMemsetAsync(c->hs_mask.p, 0xFF, sizeof(uint32_t) * nw * m, c->stream));
    const int64_t want = ((int64_t)s.n_comp * m + HASH_NT - 1) / HASH_NT;
    const unsigned grid = (unsigned)std::min<int64_t>(want, (int64_t)c->n_cu * 8);
    hipLaunchKernelGGL(k_inner_all, dim3(grid), dim3(HASH_NT), 0, c->stream, s.d_params, s.d_comp, s.n_comp, values,
                       ld, m, reinterpret_cast<uint4*>(c->hs_fresh.p));
    UT_LAUNCH_CHECK(c);
    // every mask bit set: k_hash reads each computed digest from hs_fresh (the
    // "cache" operand is never read)
    const uint4* fr = reinterpret_cast<const uint4*>(c->hs_fresh.p);
    return launch_hash_impl(c, values, ld, m, out, InnerRef{c->hs_mask.p, fr, fr, 1, 0, 0, 1, m});
  }
  return launch_hash_impl(c, values, ld, m, out, InnerRef{nullptr, nullptr, nullptr, 1, 0, 0, 1, ld});
}

int launch_pop_digests_window(ut_ctx* c, int64_t lo, int64_t wn) {
  const Space& s = c->space;
  if (s.n_comp == 0 || c->npop == 0) return 0;
  lo = std::max<int64_t>(0, std::min(lo, c->npop - 1));
  wn = std::max<int64_t>(1, std::min(wn, c->npop - lo));
  const int64_t need = (int64_t)s.n_comp * wn * 16;   // 64 hex characters per digest
  if (c->pop_dig_cap < need) {
    if (c->pop_dig) {
      UT_HIP(c, sync_all(c));
      ut::dfree(c->pop_dig);
      c->pop_dig = nullptr;
      c->pop_dig_cap = 0;
    }
    const hipError_t e = ut::dmalloc((void**)&c->pop_dig, sizeof(uint32_t) * need);
    if (e != hipSuccess) return set_err(c, UT_ENOMEM, std::string("hipMalloc: ") + hipGetErrorString(e));
    c->pop_dig_cap = need;
  }
  hipLaunchKernelGGL(k_pop_digests, dim3(grid1(wn, HASH_NT), (unsigned)s.n_comp), dim3(HASH_NT), 0, c->stream,
                     s.d_params, s.d_comp, s.n_comp, c->pop, c->npop, (const int64_t*)nullptr, (int64_t)0, lo, wn,
                     reinterpret_cast<uint4*>(c->pop_dig));
  UT_LAUNCH_CHECK(c);
  c->pop_dig_lo = lo;
  c->pop_dig_n = wn;
  c->pop_dig_valid = true;
  return 0;
}

int launch_pop_digests(ut_ctx* c, const int64_t* idx, int64_t n) {
  const Space& s = c->space;
  if (s.n_comp == 0 || c->npop == 0 || !c->pop_dig_valid || n <= 0) return 0;
  hipLaunchKernelGGL(k_pop_digests, dim3(grid1(n, HASH_NT), (unsigned)s.n_comp), dim3(HASH_NT), 0, c->stream,
                     s.d_params, s.d_comp, s.n_comp, c->pop, c->npop, idx, n, c->pop_dig_lo, c->pop_dig_n,
                     reinterpret_cast<uint4*>(c->pop_dig));
  UT_LAUNCH_CHECK(c);
  return 0;
}

int ensure_de_diff(ut_ctx* c, int64_t ld) {
  const Space& s = c->space;
  const int32_t nw = (s.n_comp + 31) / 32;
  int rc;
  if ((rc = ensure(c, c->r_mask, (size_t)nw * ld))) return rc;
  if ((rc = ensure(c, c->r_fresh, (size_t)s.n_comp * ld * 16))) return rc;   // hex digests
  if ((rc = ensure(c, c->r_pairs, (size_t)s.n_comp * ld))) return rc;
  return ensure(c, c->r_npairs, 1);
}

int launch_hash_de(ut_ctx* c, const double* values, int64_t ld, int64_t m, int64_t cand_base, uint32_t* out,
                   bool have_diff) {
  const Space& s = c->space;
  if (s.n_comp == 0 || m <= 0) return launch_hash(c, values, ld, m, out);
  int rc;
  // the targets of this call: members (cand_base + i) % npop, i < m -- one
  // contiguous range unless it wraps around the population (then all of it)
  int64_t tlo = (int64_t)((uint64_t)cand_base % (uint64_t)c->npop), tn = m;
  if (tlo + tn > c->npop) tlo = 0, tn = c->npop;
  const bool covered = c->pop_dig_valid && tlo >= c->pop_dig_lo && tlo + tn <= c->pop_dig_lo + c->pop_dig_n;
  if (!covered && (rc = launch_pop_digests_window(c, tlo, tn))) return rc;
  if ((rc = ensure_de_diff(c, ld))) return rc;
  unsigned long long* np = reinterpret_cast<unsigned long long*>(c->r_npairs.p);
  if (!have_diff) {
    UT_HIP(c, hipMemsetAsync(c->r_npairs.p, 0, sizeof(int64_t), c->stream));
    hipLaunchKernelGGL(k_de_diff, dim3(grid1(m, DIFF_NT)), dim3(DIFF_NT), 0, c->stream, s.d_params, s.d_comp,
                       s.n_comp, values, ld, m, c->pop, c->npop, cand_base, c->r_mask.p, c->r_pairs.p, np);
    UT_LAUNCH_CHECK(c);
  }
  const int64_t want = ((int64_t)s.n_comp * m + HASH_NT - 1) / HASH_NT;
  // (ctx.round_hash_hold: the round's inner digests and outer hash wait for an in-flight fit)
  const bool hold = c->round_hash_hold && c->fit_pending && hipEventQuery(c->ev_fit) == hipErrorNotReady;
  const int32_t cap = hash_cap(c, m, false, hold);
  const unsigned grid = (unsigned)std::min<int64_t>(std::max<int64_t>(want, 1), (int64_t)c->n_cu * (cap > 0 ? cap : 8));
  if (hold) UT_HIP(c, hipStreamWaitEvent(c->stream, c->ev_fit, 0));
  hipLaunchKernelGGL(k_inner_pairs, dim3(grid), dim3(HASH_NT), 0, c->stream, s.d_params, s.d_comp, values, ld,
                     c->r_pairs.p, np, reinterpret_cast<uint4*>(c->r_fresh.p));
  UT_LAUNCH_CHECK(c);
  return launch_hash_impl(c, values, ld, m, out,
                          InnerRef{c->r_mask.p, reinterpret_cast<const uint4*>(c->r_fresh.p),
                                   reinterpret_cast<const uint4*>(c->pop_dig), c->npop, cand_base, c->pop_dig_lo,
                                   c->pop_dig_n, ld},
                          hold);
}

int launch_hash_parent(ut_ctx* c, const double* values, int64_t ld, int64_t m, const double* parent, uint32_t* out) {
  const Space& s = c->space;
  if (s.n_comp == 0 || m <= 0) return launch_hash(c, values, ld, m, out);
  int rc;
  if ((rc = ensure(c, c->par_dig, (size_t)s.n_comp * 16))) return rc;
  if ((rc = ensure_de_diff(c, ld))) return rc;
  // the parent's hex inner digests: a population of one member (column p at parent[col])
  hipLaunchKernelGGL(k_pop_digests, dim3(1, (unsigned)s.n_comp), dim3(HASH_NT), 0, c->stream, s.d_params, s.d_comp,
                     s.n_comp, parent, (int64_t)1, (const int64_t*)nullptr, (int64_t)0, (int64_t)0, (int64_t)1,
                     reinterpret_cast<uint4*>(c->par_dig.p));
  UT_LAUNCH_CHECK(c);
  // which computed-digest values differ from the parent's: every child "targets" member 0
  unsigned long long* np = reinterpret_cast<unsigned long long*>(c->r_npairs.p);
  UT_HIP(c, hipMemsetAsync(c->r_npairs.p, 0, sizeof(int64_t), c->stream));
  hipLaunchKernelGGL(k_de_diff, dim3(grid1(m, DIFF_NT)), dim3(DIFF_NT), 0, c->stream, s.d_params, s.d_comp, s.n_comp,
                     values, ld, m, parent, (int64_t)1, (int64_t)0, c->r_mask.p, c->r_pairs.p, np);
  UT_LAUNCH_CHECK(c);
  const int64_t want = ((int64_t)s.n_comp * m + HASH_NT - 1) / HASH_NT;
  const unsigned grid = (unsigned)std::min<int64_t>(std::max<int64_t>(want, 1), (int64_t)c->n_cu * 8);
  hipLaunchKernelGGL(k_inner_pairs, dim3(grid), dim3(HASH_NT), 0, c->stream, s.d_params, s.d_comp, values, ld,
                     c->r_pairs.p, np, reinterpret_cast<uint4*>(c->r_fresh.p));
  UT_LAUNCH_CHECK(c);
  return launch_hash_impl(c, values, ld, m, out,
                          InnerRef{c->r_mask.p, reinterpret_cast<const uint4*>(c->r_fresh.p),
                                   reinterpret_cast<const uint4*>(c->par_dig.p), 1, 0, 0, 1, ld});
}

}  // namespace ut
