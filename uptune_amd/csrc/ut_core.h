// ut_core.h -- arithmetic shared by the gfx950 kernels and the host-side
// self-check build: Philox4x32-10 counter RNG, SHA-256, and Python's
// shortest-round-trip repr(float) (Ryu-style digit generation + CPython's
// 'r' formatting rules).
//
// Everything here is written for 64-wide CDNA4 wavefronts first (no
// dynamic register indexing, branch-light integer code) and also compiles
// as plain C++ with g++ so the same code can be checked against CPython on
// the host (tests/test_core_host.py).
//
// Reference semantics restated here:
//   * hash_value / hash_config string layout:
//       python/uptune/opentuner/search/manipulator.py:233-243 (outer message)
//       python/uptune/opentuner/search/manipulator.py:456-459 (primitive inner)
//       python/uptune/opentuner/search/manipulator.py:855-858 (complex inner)
//   * repr(float) = CPython Python/pystrtod.c format_float_short, mode 'r'
//     (exponent form iff decpt <= -4 or decpt > 16, ".0" added to integral
//     values, "%+.02d" exponent).
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define UT_HD __host__ __device__ __forceinline__
#define UT_CONST_TABLE static constexpr
#else
#include <math.h>
#define UT_HD static inline
#define UT_CONST_TABLE static constexpr
#endif

#include "ryu_tables.h"

namespace ut {

// ---------------------------------------------------------------------------
// 64x64 -> 128 helpers
// ---------------------------------------------------------------------------
UT_HD uint64_t umulhi64(uint64_t a, uint64_t b) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __umul64hi(a, b);
#else
  return (uint64_t)(((unsigned __int128)a * b) >> 64);
#endif
}

UT_HD uint32_t umulhi32(uint32_t a, uint32_t b) {
  return (uint32_t)(((uint64_t)a * b) >> 32);
}

// ---------------------------------------------------------------------------
// Philox4x32-10 (Salmon et al., SC'11).  Key = 2x32, counter = 4x32.
// ---------------------------------------------------------------------------
struct u32x4 {
  uint32_t x, y, z, w;
};

UT_HD u32x4 philox4x32_10(u32x4 c, uint32_t k0, uint32_t k1) {
  const uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u;
  const uint32_t W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint64_t p0 = (uint64_t)M0 * c.x;
    const uint64_t p1 = (uint64_t)M1 * c.z;
    const uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
    const uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
    u32x4 n;
    n.x = hi1 ^ c.y ^ k0;
    n.y = lo1;
    n.z = hi0 ^ c.w ^ k1;
    n.w = lo0;
    c = n;
    k0 += W0;
    k1 += W1;
  }
  return c;
}

// uniform double in [0,1) with 53 random bits from two 32-bit words
UT_HD double u01_from(uint32_t lo, uint32_t hi) {
  const uint64_t v = (((uint64_t)hi << 32) | lo) >> 11;
  return (double)v * (1.0 / 9007199254740992.0);
}
UT_HD uint64_t u64_from(uint32_t lo, uint32_t hi) { return ((uint64_t)hi << 32) | lo; }
// floor(x * n / 2^64): an integer in [0, n)
UT_HD uint64_t below64(uint64_t x, uint64_t n) { return umulhi64(x, n); }

// Counter layout shared by every kernel and by oracle/philox.py:
//   c.x, c.y = global candidate index (lo, hi)
//   c.z      = stream (param index p, or STREAM_* | sub)
//   c.w      = (round << 8) | op
enum : uint32_t {
  OP_INIT = 1, OP_DE = 2, OP_PSO = 3, OP_GA = 4, OP_GGA = 5,
};
enum : uint32_t {
  STREAM_CAND = 0xFFFF0000u,   // per-candidate draws: STREAM_CAND | k
  STREAM_RETRY_SHIFT = 20,     // per-param draws at GA retry r: p | (r << 20)
  STREAM_SUB_SHIFT = 28,       // second block of per-param draws: p | (s << 28)
};

UT_HD u32x4 draw(uint64_t seed, uint64_t cand, uint32_t stream, uint32_t round_, uint32_t op) {
  u32x4 c;
  c.x = (uint32_t)cand;
  c.y = (uint32_t)(cand >> 32);
  c.z = stream;
  c.w = (round_ << 8) | (op & 0xFFu);
  return philox4x32_10(c, (uint32_t)seed, (uint32_t)(seed >> 32));
}

// DE draw layout (oracle/de.py): the cr tests `random() < cr` of params
// 4b .. 4b + 3 are the four words of block (STREAM_CAND | (DE_CR_STREAM + b)),
// each a 32-bit uniform; the forced set (the first n_cross names of the
// shuffled name list, differentialevolution.py:122-125: a uniform n_cross-subset,
// n_cross <= 4) is drawn from block (STREAM_CAND | 2) by skip-rank, one word per
// element.  17 blocks per candidate at P = 64 where one block per param (its
// x, y words the cr test, its z word a sort key) took 64.
constexpr uint32_t DE_CR_STREAM = 0x100u;
UT_HD bool de_cr_pass(uint32_t w, double cr) { return (double)w * 2.3283064365386963e-10 < cr; }
UT_HD void de_forced_set(u32x4 r, int32_t P, int32_t n_cross, int32_t f[4]) {
  const uint32_t ws[4] = {r.x, r.y, r.z, r.w};
  int32_t srt[4];   // the chosen params, ascending
  const int32_t nc = n_cross < P ? n_cross : P;
  for (int k = 0; k < 4; ++k) f[k] = -1;
  for (int k = 0; k < 4; ++k) {
    if (k >= nc) break;
    int32_t v = (int32_t)umulhi32(ws[k], (uint32_t)(P - k));   // rank among the P - k unchosen params
    for (int a = 0; a < k; ++a) v += (v >= srt[a]) ? 1 : 0;
    f[k] = v;
    int a = k;
    while (a > 0 && srt[a - 1] > v) {
      srt[a] = srt[a - 1];
      --a;
    }
    srt[a] = v;
  }
}

// Permutation-operator draw sites (oracle/perm.py): a site (seed, cand,
// stream, round, op) yields a stream of 32-bit words; block b of it is the
// Philox block with op | 0x80 and key_hi ^ b.
enum : uint32_t { OP_PERM_FLAG = 0x80u };
UT_HD u32x4 perm_block(uint64_t seed, uint64_t cand, uint32_t stream, uint32_t round_, uint32_t op, uint32_t blk) {
  u32x4 c;
  c.x = (uint32_t)cand;
  c.y = (uint32_t)(cand >> 32);
  c.z = stream;
  c.w = (round_ << 8) | ((op | OP_PERM_FLAG) & 0xFFu);
  return philox4x32_10(c, (uint32_t)seed, (uint32_t)(seed >> 32) ^ blk);
}

// ---------------------------------------------------------------------------
// SHA-256 (FIPS 180-4)
// ---------------------------------------------------------------------------
UT_CONST_TABLE uint32_t SHA256_K[64] = {
    0x428a2f98u, 0x71374491u, 0xb5c0fbcfu, 0xe9b5dba5u, 0x3956c25bu, 0x59f111f1u, 0x923f82a4u, 0xab1c5ed5u,
    0xd807aa98u, 0x12835b01u, 0x243185beu, 0x550c7dc3u, 0x72be5d74u, 0x80deb1feu, 0x9bdc06a7u, 0xc19bf174u,
    0xe49b69c1u, 0xefbe4786u, 0x0fc19dc6u, 0x240ca1ccu, 0x2de92c6fu, 0x4a7484aau, 0x5cb0a9dcu, 0x76f988dau,
    0x983e5152u, 0xa831c66du, 0xb00327c8u, 0xbf597fc7u, 0xc6e00bf3u, 0xd5a79147u, 0x06ca6351u, 0x14292967u,
    0x27b70a85u, 0x2e1b2138u, 0x4d2c6dfcu, 0x53380d13u, 0x650a7354u, 0x766a0abbu, 0x81c2c92eu, 0x92722c85u,
    0xa2bfe8a1u, 0xa81a664bu, 0xc24b8b70u, 0xc76c51a3u, 0xd192e819u, 0xd6990624u, 0xf40e3585u, 0x106aa070u,
    0x19a4c116u, 0x1e376c08u, 0x2748774cu, 0x34b0bcb5u, 0x391c0cb3u, 0x4ed8aa4au, 0x5b9cca4fu, 0x682e6ff3u,
    0x748f82eeu, 0x78a5636fu, 0x84c87814u, 0x8cc70208u, 0x90befffau, 0xa4506cebu, 0xbef9a3f7u, 0xc67178f2u};

UT_HD uint32_t rotr32(uint32_t x, int n) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_alignbit(x, x, n);
#else
  return (x >> n) | (x << (32 - n));
#endif
}

// 3-input bitwise ops: one v_bitop3_b32 on gfx950 (truth table over
// a=0xF0, b=0xCC, c=0xAA)
UT_HD uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
#else
  return a ^ b ^ c;
#endif
}
UT_HD uint32_t sha_ch(uint32_t e, uint32_t f, uint32_t g) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_bitop3_b32(e, f, g, 0xCA);
#else
  return (e & f) ^ (~e & g);
#endif
}
UT_HD uint32_t sha_maj(uint32_t a, uint32_t b, uint32_t c) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0xE8);
#else
  return (a & b) ^ (a & c) ^ (b & c);
#endif
}

UT_HD void sha256_init(uint32_t H[8]) {
  H[0] = 0x6a09e667u; H[1] = 0xbb67ae85u; H[2] = 0x3c6ef372u; H[3] = 0xa54ff53au;
  H[4] = 0x510e527fu; H[5] = 0x9b05688cu; H[6] = 0x1f83d9abu; H[7] = 0x5be0cd19u;
}

// One compression.  W holds the 16 big-endian message words and is consumed
// (used as the rolling schedule), so callers pass a scratch copy.
UT_HD void sha256_compress(uint32_t H[8], uint32_t W[16]) {
  uint32_t a = H[0], b = H[1], c = H[2], d = H[3], e = H[4], f = H[5], g = H[6], h = H[7];
#pragma unroll
  for (int t = 0; t < 64; ++t) {
    uint32_t w;
    if (t < 16) {
      w = W[t];
    } else {
      const uint32_t w15 = W[(t - 15) & 15], w2 = W[(t - 2) & 15];
      const uint32_t s0 = xor3(rotr32(w15, 7), rotr32(w15, 18), w15 >> 3);
      const uint32_t s1 = xor3(rotr32(w2, 17), rotr32(w2, 19), w2 >> 10);
      w = W[t & 15] + s0 + W[(t - 7) & 15] + s1;
      W[t & 15] = w;
    }
    const uint32_t S1 = xor3(rotr32(e, 6), rotr32(e, 11), rotr32(e, 25));
    const uint32_t t1 = (h + S1 + sha_ch(e, f, g)) + (SHA256_K[t] + w);
    const uint32_t S0 = xor3(rotr32(a, 2), rotr32(a, 13), rotr32(a, 22));
    const uint32_t mj = sha_maj(a, b, c);
    h = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + S0 + mj;
  }
  H[0] += a; H[1] += b; H[2] += c; H[3] += d; H[4] += e; H[5] += f; H[6] += g; H[7] += h;
}

// Two message words of lowercase hex for the 16-bit value v (big-endian chars).
UT_HD uint32_t hex4(uint32_t v16) {
  uint32_t x = ((v16 & 0xF000u) << 12) | ((v16 & 0x0F00u) << 8) | ((v16 & 0x00F0u) << 4) | (v16 & 0x000Fu);
  const uint32_t ge10 = ((x + 0x06060606u) >> 4) & 0x01010101u;
  return x + 0x30303030u + ge10 * 39u;
}

// digest (8 big-endian words) -> 16 big-endian words of 64 hex chars
UT_HD void digest_hex(const uint32_t D[8], uint32_t HX[16]) {
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    HX[2 * i] = hex4(D[i] >> 16);
    HX[2 * i + 1] = hex4(D[i] & 0xFFFFu);
  }
}

// ---------------------------------------------------------------------------
// Shortest round-trip decimal digits of a double (Ryu d2d).
//
// The d2d core below (mulShift64, multipleOfPowerOf5, pow5bits, the
// vmIsTrailingZeros / vrIsTrailingZeros digit-removal loop) follows
// Ulf Adams' Ryu (PLDI 2018), https://github.com/ulfjack/ryu, ryu/d2s.c,
// used under its Apache License 2.0 (alternatively Boost Software License
// 1.0):  Copyright 2018 Ulf Adams.  Licensed under the Apache License,
// Version 2.0; you may not use this file except in compliance with the
// License.  You may obtain a copy at http://www.apache.org/licenses/LICENSE-2.0.
// Unless required by applicable law or agreed to in writing, software
// distributed under the License is distributed on an "AS IS" BASIS, WITHOUT
// WARRANTIES OR CONDITIONS OF ANY KIND.  The table generator
// (gen_ryu_tables.py) computes the same 128-bit power-of-5 tables from their
// definition.  Changes here: 64-bit-only device arithmetic (__umul64hi), no
// 128-bit type on the device path, and CPython's repr() formatting on top.
// ---------------------------------------------------------------------------
UT_HD uint32_t pow5bits(int32_t e) { return (uint32_t)(((uint32_t)e * 1217359u) >> 19) + 1u; }
UT_HD uint32_t log10Pow2(int32_t e) { return ((uint32_t)e * 78913u) >> 18; }
UT_HD uint32_t log10Pow5(int32_t e) { return ((uint32_t)e * 732923u) >> 20; }

UT_HD uint32_t pow5Factor(uint64_t v) {
  uint32_t count = 0;
  for (;;) {
    const uint64_t q = v / 5;
    const uint32_t r = (uint32_t)(v - 5 * q);
    if (r != 0) break;
    v = q;
    ++count;
  }
  return count;
}
UT_HD bool multipleOfPowerOf5(uint64_t v, uint32_t p) { return pow5Factor(v) >= p; }
UT_HD bool multipleOfPowerOf2(uint64_t v, uint32_t p) { return (v & ((1ull << p) - 1)) == 0; }

// (m * (mulHi*2^64 + mulLo)) >> j, j >= 64
UT_HD uint64_t mulShift64(uint64_t m, uint64_t mulLo, uint64_t mulHi, int32_t j) {
  const uint64_t b0hi = umulhi64(m, mulLo);
  const uint64_t b2lo = m * mulHi;
  const uint64_t b2hi = umulhi64(m, mulHi);
  // (b0hi + b2) as 128 bits
  const uint64_t lo = b0hi + b2lo;
  const uint64_t hi = b2hi + (lo < b0hi ? 1u : 0u);
  const int32_t s = j - 64;  // 0 < s < 64 for all reachable inputs
  return (lo >> s) | (hi << (64 - s));
}

struct Dec64 {
  uint64_t mantissa;  // decimal digits as an integer
  int32_t exponent;   // value = mantissa * 10^exponent
};

UT_HD uint32_t decimal_length17(uint64_t v) {
  uint32_t n = 1;
  uint64_t p = 10;
  for (int i = 0; i < 16; ++i) {
    n += (v >= p) ? 1u : 0u;
    p *= 10;
  }
  return n;
}

// ieee mantissa/exponent -> shortest decimal (value must be finite, non-zero)
UT_HD Dec64 d2d(uint64_t ieeeMantissa, uint32_t ieeeExponent) {
  int32_t e2;
  uint64_t m2;
  if (ieeeExponent == 0) {
    e2 = 1 - 1023 - 52 - 2;
    m2 = ieeeMantissa;
  } else {
    e2 = (int32_t)ieeeExponent - 1023 - 52 - 2;
    m2 = (1ull << 52) | ieeeMantissa;
  }
  const bool even = (m2 & 1) == 0;
  const bool acceptBounds = even;
  const uint64_t mv = 4 * m2;
  const uint32_t mmShift = (ieeeMantissa != 0 || ieeeExponent <= 1) ? 1u : 0u;

  uint64_t vr, vp, vm;
  int32_t e10;
  bool vmIsTrailingZeros = false;
  bool vrIsTrailingZeros = false;
  if (e2 >= 0) {
    const uint32_t q = log10Pow2(e2) - (e2 > 3 ? 1u : 0u);
    e10 = (int32_t)q;
    const int32_t k = 125 + (int32_t)pow5bits((int32_t)q) - 1;
    const int32_t i = -e2 + (int32_t)q + k;
    const uint64_t lo = UT_POW5_INV_SPLIT[q][0], hi = UT_POW5_INV_SPLIT[q][1];
    vr = mulShift64(mv, lo, hi, i);
    vp = mulShift64(mv + 2, lo, hi, i);
    vm = mulShift64(mv - 1 - mmShift, lo, hi, i);
    if (q <= 21) {
      const uint32_t mvMod5 = (uint32_t)(mv - 5 * (mv / 5));
      if (mvMod5 == 0) {
        vrIsTrailingZeros = multipleOfPowerOf5(mv, q);
      } else if (acceptBounds) {
        vmIsTrailingZeros = multipleOfPowerOf5(mv - 1 - mmShift, q);
      } else {
        vp -= multipleOfPowerOf5(mv + 2, q) ? 1u : 0u;
      }
    }
  } else {
    const uint32_t q = log10Pow5(-e2) - (-e2 > 1 ? 1u : 0u);
    e10 = (int32_t)q + e2;
    const int32_t i = -e2 - (int32_t)q;
    const int32_t k = (int32_t)pow5bits(i) - 125;
    const int32_t j = (int32_t)q - k;
    const uint64_t lo = UT_POW5_SPLIT[i][0], hi = UT_POW5_SPLIT[i][1];
    vr = mulShift64(mv, lo, hi, j);
    vp = mulShift64(mv + 2, lo, hi, j);
    vm = mulShift64(mv - 1 - mmShift, lo, hi, j);
    if (q <= 1) {
      vrIsTrailingZeros = true;
      if (acceptBounds) {
        vmIsTrailingZeros = mmShift == 1;
      } else {
        --vp;
      }
    } else if (q < 63) {
      vrIsTrailingZeros = multipleOfPowerOf2(mv, q);
    }
  }

  int32_t removed = 0;
  uint32_t lastRemovedDigit = 0;
  uint64_t output;
  if (vmIsTrailingZeros || vrIsTrailingZeros) {
    for (;;) {
      const uint64_t vpDiv10 = vp / 10;
      const uint64_t vmDiv10 = vm / 10;
      if (vpDiv10 <= vmDiv10) break;
      const uint32_t vmMod10 = (uint32_t)(vm - 10 * vmDiv10);
      const uint64_t vrDiv10 = vr / 10;
      const uint32_t vrMod10 = (uint32_t)(vr - 10 * vrDiv10);
      vmIsTrailingZeros &= vmMod10 == 0;
      vrIsTrailingZeros &= lastRemovedDigit == 0;
      lastRemovedDigit = vrMod10;
      vr = vrDiv10; vp = vpDiv10; vm = vmDiv10;
      ++removed;
    }
    if (vmIsTrailingZeros) {
      for (;;) {
        const uint64_t vmDiv10 = vm / 10;
        const uint32_t vmMod10 = (uint32_t)(vm - 10 * vmDiv10);
        if (vmMod10 != 0) break;
        const uint64_t vpDiv10 = vp / 10;
        const uint64_t vrDiv10 = vr / 10;
        const uint32_t vrMod10 = (uint32_t)(vr - 10 * vrDiv10);
        vrIsTrailingZeros &= lastRemovedDigit == 0;
        lastRemovedDigit = vrMod10;
        vr = vrDiv10; vp = vpDiv10; vm = vmDiv10;
        ++removed;
      }
    }
    if (vrIsTrailingZeros && lastRemovedDigit == 5 && (vr % 2) == 0) lastRemovedDigit = 4;
    output = vr + (((vr == vm && (!acceptBounds || !vmIsTrailingZeros)) || lastRemovedDigit >= 5) ? 1u : 0u);
  } else {
    bool roundUp = false;
    const uint64_t vpDiv100 = vp / 100;
    const uint64_t vmDiv100 = vm / 100;
    if (vpDiv100 > vmDiv100) {
      const uint64_t vrDiv100 = vr / 100;
      const uint32_t vrMod100 = (uint32_t)(vr - 100 * vrDiv100);
      roundUp = vrMod100 >= 50;
      vr = vrDiv100; vp = vpDiv100; vm = vmDiv100;
      removed += 2;
    }
    for (;;) {
      const uint64_t vpDiv10 = vp / 10;
      const uint64_t vmDiv10 = vm / 10;
      if (vpDiv10 <= vmDiv10) break;
      const uint64_t vrDiv10 = vr / 10;
      const uint32_t vrMod10 = (uint32_t)(vr - 10 * vrDiv10);
      roundUp = vrMod10 >= 5;
      vr = vrDiv10; vp = vpDiv10; vm = vmDiv10;
      ++removed;
    }
    output = vr + ((vr == vm || roundUp) ? 1u : 0u);
  }
  Dec64 fd;
  fd.exponent = e10 + removed;
  fd.mantissa = output;
  return fd;
}

// ---------------------------------------------------------------------------
// repr(float) / repr(int) emitters.  Emit::put(pos, byte) writes one byte at
// string position pos; the function returns the string length.  Positions
// are computed in closed form so digits can be produced least-significant
// first without any dynamic register indexing.
// ---------------------------------------------------------------------------
template <class Emit>
UT_HD int repr_double(double x, Emit& out) {
  uint64_t bits;
#if defined(__HIP_DEVICE_COMPILE__)
  bits = (uint64_t)__double_as_longlong(x);
#else
  __builtin_memcpy(&bits, &x, 8);
#endif
  const bool neg = (bits >> 63) != 0;
  const uint64_t mant = bits & ((1ull << 52) - 1);
  const uint32_t expo = (uint32_t)((bits >> 52) & 0x7FFu);
  if (expo == 0x7FFu) {
    if (mant != 0) {
      out.put(0, 'n'); out.put(1, 'a'); out.put(2, 'n');
      return 3;
    }
    int s = 0;
    if (neg) out.put(s++, '-');
    out.put(s, 'i'); out.put(s + 1, 'n'); out.put(s + 2, 'f');
    return s + 3;
  }
  uint64_t digits;
  int32_t n, decpt;
  const int32_t e2i = (int32_t)expo - 1023 - 52;
  const uint64_t m2i = (1ull << 52) | mant;
  if (expo == 0 && mant == 0) {
    digits = 0;
    n = 1;
    decpt = 1;
  } else if (expo != 0 && e2i <= 0 && e2i >= -52 && (m2i & ((1ull << -e2i) - 1)) == 0) {
    // an integer in [1, 2^53) (Ryu's d2d_small_int): its shortest digits are the
    // integer without its trailing zeros.  Taking this path keeps such values
    // (e.g. a parameter clamped to a bound, 1000.0) out of d2d's trailing-zero
    // branch, whose digit-removal loop would stall every lane of their wave.
    uint64_t v = m2i >> -e2i;
    int32_t e10 = 0;
    for (;;) {
      const uint64_t q = v / 10;
      if (v - 10 * q != 0) break;
      v = q;
      ++e10;
    }
    digits = v;
    n = (int32_t)decimal_length17(digits);
    decpt = n + e10;
  } else {
    const Dec64 d = d2d(mant, expo);
    digits = d.mantissa;
    n = (int32_t)decimal_length17(digits);
    decpt = n + d.exponent;
  }
  const int s = neg ? 1 : 0;
  if (neg) out.put(0, '-');
  // The four layouts of repr (Python's float_repr_style 'short'):
  //   exponent  d[.ddd]e(+|-)XX      decpt <= -4 or decpt > 16
  //   leading   0.000ddd             decpt <= 0
  //   inner     ddd.ddd              0 < decpt < n
  //   trailing  ddd000.0             decpt >= n
  // The digits are emitted by ONE loop for every layout -- digit i goes to
  // s + i + shift + (i >= split) -- so lanes of a wave that format values of
  // different layouts (e.g. 1000.0 beside 123.456) do not run several digit
  // loops (each a 64-bit division by 10 per digit) one after the other.
  const bool use_exp = (decpt <= -4) || (decpt > 16);
  int shift, split;
  if (use_exp) {
    shift = 0;
    split = 1;
  } else if (decpt <= 0) {
    shift = 2 - decpt;
    split = 1 << 30;
  } else if (decpt < n) {
    shift = 0;
    split = decpt;
  } else {
    shift = 0;
    split = 1 << 30;
  }
  for (int i = n - 1; i >= 0; --i) {
    const uint64_t q = digits / 10;
    const uint32_t dg = (uint32_t)(digits - 10 * q);
    digits = q;
    out.put(s + i + shift + (i >= split ? 1 : 0), (uint8_t)('0' + dg));
  }
  if (use_exp) {
    int pos = s + n + (n > 1 ? 1 : 0);
    if (n > 1) out.put(s + 1, '.');
    int e = decpt - 1;
    out.put(pos++, 'e');
    out.put(pos++, e < 0 ? '-' : '+');
    if (e < 0) e = -e;
    if (e >= 100) {
      out.put(pos++, (uint8_t)('0' + e / 100));
      e %= 100;
    }
    out.put(pos++, (uint8_t)('0' + e / 10));
    out.put(pos++, (uint8_t)('0' + e % 10));
    return pos;
  }
  if (decpt <= 0) {
    out.put(s, '0');
    out.put(s + 1, '.');
    for (int z = 0; z < -decpt; ++z) out.put(s + 2 + z, '0');
    return s + 2 - decpt + n;
  }
  if (decpt < n) {
    out.put(s + decpt, '.');
    return s + n + 1;
  }
  for (int z = n; z < decpt; ++z) out.put(s + z, '0');
  out.put(s + decpt, '.');
  out.put(s + decpt + 1, '0');
  return s + decpt + 2;
}

template <class Emit>
UT_HD int repr_int64(int64_t v, Emit& out) {
  const bool neg = v < 0;
  uint64_t u = neg ? (uint64_t)0 - (uint64_t)v : (uint64_t)v;
  const int s = neg ? 1 : 0;
  if (neg) out.put(0, '-');
  uint32_t n = 1;
  {
    uint64_t p = 10;
    for (int i = 0; i < 19; ++i) {
      n += (u >= p) ? 1u : 0u;
      if (p > UINT64_C(1844674407370955161)) break;
      p *= 10;
    }
  }
  for (int i = (int)n - 1; i >= 0; --i) {
    const uint64_t q = u / 10;
    out.put(s + i, (uint8_t)('0' + (uint32_t)(u - 10 * q)));
    u = q;
  }
  return s + (int)n;
}

// ---------------------------------------------------------------------------
// Deterministic exp / log / normal draws.  Built only from IEEE +,-,*,/,
// sqrt and exponent-field manipulation, evaluated in a fixed order (the
// kernels are compiled with -ffp-contract=off), so the device and the numpy
// oracle (oracle/mathx.py) produce identical bits -- libm/ocml results may
// differ by an ulp and would otherwise leak into discrete PSO/GA outcomes.
// Accuracy ~1 ulp over the ranges used.
// ---------------------------------------------------------------------------
UT_HD double bits_to_d(uint64_t b) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __longlong_as_double((long long)b);
#else
  double d;
  __builtin_memcpy(&d, &b, 8);
  return d;
#endif
}
UT_HD uint64_t d_to_bits(double d) {
#if defined(__HIP_DEVICE_COMPILE__)
  return (uint64_t)__double_as_longlong(d);
#else
  uint64_t b;
  __builtin_memcpy(&b, &d, 8);
  return b;
#endif
}
UT_HD double dsqrt(double x) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __dsqrt_rn(x);
#else
  return __builtin_sqrt(x);
#endif
}

constexpr double UT_LN2_HI = 6.93147180369123816490e-01;  // ln2 with 32 trailing zero bits
constexpr double UT_LN2_LO = 1.90821492927058770002e-10;
constexpr double UT_INV_LN2 = 1.44269504088896338700e+00;
constexpr double UT_SQRT2 = 1.41421356237309514547e+00;

// natural log for positive normal x
UT_HD double ut_log(double x) {
  const uint64_t b = d_to_bits(x);
  int32_t e = (int32_t)((b >> 52) & 0x7FF) - 1023;
  double m = bits_to_d((b & 0x000FFFFFFFFFFFFFull) | 0x3FF0000000000000ull);  // [1, 2)
  if (m > UT_SQRT2) {
    m = bits_to_d((b & 0x000FFFFFFFFFFFFFull) | 0x3FE0000000000000ull);        // [0.5, 1)
    e += 1;
  }
  const double s = (m - 1.0) / (m + 1.0);
  const double s2 = s * s;
  double p = 1.0 / 23.0;
  p = p * s2 + 1.0 / 21.0;
  p = p * s2 + 1.0 / 19.0;
  p = p * s2 + 1.0 / 17.0;
  p = p * s2 + 1.0 / 15.0;
  p = p * s2 + 1.0 / 13.0;
  p = p * s2 + 1.0 / 11.0;
  p = p * s2 + 1.0 / 9.0;
  p = p * s2 + 1.0 / 7.0;
  p = p * s2 + 1.0 / 5.0;
  p = p * s2 + 1.0 / 3.0;
  const double lm = (2.0 * s) + ((2.0 * s) * (s2 * p));
  const double fe = (double)e;
  return (fe * UT_LN2_HI) + ((fe * UT_LN2_LO) + lm);
}

// exp(x); 0 for x < -745.2, +inf for x > 709.78
UT_HD double ut_exp(double x) {
  if (x != x) return x;
  if (x > 709.782712893384) return bits_to_d(0x7FF0000000000000ull);
  if (x < -745.2) return 0.0;
  const double kd = rint(x * UT_INV_LN2);
  const double r = (x - kd * UT_LN2_HI) - kd * UT_LN2_LO;
  double p = 1.0 / 6227020800.0;        // 1/13!
  p = p * r + 1.0 / 479001600.0;
  p = p * r + 1.0 / 39916800.0;
  p = p * r + 1.0 / 3628800.0;
  p = p * r + 1.0 / 362880.0;
  p = p * r + 1.0 / 40320.0;
  p = p * r + 1.0 / 5040.0;
  p = p * r + 1.0 / 720.0;
  p = p * r + 1.0 / 120.0;
  p = p * r + 1.0 / 24.0;
  p = p * r + 1.0 / 6.0;
  p = p * r + 0.5;
  p = p * r + 1.0;
  p = p * r + 1.0;
  int32_t k = (int32_t)kd;
  if (k > 1023) {  // x just below the overflow threshold: 2^k in two steps
    p = p * 2.0;
    k -= 1;
  }
  if (k < -1021) {
    p = p * bits_to_d((uint64_t)(k + 1000 + 1023) << 52);
    return p * bits_to_d((uint64_t)(-1000 + 1023) << 52);
  }
  return p * bits_to_d((uint64_t)(k + 1023) << 52);
}

// standard normal by Marsaglia's polar method over counter draws; attempt a
// uses stream (stream | a << 24).  16 attempts (P(all rejected) ~ 2e-11,
// then 0.0).
UT_HD double normal_draw(uint64_t seed, uint64_t cand, uint32_t stream, uint32_t round_, uint32_t op) {
  for (uint32_t a = 0; a < 16; ++a) {
    const u32x4 r = draw(seed, cand, stream | (a << 24), round_, op);
    const double u = 2.0 * u01_from(r.x, r.y) - 1.0;
    const double v = 2.0 * u01_from(r.z, r.w) - 1.0;
    const double s = u * u + v * v;
    if (s > 0.0 && s < 1.0) return u * dsqrt((-2.0 * ut_log(s)) / s);
  }
  return 0.0;
}

// ---------------------------------------------------------------------------
// Double-double 2^x for the scaled parameter kinds (manipulator.py:778-797):
//   LogIntegerParameter._unscale = int(round(2.0 ** v - 1.0 + min))
// ~2^-100 relative before the one final rounding; the stored integer is
// rounded again, so it equals CPython's pow-based value on every argument
// tried (tests/test_core_host.py test_logint_unscale_matches_cpython).
// (_scale = math.log(v + 1.0 - min, 2.0) is libm_log below, restated exactly.)
// ---------------------------------------------------------------------------
struct dd {
  double hi, lo;
};
UT_HD double fma_rn(double a, double b, double c) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __fma_rn(a, b, c);
#else
  return __builtin_fma(a, b, c);
#endif
}
UT_HD dd two_sum(double a, double b) {
  const double s = a + b, bb = s - a;
  return dd{s, (a - (s - bb)) + (b - bb)};
}
UT_HD dd fast_two_sum(double a, double b) {  // |a| >= |b|
  const double s = a + b;
  return dd{s, b - (s - a)};
}
UT_HD dd two_prod(double a, double b) {
  const double p = a * b;
  return dd{p, fma_rn(a, b, -p)};
}
UT_HD dd dd_add(dd a, dd b) {
  dd s = two_sum(a.hi, b.hi);
  const dd t = two_sum(a.lo, b.lo);
  s.lo += t.hi;
  s = fast_two_sum(s.hi, s.lo);
  s.lo += t.lo;
  return fast_two_sum(s.hi, s.lo);
}
UT_HD dd dd_mul(dd a, dd b) {
  dd p = two_prod(a.hi, b.hi);
  p.lo += a.hi * b.lo + a.lo * b.hi;
  return fast_two_sum(p.hi, p.lo);
}
UT_HD dd dd_mul_d(dd a, double b) {
  dd p = two_prod(a.hi, b);
  p.lo += a.lo * b;
  return fast_two_sum(p.hi, p.lo);
}
UT_HD dd dd_div_d(dd a, double b) {
  const double q1 = a.hi / b;
  const dd p = two_prod(q1, b);
  const double r = ((a.hi - p.hi) - p.lo) + a.lo;
  return fast_two_sum(q1, r / b);
}
UT_HD dd dd_ldexp(dd a, int32_t k) {  // exact scaling by 2^k (|k| <= 1000, normal results)
  const double s = bits_to_d((uint64_t)(k + 1023) << 52);
  return dd{a.hi * s, a.lo * s};
}

constexpr double UT_LN2_DD_HI = 0x1.62e42fefa39efp-1;   // log(2.0) rounded = 6.93147180559945286e-01
constexpr double UT_LN2_DD_LO = 0x1.abc9e3b39803fp-56;  // ln 2 - UT_LN2_DD_HI

// exp of a double-double argument, |x| < 700
UT_HD dd dd_exp(dd x) {
  const double kd = rint(x.hi * UT_INV_LN2);
  dd r = dd_add(x, dd_mul_d(dd{UT_LN2_DD_HI, UT_LN2_DD_LO}, -kd));  // |r| <= 0.35
  r = dd_ldexp(r, -8);                                                  // |r| <= 1.4e-3
  // expm1(r) = r (1 + r/2 (1 + r/3 (1 + ... r/10)))
  dd p{1.0, 0.0};
  for (int k = 10; k >= 2; --k) p = dd_add(dd{1.0, 0.0}, dd_div_d(dd_mul(r, p), (double)k));
  dd a = dd_mul(r, p);
  for (int i = 0; i < 8; ++i) a = dd_add(dd{2.0 * a.hi, 2.0 * a.lo}, dd_mul(a, a));  // (1+a)^2 - 1
  return dd_ldexp(dd_add(dd{1.0, 0.0}, a), (int32_t)kd);
}

// 2.0 ** s, |s| < 1000
UT_HD double exp2_cr(double s) {
  dd t = two_prod(s, UT_LN2_DD_HI);
  t.lo += s * UT_LN2_DD_LO;
  t = fast_two_sum(t.hi, t.lo);
  return dd_exp(t).hi;
}

// ---------------------------------------------------------------------------
// libm_log: the natural log CPython's math.log calls on this image, bit for bit.
// glibc 2.35 x86-64 dispatches log() by ifunc; on CPUs with FMA + AVX2 (the
// build container and the MI355X hosts) it runs the FMA build, __log_fma
// (sysdeps/ieee754/dbl-64/e_log.c compiled with -mfma -mavx2).  Its result is
// not correctly rounded everywhere (<= 0.52 ulp), so matching it needs the
// same table (libm_log_data.h, read out of libm.so.6 by
// gen_libm_log_tables.py) and the same operation sequence, including the
// multiply-adds the compiler fused.  The sequence below is the one in the
// __log_fma machine code, with every fused step an explicit fma_rn and every
// other step a separately rounded IEEE op (this header is compiled with
// -ffp-contract=off).  Checked against CPython's math.log on every integer
// in [1, 2^22], 10^6 random integers below 2^31 and random doubles
// (tests/test_core_host.py test_py_log2_matches_cpython), and on the GPU box's
// own CPython (tests/test_gpu_parity.py test_logint_large_range_bit_exact).
// ---------------------------------------------------------------------------
}  // namespace ut
#include "libm_log_data.h"
namespace ut {

UT_HD double libm_log(double x) {
  uint64_t ix = d_to_bits(x);
  // |x - 1| small: ix - asuint64(1 - 0x1p-4) < asuint64(1 + 0x1.09p-4) - asuint64(1 - 0x1p-4)
  if (ix - 0x3fee000000000000ull < 0x0003090000000000ull) {
    if (ix == 0x3ff0000000000000ull) return 0.0;
    const double* B = LIBM_LOG_B;
    const double r = x - 1.0;
    double t1 = fma_rn(r, B[2], B[1]);
    double t4 = fma_rn(r, B[5], B[4]);
    double t7 = fma_rn(r, B[8], B[7]);
    const double r2 = r * r;
    t1 = fma_rn(r2, B[3], t1);
    t4 = fma_rn(r2, B[6], t4);
    const double r3 = r * r2;
    t7 = fma_rn(r2, B[9], t7);
    t7 = fma_rn(r3, B[10], t7);
    t7 = fma_rn(t7, r3, t4);
    const double poly = fma_rn(t7, r3, t1);
    // rhi = r + w - w with w = r * 0x1p27 (fused: fma(r, 2^27, r), then fnmadd)
    const double rhi = fma_rn(-r, 0x1p27, fma_rn(r, 0x1p27, r));
    const double rh2 = rhi * rhi;
    const double rlo = r - rhi;
    const double hi = fma_rn(rh2, B[0], r);      // r + rhi*rhi*B0
    double lo = fma_rn(rh2, B[0], r - hi);       // r - hi + w
    lo = fma_rn(B[0] * rlo, r + rhi, lo);        // lo += B0*rlo*(rhi + r)
    const double y = fma_rn(poly, r3, lo);
    return hi + y;
  }
  const uint32_t top = (uint32_t)(ix >> 48);
  if (top - 0x0010u >= 0x7ff0u - 0x0010u) {
    if ((ix << 1) == 0) return -bits_to_d(0x7FF0000000000000ull);     // log(+-0) = -inf
    if (ix == 0x7FF0000000000000ull) return x;                        // log(inf) = inf
    if ((top & 0x8000u) || (top & 0x7ff0u) == 0x7ff0u) return bits_to_d(0x7FF8000000000000ull);  // x < 0, NaN
    ix = d_to_bits(x * 0x1p52) - (52ull << 52);                       // subnormal: normalise
  }
  const uint64_t tmp = ix - 0x3fe6000000000000ull;
  const int32_t i = (int32_t)((tmp >> 45) & 127);
  const int32_t k = (int32_t)((int64_t)tmp >> 52);
  const double z = bits_to_d(ix - (tmp & 0xfff0000000000000ull));
  const double invc = LIBM_LOG_TAB[2 * i], logc = LIBM_LOG_TAB[2 * i + 1];
  const double kd = (double)k;
  const double r = fma_rn(z, invc, -1.0);                 // vfmadd132sd
  const double w = fma_rn(kd, LIBM_LOG_LN2HI, logc);      // vfmadd213sd
  const double p12 = fma_rn(r, LIBM_LOG_A[2], LIBM_LOG_A[1]);
  const double hi = r + w;
  const double r2 = r * r;
  double lo = (w - hi) + r;
  lo = fma_rn(kd, LIBM_LOG_LN2LO, lo);                    // vfmadd231sd
  const double rr2 = r * r2;
  const double p34 = fma_rn(r, LIBM_LOG_A[4], LIBM_LOG_A[3]);
  const double lo2 = fma_rn(r2, LIBM_LOG_A[0], lo);
  const double p = fma_rn(p34, r2, p12);
  const double y = fma_rn(rr2, p, lo2);
  return y + hi;
}

constexpr double UT_LIBM_LOG2 = 0x1.62e42fefa39efp-1;   // libm log(2.0)

// math.log(x, 2.0) as CPython evaluates it: log(x) / log(2.0)
// (Modules/mathmodule.c loghelper: num = m_log(x), den = m_log(base))
UT_HD double py_log2(double x) { return libm_log(x) / UT_LIBM_LOG2; }

// ---------------------------------------------------------------------------
// Parameter value arithmetic (unit encoding) -- bit-exact restatement of
//   get_unit_value  manipulator.py:473-488
//   set_unit_value  manipulator.py:490-503
//   op4_set_linear  manipulator.py:523-542
// Compiled with -ffp-contract=off: every multiply and add rounds separately
// and in Python's left-to-right order.
// ---------------------------------------------------------------------------
UT_HD double py_min(double a, double b) { return (b < a) ? b : a; }  // Python min(a, b)
UT_HD double py_max(double a, double b) { return (b > a) ? b : a; }  // Python max(a, b)

}  // namespace ut
