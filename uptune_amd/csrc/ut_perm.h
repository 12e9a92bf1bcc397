// ut_perm.h -- PermutationParameter operators on the device, one lane per
// candidate.  Bit-exact restatement of oracle/perm.py, which restates
//   op1_randomize            manipulator.py:1057-1064 (random.shuffle)
//   op1_small_random_change  manipulator.py:1066-1079
//   op3_cross_PX / PMX / CX / OX1 / OX3   manipulator.py:1179-1353
//   op3_cross / op3_swarm    manipulator.py:1096-1140
// with random.* replaced by the words of a perm draw site (ut_core.h
// perm_block).  A permutation is `size` SoA columns holding item indices (as
// f64); a lane's element k lives at base[k * ld] (ld = 1 for a row shared by
// every lane, e.g. the global best).  Scratch lists (PMX) live in a
// per-call workspace with the same [slot][ld] layout.
#pragma once
#include "ut_internal.h"

namespace ut {

enum : int32_t { X_NONE = 0, X_OX1 = 1, X_OX3 = 2, X_PX = 3, X_CX = 4, X_PMX = 5 };

struct PRow {  // read-only permutation of one lane
  const double* p;
  int64_t ld;
  __device__ __forceinline__ int32_t operator[](int32_t k) const { return (int32_t)p[(int64_t)k * ld]; }
};

struct WRow {  // writable permutation / scratch list of one lane
  double* p;
  int64_t ld;
  __device__ __forceinline__ int32_t get(int32_t k) const { return (int32_t)p[(int64_t)k * ld]; }
  __device__ __forceinline__ void set(int32_t k, int32_t v) const { p[(int64_t)k * ld] = (double)v; }
  __device__ __forceinline__ PRow ro() const { return PRow{p, ld}; }
};

// word stream of one draw site
struct PermRng {
  uint64_t seed, g;
  uint32_t stream, round_, op;
  uint32_t blk;
  u32x4 b;
  __device__ PermRng(uint64_t seed_, uint64_t g_, uint32_t stream_, uint32_t round__, uint32_t op_)
      : seed(seed_), g(g_), stream(stream_), round_(round__), op(op_), blk(~0u), b{0u, 0u, 0u, 0u} {}
  __device__ uint32_t word(uint32_t k) {
    const uint32_t q = k >> 2;
    if (q != blk) {
      blk = q;
      b = perm_block(seed, g, stream, round_, op, q);
    }
    const uint32_t s = k & 3u;
    return s == 0 ? b.x : (s == 1 ? b.y : (s == 2 ? b.z : b.w));
  }
};

// randint(a, b) = a + randbelow(b - a + 1)
__device__ __forceinline__ int32_t p_randint(uint32_t w, int32_t a, int32_t b) {
  return a + (int32_t)umulhi32(w, (uint32_t)(b - a + 1));
}

__device__ __forceinline__ void perm_copy(WRow dst, PRow src, int32_t S) {
  for (int32_t k = 0; k < S; ++k) dst.set(k, src[k]);
}

__device__ __forceinline__ bool perm_equal(PRow a, PRow b, int32_t S) {
  bool eq = true;
  for (int32_t k = 0; k < S && eq; ++k) eq = a[k] == b[k];
  return eq;
}

__device__ __forceinline__ void perm_identity(WRow dst, int32_t S) {
  for (int32_t k = 0; k < S; ++k) dst.set(k, k);
}

// random.shuffle(x): for i in reversed(range(1, len(x))): j = randbelow(i + 1); swap
__device__ __forceinline__ void perm_shuffle(WRow x, int32_t S, PermRng& R) {
  uint32_t s = 0;
  for (int32_t i = S - 1; i >= 1; --i, ++s) {
    const int32_t j = (int32_t)umulhi32(R.word(s), (uint32_t)(i + 1));
    const int32_t a = x.get(i), c = x.get(j);
    x.set(i, c);
    x.set(j, a);
  }
}

// op1_small_random_change(p = 0.25)
__device__ __forceinline__ void perm_small_change(WRow x, int32_t S, PermRng& R) {
  for (int32_t i = 1; i < S; ++i) {
    if ((double)R.word((uint32_t)(i - 1)) * (1.0 / 4294967296.0) < 0.25) {
      const int32_t a = x.get(i - 1), c = x.get(i);
      x.set(i - 1, c);
      x.set(i, a);
    }
  }
}

__device__ __forceinline__ int32_t default_d(int32_t S) {
  const int32_t d = (int32_t)rint((double)S * 0.3);  // int(round(size * 0.3))
  return d > 1 ? d : 1;
}

// OX1 (r2 = r1) / OX3: c1 = p1 minus p2[r2:r2+d]; out = c1[:r1] + p2[r2:r2+d] + c1[r1:]
__device__ void cross_ox(WRow out, PRow p1, PRow p2, int32_t S, int32_t d, bool ox3, PermRng& R) {
  if (d == 0) d = default_d(S);
  if (d > S) { perm_copy(out, p1, S); return; }
  const int32_t r1 = p_randint(R.word(0), 0, S - d);
  const int32_t r2 = ox3 ? p_randint(R.word(1), 0, S - d) : r1;
  int32_t k = 0;
  for (int32_t q = 0; q < S; ++q) {
    const int32_t x = p1[q];
    bool in = false;
    for (int32_t t = 0; t < d; ++t) in |= p2[r2 + t] == x;
    if (!in) {
      out.set(k < r1 ? k : k + d, x);
      ++k;
    }
  }
  for (int32_t t = 0; t < d; ++t) out.set(r1 + t, p2[r2 + t]);
}

// PX: sorted(p1[:c], key=p2.index) + p1[c:], c = randint(2, S)
__device__ void cross_px(WRow out, PRow p1, PRow p2, int32_t S, PermRng& R) {
  if (S < 2) { perm_copy(out, p1, S); return; }
  const int32_t c = p_randint(R.word(0), 2, S);
  int32_t k = 0;
  for (int32_t q = 0; q < S && k < c; ++q) {
    const int32_t x = p2[q];
    bool in = false;
    for (int32_t t = 0; t < c; ++t) in |= p1[t] == x;
    if (in) out.set(k++, x);
  }
  for (int32_t q = c; q < S; ++q) out.set(q, p1[q]);
}

// CX: the cycle through a random start takes p2's values
__device__ void cross_cx(WRow out, PRow p1, PRow p2, int32_t S, PermRng& R) {
  perm_copy(out, p1, S);
  const int32_t s = p_randint(R.word(0), 0, S - 1);
  int32_t i = s;
  for (int32_t n = 0; n < S; ++n) {
    out.set(i, p2[i]);
    const int32_t val = p1[i];
    int32_t nx = 0;
    while (nx < S && p2[nx] != val) ++nx;  // p2.index(val)
    i = nx;
    if (i == s || i >= S) break;
  }
}

// PMX, literally (manipulator.py:1198-1262): c1 / c2 lists in scratch
// slots [0, d) and [d, 2d), removed candidate positions flagged in [2d, 2d+S)
__device__ void cross_pmx(WRow out, PRow p1, PRow p2, int32_t S, int32_t d, WRow scr, PermRng& R) {
  if (d == 0) d = default_d(S);
  if (d > S) { perm_copy(out, p1, S); return; }
  const int32_t r = p_randint(R.word(0), 0, S - d);
  WRow A{scr.p, scr.ld}, B{scr.p + (int64_t)d * scr.ld, scr.ld}, F{scr.p + (int64_t)2 * d * scr.ld, scr.ld};
  for (int32_t q = 0; q < S; ++q) {
    out.set(q, (q >= r && q < r + d) ? p2[q] : p1[q]);
    F.set(q, 0);
  }
  for (int32_t t = 0; t < d; ++t) {
    A.set(t, p1[r + t]);
    B.set(t, p2[r + t]);
  }
  int32_t h = 0, len = d;  // the lists are A[h .. h+len), B[h .. h+len)
  while (len > 0) {
    const int32_t n = A.get(h);
    for (;;) {  // while c2[0] in c1
      const int32_t b0 = B.get(h);
      int32_t li = -1;
      for (int32_t t = h; t < h + len && li < 0; ++t)
        if (A.get(t) == b0) li = t;
      if (li < 0) break;
      if (n == b0) break;
      const int32_t link = B.get(li);
      for (int32_t t = li; t + 1 < h + len; ++t) {  // del c2[link_idx]; del c1[link_idx]
        B.set(t, B.get(t + 1));
        A.set(t, A.get(t + 1));
      }
      --len;
      B.set(h, link);
    }
    const int32_t b0 = B.get(h);
    if (n != b0) {
      int32_t ni = -1;
      for (int32_t t = h; t < h + len && ni < 0; ++t)
        if (B.get(t) == n) ni = t;
      if (ni >= 0) {
        B.set(ni, b0);
      } else {
        for (int32_t q = 0; q < S; ++q) {  // candidate_indices, ascending
          if (q >= r && q < r + d) continue;
          if (F.get(q)) continue;
          if (out.get(q) == b0) {
            out.set(q, A.get(h));
            F.set(q, 1);
            break;
          }
        }
      }
    }
    ++h;
    --len;
  }
}

// op3_cross_<xop>(out, p1, p2, d); out must not alias p1 or p2
__device__ void perm_cross(int32_t xop, WRow out, PRow p1, PRow p2, int32_t S, int32_t d, WRow scr, PermRng& R) {
  switch (xop) {
    case X_OX1: cross_ox(out, p1, p2, S, d, false, R); break;
    case X_OX3: cross_ox(out, p1, p2, S, d, true, R); break;
    case X_PX: cross_px(out, p1, p2, S, R); break;
    case X_CX: cross_cx(out, p1, p2, S, R); break;
    case X_PMX: cross_pmx(out, p1, p2, S, d, scr, R); break;
    default: perm_copy(out, p1, S); break;
  }
}

}  // namespace ut
