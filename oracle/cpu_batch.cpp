// cpu_batch.cpp -- TEST / MEASUREMENT INFRASTRUCTURE, not the product.
//
// Batch CPU baseline "B1" of SURVEY.md §8(d)(ii): the same algorithms as the
// device path, vectorised over candidates on every host core (OpenMP), for
// bench.py's cpu_baseline leg and the CPU tests that pin it to the oracle.
// Nothing under uptune_amd/ loads this library.
//
//   cpub_de_hash_float   DE/rand/1/bin trial per candidate (oracle/de.py,
//                        differentialevolution.py:105-129) for FloatParameter
//                        spaces, then hash_config (oracle/hashing.py,
//                        manipulator.py:233-243, Python-3 layout) of the trial
//   cpub_dedup           history set + in-batch first occurrence (oracle/select.py)
//
// The per-candidate arithmetic is the shared restatement in
// uptune_amd/csrc/ut_core.h (Philox draws, CPython repr(float)), compiled here
// with g++ -O3 -fopenmp -ffp-contract=off; SHA-256 is OpenSSL's (libcrypto,
// SHA-NI where the CPU has it) -- the implementation CPython's hashlib calls,
// so the baseline hashes as fast as the host can.
#include <openssl/sha.h>
#include <stdint.h>
#include <string.h>

#include <string>
#include <unordered_set>
#include <vector>

#include "../uptune_amd/csrc/ut_core.h"

namespace {

struct BufEmit {
  char* p;
  void put(int pos, uint8_t c) { p[pos] = (char)c; }
};

const char HEX[] = "0123456789abcdef";

// OpenSSL's low-level SHA-256 (SHA256_Init/Update/Final: straight to the
// SHA-NI / AVX2 block function; the one-shot SHA256() goes through the EVP
// fetch path, whose locking serialised the OpenMP threads)
inline void sha256(const void* p, size_t n, uint8_t out[32]) {
  SHA256_CTX c;
  SHA256_Init(&c);
  SHA256_Update(&c, p, n);
  SHA256_Final(out, &c);
}

void pick_donors(uint32_t w0, uint32_t w1, uint32_t w2, int64_t npop, int64_t t, int64_t& d1, int64_t& d2,
                 int64_t& d3) {
  const int64_t Q = npop - 1;
  const int64_t a = (int64_t)ut::umulhi32(w0, (uint32_t)Q);
  int64_t b = (int64_t)ut::umulhi32(w1, (uint32_t)(Q - 1));
  b += (b >= a);
  const int64_t s0 = a < b ? a : b, s1 = a < b ? b : a;
  int64_t c = (int64_t)ut::umulhi32(w2, (uint32_t)(Q - 2));
  c += (c >= s0);
  c += (c >= s1);
  d1 = a + (a >= t);
  d2 = b + (b >= t);
  d3 = c + (c >= t);
}

struct Dig {
  uint8_t b[32];
  bool operator==(const Dig& o) const { return memcmp(b, o.b, 32) == 0; }
};
struct DigHash {
  size_t operator()(const Dig& d) const {
    size_t h;
    memcpy(&h, d.b, sizeof h);
    return h;
  }
};

}  // namespace

extern "C" {

// pop: [P][npop] stored values; trial: [P][m]; digest: [m][32].  lo/hi: the
// FloatParameter bounds; order[r] = param index at sorted position r; the
// name of param p is names[name_off[p] .. name_off[p + 1]).
int cpub_de_hash_float(int32_t P, const double* lo, const double* hi, const int32_t* order, const char* names,
                       const int32_t* name_off, const double* pop, int64_t npop, uint64_t seed, uint32_t round_,
                       int64_t cand_base, int64_t m, double cr, int32_t n_cross, double* trial, uint8_t* digest) {
  if (P < 1 || npop < 4 || n_cross < 0 || n_cross > 4) return -1;
  // outer-message pieces that do not depend on the candidate: name_i and str(i) + "|"
  std::vector<std::string> head(P), tail(P);
  for (int r = 0; r < P; ++r) {
    const int p = order[r];
    head[r].assign(names + name_off[p], names + name_off[p + 1]);
    tail[r] = std::to_string(r) + "|";
  }
#pragma omp parallel for schedule(static, 256)
  for (int64_t i = 0; i < m; ++i) {
    const uint64_t g = (uint64_t)(cand_base + i);
    const int64_t t = (int64_t)(g % (uint64_t)npop);
    const ut::u32x4 rc = ut::draw(seed, g, ut::STREAM_CAND | 0u, round_, ut::OP_DE);
    int64_t d1, d2, d3;
    pick_donors(rc.x, rc.y, rc.z, npop, t, d1, d2, d3);
    const ut::u32x4 rf = ut::draw(seed, g, ut::STREAM_CAND | 1u, round_, ut::OP_DE);
    const double F = ut::u01_from(rf.x, rf.y) / 2.0 + 0.5;
    int32_t fset[4];
    ut::de_forced_set(ut::draw(seed, g, ut::STREAM_CAND | 2u, round_, ut::OP_DE), P, n_cross, fset);
    ut::u32x4 r{0, 0, 0, 0};
    for (int32_t p = 0; p < P; ++p) {
      if ((p & 3) == 0) r = ut::draw(seed, g, ut::STREAM_CAND | (ut::DE_CR_STREAM + (uint32_t)(p >> 2)), round_, ut::OP_DE);
      const uint32_t w = (p & 3) == 0 ? r.x : (p & 3) == 1 ? r.y : (p & 3) == 2 ? r.z : r.w;
      const bool forced = p == fset[0] || p == fset[1] || p == fset[2] || p == fset[3];
      const double* col = pop + (int64_t)p * npop;
      double v = col[t];
      if (forced || ut::de_cr_pass(w, cr)) {
        const double span = hi[p] - lo[p];
        if (lo[p] < hi[p]) {
          const double va = (col[d1] - lo[p]) / span, vb = (col[d2] - lo[p]) / span, vc = (col[d3] - lo[p]) / span;
          double u = (1.0 * va + F * vb) + (-F) * vc;
          u = ut::py_max(0.0, ut::py_min(u, 1.0));
          double val = u * span + lo[p];
          v = ut::py_max(lo[p], ut::py_min(val, hi[p]));
        }
      }
      trial[(int64_t)p * m + i] = v;
    }
    // hash_config: sha256 over name ‖ str(sha256(repr(v)).hexdigest().encode()) ‖ str(i) ‖ "|"
    thread_local std::string msg;
    msg.clear();
    for (int r = 0; r < P; ++r) {
      const int p = order[r];
      char rep[40];
      BufEmit e{rep};
      const int n = ut::repr_double(trial[(int64_t)p * m + i], e);
      uint8_t d[32];
      sha256(rep, (size_t)n, d);
      char hx[67];
      hx[0] = 'b';
      hx[1] = '\'';
      for (int k = 0; k < 32; ++k) {
        hx[2 + 2 * k] = HEX[d[k] >> 4];
        hx[3 + 2 * k] = HEX[d[k] & 15];
      }
      hx[66] = '\'';
      msg.append(head[r]);
      msg.append(hx, 67);
      msg.append(tail[r]);
    }
    sha256(msg.data(), msg.size(), digest + 32 * i);
  }
  return 0;
}

// dup[i] = 1 if digest i is in the history or repeats an earlier candidate
int64_t cpub_dedup(const uint8_t* digest, int64_t m, const uint8_t* hist, int64_t nh, uint8_t* dup) {
  std::unordered_set<Dig, DigHash> seen;
  seen.reserve((size_t)(m + nh) * 2);
  Dig d;
  for (int64_t j = 0; j < nh; ++j) {
    memcpy(d.b, hist + 32 * j, 32);
    seen.insert(d);
  }
  int64_t n = 0;
  for (int64_t i = 0; i < m; ++i) {
    memcpy(d.b, digest + 32 * i, 32);
    dup[i] = seen.insert(d).second ? 0 : 1;
    n += dup[i];
  }
  return n;
}

}  // extern "C"
