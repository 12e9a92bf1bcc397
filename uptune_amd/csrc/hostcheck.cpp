// Host (g++) build of ut_core.h, used ONLY by tests/test_core_host.py to
// check the shared arithmetic against CPython (repr, hashlib) without a GPU.
// Nothing in the product path loads this library.
#include <stddef.h>
#include <string.h>
#include "ut_core.h"
#include "../../include/uthot.h"

namespace {
struct BufEmit {
  char* p;
  void put(int pos, uint8_t c) { p[pos] = (char)c; }
};
}  // namespace

extern "C" {
// C-ABI struct sizes as the C compiler lays them out (checked against the
// ctypes mirrors in uptune_amd/_lib.py)
long long uthc_sizeof(int which) {
  switch (which) {
    case 0: return (long long)sizeof(ut_param_desc);
    case 1: return (long long)sizeof(ut_gp_hyper);
    case 2: return (long long)sizeof(ut_round_out);
    case 3: return (long long)sizeof(ut_de_params);
    case 4: return (long long)sizeof(ut_acq);
    case 5: return (long long)sizeof(ut_pso_params);
    case 6: return (long long)sizeof(ut_ga_params);
    case 7: return (long long)sizeof(ut_tree_node);
    case 8: return (long long)sizeof(ut_prune_stats);
    default: return -1;
  }
}
int uthc_repr_double(double x, char* out) {
  BufEmit e{out};
  return ut::repr_double(x, e);
}
int uthc_repr_int64(long long v, char* out) {
  BufEmit e{out};
  return ut::repr_int64((int64_t)v, e);
}
void uthc_sha256(const unsigned char* msg, size_t len, unsigned char* out32) {
  uint32_t H[8];
  ut::sha256_init(H);
  size_t total = len + 9;
  size_t nblk = (total + 63) / 64;
  for (size_t b = 0; b < nblk; ++b) {
    uint32_t W[16];
    for (int w = 0; w < 16; ++w) {
      uint32_t v = 0;
      for (int t = 0; t < 4; ++t) {
        size_t pos = b * 64 + w * 4 + t;
        uint32_t byte;
        if (pos < len) byte = msg[pos];
        else if (pos == len) byte = 0x80;
        else if (pos >= nblk * 64 - 8) byte = (uint32_t)(((unsigned long long)len * 8) >> (8 * (nblk * 64 - 1 - pos))) & 0xFF;
        else byte = 0;
        v = (v << 8) | byte;
      }
      W[w] = v;
    }
    ut::sha256_compress(H, W);
  }
  for (int i = 0; i < 8; ++i)
    for (int t = 0; t < 4; ++t) out32[i * 4 + t] = (unsigned char)(H[i] >> (24 - 8 * t));
}
void uthc_philox(unsigned long long seed, unsigned long long cand, unsigned stream, unsigned round_, unsigned op,
                 unsigned* out4) {
  ut::u32x4 r = ut::draw(seed, cand, stream, round_, op);
  out4[0] = r.x; out4[1] = r.y; out4[2] = r.z; out4[3] = r.w;
}
void uthc_py_log2(const double* x, double* out, long long n) {
  for (long long i = 0; i < n; ++i) out[i] = ut::py_log2(x[i]);
}
void uthc_libm_log(const double* x, double* out, long long n) {
  for (long long i = 0; i < n; ++i) out[i] = ut::libm_log(x[i]);
}
void uthc_exp2(const double* x, double* out, long long n) {
  for (long long i = 0; i < n; ++i) out[i] = ut::exp2_cr(x[i]);
}
void uthc_logint_unscale(const double* s, double mn, double* out, long long n) {
  for (long long i = 0; i < n; ++i) out[i] = rint((ut::exp2_cr(s[i]) - 1.0) + mn);
}
void uthc_philox_raw(const unsigned* ctr4, const unsigned* key2, unsigned* out4) {
  ut::u32x4 c{ctr4[0], ctr4[1], ctr4[2], ctr4[3]};
  ut::u32x4 r = ut::philox4x32_10(c, key2[0], key2[1]);
  out4[0] = r.x; out4[1] = r.y; out4[2] = r.z; out4[3] = r.w;
}
}
