// Experiment (round 3): what bounds the f16x3 variance contraction, and a
// 256 x 256-tile variant.  Standalone; includes the library kernels.
//   base      the library's k_gp_var_h3 (blocked operands; round 3's shipped form)
//   w3<BK,NS,MODE>  256 x 256 tiles, 8 waves of 64 rows x 128 columns, NS-slot
//             glds ring of BK-k stages (2 x 64 KiB at BK 32, 4 x 32 KiB at BK 16)
//     MODE 0  as it would ship
//     MODE 1  no ring refills (LDS stale): MFMA + LDS reads + barriers only
//     MODE 2  B (K*) always from strip 0 (every B byte an L2 hit)
//     MODE 3  MODE 2 + A from row tile 0
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -I uptune_amd/csrc scripts/exp/h3_probe.hip -o gpurun_tmp/h3_probe
//   gpurun_tmp/h3_probe NPAD M REPS
// "base" is the library's shipped kernel (blocked operands, 256 x 256 tiles);
// the w3 kernels below read row-major planes or the blocked copies.
#include "../../uptune_amd/csrc/gp_gemm.hip"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <type_traits>

namespace ut {


// row-major-plane helpers (the round-2 kernel's, kept here for the w3 variants)
template <int BK>
__device__ __forceinline__ int p_swz(int r, int c) { return BK == 32 ? c ^ ((r >> 2) & 3) : c ^ ((r >> 3) & 1); }
template <int BK>
__device__ __forceinline__ void p_glds(const _Float16* __restrict__ src, int64_t ld, int32_t rb, int32_t k0,
                                       _Float16* plane, int lane) {
  constexpr int CH = BK / 8;
  const int rl = lane / CH;
  const int ch = p_swz<BK>(rb + rl, lane % CH);
  const _Float16* base = src + (int64_t)rb * ld + k0;
  const uint32_t loff = (uint32_t)rl * (uint32_t)ld + (uint32_t)(ch * 8);
  __builtin_amdgcn_global_load_lds(base + loff, (__attribute__((address_space(3))) void*)(plane + rb * BK), 16, 0, 0);
}
template <int BK>
__device__ __forceinline__ vh8 p_frag(const _Float16* plane, int r, int c) {
  return *reinterpret_cast<const vh8*>(plane + r * BK + (p_swz<BK>(r, c) << 3));
}

template <int BK>
struct W3 {
  static constexpr int BM = 256, BN = 256;
  static constexpr int SA = BM * BK;       // fp16 elements per plane (A and B alike)
  static constexpr int STAGE = 4 * SA;     // A hi, A lo, B hi, B lo
  static constexpr int RPI = 64 / (BK / 8);
};

template <int BK, int NS, int PART>
__device__ __forceinline__ void w3_issue(const _Float16* __restrict__ A, int64_t a_lo, const _Float16* __restrict__ B,
                                         int64_t b_lo, int64_t ld, int32_t k0, _Float16* st, int w, int lane) {
  using C = W3<BK>;
  constexpr int R = 32;  // rows per wave per plane
  if constexpr (PART & 1) {
#pragma unroll
    for (int u = 0; u < R / C::RPI; ++u) {
      p_glds<BK>(A, ld, w * R + u * C::RPI, k0, st, lane);
      p_glds<BK>(A + a_lo, ld, w * R + u * C::RPI, k0, st + C::SA, lane);
    }
  }
  if constexpr (PART & 2) {
#pragma unroll
    for (int u = 0; u < R / C::RPI; ++u) {
      p_glds<BK>(B, ld, w * R + u * C::RPI, k0, st + 2 * C::SA, lane);
      p_glds<BK>(B + b_lo, ld, w * R + u * C::RPI, k0, st + 3 * C::SA, lane);
    }
  }
}

// blocked, pre-swizzled operand layout: 256-row x 32-k blocks of 16 KiB per
// plane, block (rb, kb) at ((rb * (K / 32) + kb) * 8192) elements; inside a
// block row r, 16-B chunk c sits at r * 32 + ((c ^ ((r >> 2) & 3)) << 3): the
// LDS image, so a stage is two contiguous 16-KiB copies per operand
template <int PART>
__device__ __forceinline__ void w3_issue_blk(const _Float16* __restrict__ Ab, int64_t a_lo,
                                             const _Float16* __restrict__ Bb, int64_t b_lo, _Float16* st, int w,
                                             int lane) {
  constexpr int SA = 256 * 32;
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int off = w * 1024 + u * 512;  // this wave's two 1-KiB pieces of each 16-KiB block
    if constexpr (PART & 1) {
      __builtin_amdgcn_global_load_lds(Ab + off + lane * 8, (__attribute__((address_space(3))) void*)(st + off), 16, 0, 0);
      __builtin_amdgcn_global_load_lds(Ab + a_lo + off + lane * 8,
                                       (__attribute__((address_space(3))) void*)(st + SA + off), 16, 0, 0);
    }
    if constexpr (PART & 2) {
      __builtin_amdgcn_global_load_lds(Bb + off + lane * 8, (__attribute__((address_space(3))) void*)(st + 2 * SA + off),
                                       16, 0, 0);
      __builtin_amdgcn_global_load_lds(Bb + b_lo + off + lane * 8,
                                       (__attribute__((address_space(3))) void*)(st + 3 * SA + off), 16, 0, 0);
    }
  }
}

template <int BK, int NS, class Mid>
__device__ __forceinline__ void w3_step(const _Float16* st, int wm, int wn, int lane, int imin, vf16 (&acc)[2][4],
                                        Mid&& mid) {
  using C = W3<BK>;
  const _Float16* ah = st;
  const _Float16* al = st + C::SA;
  const _Float16* bh = st + 2 * C::SA;
  const _Float16* bl = st + 3 * C::SA;
#pragma unroll
  for (int s = 0; s < BK / 16; ++s) {
    if constexpr (BK / 16 > 1) {
      if (s == 1) {
        __builtin_amdgcn_sched_barrier(0);
        mid();
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    const int c = 2 * s + (lane >> 5);
    vh8 fbh[4], fbl[4];
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) {
      const int r = wn * 128 + jj * 32 + (lane & 31);
      fbh[jj] = p_frag<BK>(bh, r, c);
      fbl[jj] = p_frag<BK>(bl, r, c);
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      if (i < imin) continue;
      const int r = wm * 64 + i * 32 + (lane & 31);
      const vh8 fah = p_frag<BK>(ah, r, c), fal = p_frag<BK>(al, r, c);
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) {
        acc[i][jj] = __builtin_amdgcn_mfma_f32_32x32x16_f16(fal, fbh[jj], acc[i][jj], 0, 0, 0);
        acc[i][jj] = __builtin_amdgcn_mfma_f32_32x32x16_f16(fah, fbl[jj], acc[i][jj], 0, 0, 0);
        acc[i][jj] = __builtin_amdgcn_mfma_f32_32x32x16_f16(fah, fbh[jj], acc[i][jj], 0, 0, 0);
      }
    }
  }
}

// part rows: one per 256-row tile (RT2 of them)
template <int BK, int NS, int MODE, bool BLK = false>
__global__ __launch_bounds__(512, 2) void k_h3w(const _Float16* __restrict__ A, int64_t a_lo,
                                                const _Float16* __restrict__ B, int64_t b_lo, int64_t ld, int32_t K,
                                                int32_t RT2, int32_t CT, int64_t m, int32_t* __restrict__ ticket,
                                                double* __restrict__ part, int64_t ldp, double unscale2) {
  using C = W3<BK>;
  static_assert(NS * C::STAGE * 2 <= 160 * 1024 - 64, "LDS");
  __shared__ __attribute__((aligned(16))) _Float16 lds[NS * C::STAGE + 8];
  int32_t& s_item = *reinterpret_cast<int32_t*>(lds + NS * C::STAGE);
  const int t = threadIdx.x, lane = t & 63;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  // waves w and w + 4 share a SIMD: give them row groups wm and 3 - wm so the
  // diagonal block's skipped work is balanced per SIMD
  const int wm = w < 4 ? w : 7 - w, wn = w < 4 ? 0 : 1;
  const int32_t xcd = blockIdx.x & 7;

  for (;;) {
    if (t == 0) s_item = atomicAdd(&ticket[xcd], 1);
    __syncthreads();
    const int32_t j = s_item;
    const int32_t ct = (j / RT2) * 8 + xcd;
    if (ct >= CT) break;
    const int32_t rt = RT2 - 1 - (j % RT2);
    const int64_t col0 = (int64_t)ct * C::BN;
    const int32_t row0 = rt * C::BM;
    const int32_t nk = min(K, row0 + C::BM) / BK;
    const _Float16* At = A + (int64_t)(MODE == 3 ? 0 : row0) * ld;
    const _Float16* Bt = B + (MODE >= 2 ? 0 : col0) * ld;

    vf16 acc[2][4];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int jj = 0; jj < 4; ++jj)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[i][jj][r] = 0.0f;

    const int32_t KB = K / 32;
    const _Float16* Ab = A + (int64_t)(MODE == 3 ? 0 : rt) * KB * 8192;
    const _Float16* Bb = B + (MODE >= 2 ? 0 : (int64_t)ct) * KB * 8192;
    auto issue = [&](int32_t kt, _Float16* dst, auto part) {
      constexpr int P = decltype(part)::value;
      if constexpr (BLK) {
        static_assert(BK == 32, "blocked layout: 32-k stages");
        w3_issue_blk<P>(Ab + (int64_t)kt * 8192, a_lo, Bb + (int64_t)kt * 8192, b_lo, dst, w, lane);
      } else {
        w3_issue<BK, NS, P>(At, a_lo, Bt, b_lo, ld, kt * BK, dst, w, lane);
      }
    };
    using P1 = std::integral_constant<int, 1>;
    using P2 = std::integral_constant<int, 2>;
    using P3 = std::integral_constant<int, 3>;
#pragma unroll
    for (int q = 0; q < NS - 1; ++q)
      if (q < nk) issue(q, lds + q * C::STAGE, P3{});
    constexpr bool SPLIT = BK / 16 > 1;
    constexpr int PW = 4 * 32 / C::RPI;  // glds per wave per stage
    auto pipe = [&](int32_t kt) -> const _Float16* {
      if (MODE != 1) {
        if (kt + NS - 2 < nk)
          wait_vmcnt<PW * (NS - 2)>();
        else
          wait_vmcnt<0>();
      }
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      if (MODE != 1 && kt + NS - 1 < nk) {
        if constexpr (SPLIT) issue(kt + NS - 1, lds + ((kt + NS - 1) % NS) * C::STAGE, P1{});
        else issue(kt + NS - 1, lds + ((kt + NS - 1) % NS) * C::STAGE, P3{});
      }
      return lds + (kt % NS) * C::STAGE;
    };
    auto refill_b = [&](int32_t kt) {
      return [&, kt]() {
        if (MODE != 1 && SPLIT && kt + NS - 1 < nk) issue(kt + NS - 1, lds + ((kt + NS - 1) % NS) * C::STAGE, P2{});
      };
    };
    const int32_t nfull = min(nk, row0 / BK);
    for (int32_t kt = 0; kt < nfull; ++kt) w3_step<BK, NS>(pipe(kt), wm, wn, lane, 0, acc, refill_b(kt));
    for (int32_t kt = nfull; kt < nk; ++kt) {
      const _Float16* st = pipe(kt);
      const int kd = ((kt - nfull) * BK) / 32 - 2 * wm;
      const int imin = kd < 0 ? 0 : kd;
      if (imin < 2) w3_step<BK, NS>(st, wm, wn, lane, imin, acc, refill_b(kt));
      else refill_b(kt)();
    }
    if (MODE == 1) wait_vmcnt<0>();

    __syncthreads();
    double* red = reinterpret_cast<double*>(lds);  // [4][256]
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) {
      const int cl = wn * 128 + jj * 32 + (lane & 31);
      double s = 0.0;
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) s += (double)acc[i][jj][r] * (double)acc[i][jj][r];
      s += __shfl_xor(s, 32);
      if ((lane >> 5) == 0) red[wm * 256 + cl] = s;
    }
    __syncthreads();
    if (t < 256) {
      const int64_t col = col0 + t;
      if (col < m) part[(int64_t)rt * ldp + col] = ((red[t] + red[256 + t]) + (red[512 + t] + red[768 + t])) * unscale2;
    }
  }
}


// q4: one wave per SIMD (a 4-wave workgroup, up to 512 VGPRs per lane), 256 x 256
// tiles on the blocked operands, each wave 128 rows x 128 columns (4 x 4 blocks
// of 32 x 32: 256 accumulator registers); 16 ds_read_b128 per 48 MFMAs (0.33
// per MFMA against 0.5 at 8 waves); each wave issues 16 of a stage's 64 glds,
// four between every k16 sub-step's MFMA groups.
//   MODE 0 as it would ship, 1 no refills
template <int MODE>
__global__ __launch_bounds__(256, 1) void k_h3q(const _Float16* __restrict__ A, int64_t a_lo,
                                                const _Float16* __restrict__ B, int64_t b_lo, int32_t K, int32_t RT2,
                                                int32_t CT, int64_t m, int32_t* __restrict__ ticket,
                                                double* __restrict__ part, int64_t ldp, double unscale2) {
  __shared__ __attribute__((aligned(16))) _Float16 lds[H3_NS * H3_STAGE + 8];
  int32_t& s_item = *reinterpret_cast<int32_t*>(lds + H3_NS * H3_STAGE);
  const int t = threadIdx.x, lane = t & 63;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const int wm = w >> 1, wn = w & 1;
  const int32_t xcd = blockIdx.x & 7;
  const int32_t KB = K / H3_BK;
  // this wave's 16 pieces of a stage: plane p (0 A hi, 1 A lo, 2 B hi, 3 B lo), pieces 4w .. 4w+3 of 16 per plane
  auto issue_part = [&](const _Float16* Ab, const _Float16* Bb, _Float16* st, int part_) {
    // part_ 0..3: plane part_
    const _Float16* src = part_ == 0 ? Ab : part_ == 1 ? Ab + a_lo : part_ == 2 ? Bb : Bb + b_lo;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int off = (w * 4 + u) * 512;
      __builtin_amdgcn_global_load_lds(src + off + lane * 8,
                                       (__attribute__((address_space(3))) void*)(st + part_ * H3_BLK + off), 16, 0, 0);
    }
  };
  for (;;) {
    if (t == 0) s_item = atomicAdd(&ticket[xcd], 1);
    __syncthreads();
    const int32_t j = s_item;
    const int32_t ct = (j / RT2) * 8 + xcd;
    if (ct >= CT) break;
    const int32_t rt = RT2 - 1 - (j % RT2);
    const int32_t row0 = rt * H3_BM;
    const int32_t nk = min(K, row0 + H3_BM) / H3_BK;
    const _Float16* Ab = A + (int64_t)rt * KB * H3_BLK;
    const _Float16* Bb = B + (int64_t)ct * KB * H3_BLK;
    vf16 acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int jj = 0; jj < 4; ++jj)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[i][jj][r] = 0.0f;
    for (int q = 0; q < 4; ++q) issue_part(Ab, Bb, lds, q);
    const int32_t nfull = min(nk, row0 / H3_BK);
    for (int32_t kt = 0; kt < nk; ++kt) {
      if (MODE != 1) wait_vmcnt<0>();
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      const bool nxt = MODE != 1 && kt + 1 < nk;
      _Float16* nst = lds + ((kt + 1) & 1) * H3_STAGE;
      const _Float16* st = lds + (kt & 1) * H3_STAGE;
      const _Float16* ah = st;
      const _Float16* al = st + H3_BLK;
      const _Float16* bh = st + 2 * H3_BLK;
      const _Float16* bl = st + 3 * H3_BLK;
      const int kd = kt < nfull ? -100 : (kt - nfull) - 4 * wm;   // 32-row blocks above the diagonal
      const int imin = kd < 0 ? 0 : kd;
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        const int c = 2 * s2 + (lane >> 5);
        vh8 fbh[4], fbl[4];
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
          const int r = wn * 128 + jj * 32 + (lane & 31);
          fbh[jj] = h3_frag(bh, r, c);
          fbl[jj] = h3_frag(bl, r, c);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          if (nxt && (i & 1) == 0) {
            __builtin_amdgcn_sched_barrier(0);
            issue_part(Ab + (int64_t)(kt + 1) * H3_BLK, Bb + (int64_t)(kt + 1) * H3_BLK, nst, 2 * s2 + (i >> 1));
            __builtin_amdgcn_sched_barrier(0);
          }
          if (i < imin) continue;
          const int r = wm * 128 + i * 32 + (lane & 31);
          const vh8 fah = h3_frag(ah, r, c), fal = h3_frag(al, r, c);
#pragma unroll
          for (int jj = 0; jj < 4; ++jj) {
            acc[i][jj] = __builtin_amdgcn_mfma_f32_32x32x16_f16(fal, fbh[jj], acc[i][jj], 0, 0, 0);
            acc[i][jj] = __builtin_amdgcn_mfma_f32_32x32x16_f16(fah, fbl[jj], acc[i][jj], 0, 0, 0);
            acc[i][jj] = __builtin_amdgcn_mfma_f32_32x32x16_f16(fah, fbh[jj], acc[i][jj], 0, 0, 0);
          }
        }
      }
    }
    if (MODE == 1) wait_vmcnt<0>();
    __syncthreads();
    double* red = reinterpret_cast<double*>(lds);  // [2][256]
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) {
      const int cl = wn * 128 + jj * 32 + (lane & 31);
      double sum = 0.0;
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) sum += (double)acc[i][jj][r] * (double)acc[i][jj][r];
      sum += __shfl_xor(sum, 32);
      if ((lane >> 5) == 0) red[wm * 256 + cl] = sum;
    }
    __syncthreads();
    {
      const int64_t col = (int64_t)ct * 256 + t;
      if (col < m) part[(int64_t)rt * ldp + col] = (red[t] + red[256 + t]) * unscale2;
    }
  }
}

}  // namespace ut

using namespace ut;

#define CK(x)                                                                           \
  do {                                                                                  \
    hipError_t e = (x);                                                                 \
    if (e != hipSuccess) {                                                              \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e)); \
      exit(1);                                                                          \
    }                                                                                   \
  } while (0)

// hi plane ~ U(-1, 1) in fp16, lo plane = a value below hi's half-ulp; A lower
// triangular ([row][k] zero for k > row) when tri
__global__ void k_fill16(_Float16* p, int64_t rows, int64_t ld, int64_t lo_off, uint64_t seed, int tri) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < rows * ld; i += (int64_t)gridDim.x * blockDim.x) {
  uint64_t x = (uint64_t)i * 0x9E3779B97F4A7C15ull + seed;
  x ^= x >> 31;
  x *= 0xBF58476D1CE4E5B9ull;
  x ^= x >> 29;
  float v = (float)((double)(x >> 11) * (1.0 / 9007199254740992.0) - 0.5) * 2.0f;
  float lo = (float)((double)((x >> 3) & 0xFFFF) / 65536.0 - 0.5) * 9.765625e-4f * fabsf(v);
  if (tri && (i % ld) > (i / ld)) v = lo = 0.0f;
  p[i] = (_Float16)v;
  p[lo_off + i] = (_Float16)lo;
  }
}

// row-major planes [R][K] -> blocked planes (w3_issue_blk's layout)
__global__ void k_to_blk(const _Float16* src, int64_t lo_src, _Float16* dst, int64_t lo_dst, int64_t R, int32_t K) {
  const int64_t n = R * K;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = i / K;
    const int32_t k = (int32_t)(i % K);
    const int rr = (int)(r & 255), c = (k & 31) >> 3;
    const int64_t o = ((r >> 8) * (K / 32) + (k >> 5)) * 8192 + rr * 32 + ((c ^ ((rr >> 2) & 3)) << 3) + (k & 7);
    dst[o] = src[i];
    dst[lo_dst + o] = src[lo_src + i];
  }
}

__global__ void k_colsum(const double* part, int32_t R, int64_t ldp, int64_t m, double* out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= m) return;
  double s = 0;
  for (int r = 0; r < R; ++r) s += part[(int64_t)r * ldp + i];
  out[i] = s;
}

int main(int argc, char** argv) {
  const int npad = argc > 1 ? atoi(argv[1]) : 4096;
  const int64_t m = argc > 2 ? atoll(argv[2]) : (1 << 21);
  const int reps = argc > 3 ? atoi(argv[3]) : 3;
  const int64_t ldk = ((m + 255) / 256) * 256;
  _Float16 *A, *B;
  double *part, *cs;
  CK(hipMalloc(&A, sizeof(_Float16) * 2 * (int64_t)npad * npad));
  CK(hipMalloc(&B, sizeof(_Float16) * 2 * (int64_t)npad * ldk));
  const int RT = npad / 128, RT2 = npad / 256;
  CK(hipMalloc(&part, sizeof(double) * RT * ldk));
  CK(hipMalloc(&cs, sizeof(double) * ldk));
  const int64_t na = (int64_t)npad * npad, nb = (int64_t)npad * ldk;
  k_fill16<<<65536, 256>>>(A, npad, npad, na, 1, 1);
  k_fill16<<<65536, 256>>>(B, ldk, npad, nb, 2, 0);
  unsigned long long* amax;
  CK(hipMalloc(&amax, 8));
  const double one = 1.0;
  CK(hipMemcpy(amax, &one, 8, hipMemcpyHostToDevice));
  CK(hipDeviceSynchronize());
  int32_t* ticket;
  CK(hipMalloc(&ticket, sizeof(int32_t) * 8));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const double flops = (double)m * npad * (npad + 1);
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  const int ncu = prop.multiProcessorCount;
  printf("npad %d m %lld ncu %d\n", npad, (long long)m, ncu);
  auto timeit = [&](const char* name, auto launch) {
    auto one_ = [&] {
      CK(hipMemsetAsync(ticket, 0, sizeof(int32_t) * 8, 0));
      launch();
    };
    one_();
    CK(hipGetLastError());
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    for (int r = 0; r < reps; ++r) one_();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    ms /= reps;
    printf("%-44s %9.3f ms  %7.1f TF/s  (%.3f of 839)\n", name, ms, flops / ms * 1e-9, flops / ms * 1e-9 / 839.0);
    fflush(stdout);
  };
  std::vector<double> ref(m), got(m);
  auto colsum = [&](int R, std::vector<double>& dst) {
    k_colsum<<<(unsigned)((m + 255) / 256), 256>>>(part, R, ldk, m, cs);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(dst.data(), cs, sizeof(double) * m, hipMemcpyDeviceToHost));
  };
  const int CT = (int)(ldk / 256);
  auto cmp = [&](const char* what) {
    double md = 0;
    for (int64_t q = 0; q < m; ++q) md = std::max(md, std::abs(ref[q] - got[q]) / (std::abs(ref[q]) + 1e-30));
    printf("    %s vs base: max rel diff %.3e\n", what, md);
    fflush(stdout);
  };
#define W3RUN(BK, NS, MODE, NAME)                                                                                \
  timeit(NAME, [&] {                                                                                            \
    hipLaunchKernelGGL((k_h3w<BK, NS, MODE>), dim3(ncu), dim3(512), 0, 0, A, na, B, nb, (int64_t)npad, npad, RT2, \
                       CT, m, ticket, part, ldk, 1.0);                                                          \
  })
  _Float16 *Ab, *Bb;
  CK(hipMalloc(&Ab, sizeof(_Float16) * 2 * na));
  CK(hipMalloc(&Bb, sizeof(_Float16) * 2 * nb));
  k_to_blk<<<65536, 256>>>(A, na, Ab, na, npad, npad);
  k_to_blk<<<65536, 256>>>(B, nb, Bb, nb, ldk, npad);
  CK(hipDeviceSynchronize());
  timeit("base: library k_gp_var_h3 (blocked)", [&] {
    hipLaunchKernelGGL(k_gp_var_h3, dim3(ncu), dim3(512), 0, 0, Ab, na, Bb, nb, npad, RT2, CT, m, ticket, part, ldk,
                       amax, -14);
  });
  colsum(RT2, ref);
  timeit("q4: one wave per SIMD, 128 x 128 per wave", [&] {
    hipLaunchKernelGGL((k_h3q<0>), dim3(ncu), dim3(256), 0, 0, Ab, na, Bb, nb, npad, RT2, CT, m, ticket, part, ldk, 1.0);
  });
  colsum(RT2, got);
  cmp("q4");
  timeit("q4 no refills", [&] {
    hipLaunchKernelGGL((k_h3q<1>), dim3(ncu), dim3(256), 0, 0, Ab, na, Bb, nb, npad, RT2, CT, m, ticket, part, ldk, 1.0);
  });
  W3RUN(32, 2, 0, "w3 BK32 NS2 (row-major planes)");
  colsum(RT2, got);
  cmp("w3 BK32 NS2");
  {
    timeit("w3 BK32 NS2 blocked", [&] {
      hipLaunchKernelGGL((k_h3w<32, 2, 0, true>), dim3(ncu), dim3(512), 0, 0, Ab, na, Bb, nb, (int64_t)npad, npad, RT2,
                         CT, m, ticket, part, ldk, 1.0);
    });
    colsum(RT2, got);
    cmp("w3 blocked");
    timeit("w3 BK32 NS2 blocked, A tile 0, B strip 0", [&] {
      hipLaunchKernelGGL((k_h3w<32, 2, 3, true>), dim3(ncu), dim3(512), 0, 0, Ab, na, Bb, nb, (int64_t)npad, npad, RT2,
                         CT, m, ticket, part, ldk, 1.0);
    });
    timeit("w3 BK32 NS2 blocked, B strip 0", [&] {
      hipLaunchKernelGGL((k_h3w<32, 2, 2, true>), dim3(ncu), dim3(512), 0, 0, Ab, na, Bb, nb, (int64_t)npad, npad, RT2,
                         CT, m, ticket, part, ldk, 1.0);
    });
  }
  CK(hipFree(Ab));
  CK(hipFree(Bb));
  W3RUN(16, 4, 0, "w3 BK16 NS4");
  colsum(RT2, got);
  cmp("w3 BK16 NS4");
  W3RUN(32, 2, 1, "w3 BK32 NS2 no refills");
  W3RUN(32, 2, 2, "w3 BK32 NS2 B strip 0");
  W3RUN(32, 2, 3, "w3 BK32 NS2 A tile 0, B strip 0");
  W3RUN(16, 4, 1, "w3 BK16 NS4 no refills");
  W3RUN(16, 4, 2, "w3 BK16 NS4 B strip 0");
  return 0;
}
