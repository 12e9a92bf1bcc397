// ut_internal.h -- context, device-side space description and launch
// helpers shared by the libuthot translation units.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <algorithm>
#include <functional>
#include <initializer_list>
#include <string>
#include <vector>

#include "../../include/uthot.h"
#include "ut_core.h"

namespace ut {

// Per-parameter record in device memory (uniform across a wave: every lane of
// a candidate-parallel kernel reads the same record, so these become scalar
// loads).
struct DevParam {
  int32_t kind;
  int32_t hash_mode;   // HM_LUT / HM_FLOAT / HM_INT / HM_LOGINT
  int64_t lut_base;    // first digest of this param in the LUT buffer
  int64_t lut_n;       // LUT entries (indices are clamped to [0, lut_n))
  double lo, hi;       // FLOAT/INT/LOGINT: stored-value bounds (min_value, max_value);
                       // POW2: exponent bounds (its legal_range, manipulator.py:829-830)
  double u_lo, u_hi;   // unit-encoding range of the searched value (get_value):
                       // widened for integer types; LOGINT: the scaled legal_range
  double u_span;       // u_hi - u_lo, rounded as Python rounds it
  int64_t n_opt;       // ENUM/BOOL option count
  int32_t feat_col;    // first GP feature column
  int32_t n_feat;      // GP feature columns of this param
  int64_t vtab_base;   // LOGINT: first entry of get_value(v) for v = lo.. in the value table
  int64_t vtab_n;      // LOGINT: table entries; 0 = compute the log on the device
  int32_t col;         // first SoA value column (PERM: `psize` columns of item indices)
  int32_t psize;       // PERM: permutation size S; 1 for every other kind
  int32_t wcol;        // PERM: first of its S columns in the GA parent workspace
  int32_t pslot;       // PERM: slot of its inner digest in the per-round perm digest buffer
  int32_t cslot;       // HM_FLOAT / HM_INT / HM_LOGINT (inner digest computed on the device):
                       // its slot in the population inner-digest cache; -1 otherwise
  int32_t pad_;
};

enum : int32_t { HM_LUT = 0, HM_FLOAT = 1, HM_INT = 2, HM_LOGINT = 3, HM_PERM = 4 };

// One 32-bit word of the fixed-layout outer hash message: the constant bytes
// plus, when the word overlaps a digest "hole", where its hex bytes come from
// in the kernel's 32-register hex array (hole j lives in slot j % 2).  8 bytes,
// read with scalar loads (every lane of a wave uses the same word).
struct HashWord {
  uint32_t tmpl;   // constant bytes (zero where hex characters go)
  uint32_t info;   // 0 = no hole; else HW_* fields
};
enum : uint32_t {
  HW_LO_VALID = 1u << 6,   // bits 0..4: hex register of the word's first bytes
  HW_HI_POS = 8,           // bits 8..12: hex register of its last bytes
  HW_HI_VALID = 1u << 14,
  HW_SHIFT_POS = 16,       // bits 16..20: left shift of the 64-bit concatenation, in bits
  HW_HOLE = 1u << 31,
};

struct Space {
  int32_t P = 0;                          // parameters
  int32_t ncols = 0;                      // SoA value columns (P + sum over PERM of size - 1)
  int32_t n_perm = 0;                     // PERM parameters
  int32_t perm_cols = 0;                  // sum of PERM sizes
  int32_t perm_smax = 0;                  // largest PERM size
  int32_t n_feat = 0;
  int32_t py2 = 0;
  std::vector<DevParam> host_params;
  std::vector<int32_t> host_order;        // sorted position -> param index
  int64_t outer_len = 0;
  int64_t outer_blocks = 0;
  DevParam* d_params = nullptr;
  int32_t* d_order = nullptr;             // sorted position -> param index
  HashWord* d_words = nullptr;            // outer_blocks * 16
  int32_t* d_block_last = nullptr;        // last sorted position needed by each block
  uint32_t* d_lut = nullptr;              // digests as hex [*][16 words]
  double* d_vtab = nullptr;               // LOGINT get_value tables (host-computed by CPython)
  int32_t* d_order_col = nullptr;         // sorted position -> first value column
  int32_t* d_perm_params = nullptr;       // PERM param indices, by digest slot
  uint8_t* d_perm_bytes = nullptr;        // concatenated repr(item) bytes of every PERM param
  int32_t* d_perm_off = nullptr;          // per PERM param: S + 1 offsets into d_perm_bytes
  int32_t* d_perm_offbase = nullptr;      // per PERM slot: first entry in d_perm_off
  int32_t* d_perm_len = nullptr;          // per PERM slot: len(repr(list)) (constant per param)
  int32_t n_comp = 0;                     // params whose inner digest is computed (cslot >= 0)
  int32_t* d_comp = nullptr;              // cslot -> param index
  int32_t* d_col_param = nullptr;         // value column -> its param (first column of a non-PERM param), or -1
  // categorical K* (gp_gemm.hip): ENUM / BOOL params are one-hot blocks of the
  // GP features, so their part of |x - u|^2 is (2 or 1) / ell^2 per mismatching
  // param -- an integer dot product of one-hot codes, taken on the int8 MFMA;
  // the other ("numeric") features go through the fp64 K* contraction
  int32_t n_cat = 0;                      // ENUM + BOOL params
  int32_t cat_k = 0;                      // int8 code columns (ENUM: n_opt, BOOL: 2), padded to 128
  int32_t n_num = 0;                      // numeric features
  std::vector<int32_t> host_cat;          // the ENUM / BOOL param indices
  std::vector<int32_t> host_num_feat;     // numeric k -> feature column
  int32_t* d_cat_ccol = nullptr;          // per param: first code column (-1: numeric param)
  int32_t* d_num_feat = nullptr;          // numeric k -> feature column
  int32_t* d_feat_num = nullptr;          // feature column -> numeric k, or -1 (categorical)
};

template <class T>
struct DevBuf {
  T* p = nullptr;
  size_t n = 0;
};

// Per-stage device time of the scoring rounds: events are recorded while the
// rounds run and read only when a stage time is asked for, so timing adds no
// host synchronisation between rounds (consecutive rounds still overlap).
struct Timing {
  struct Mark {
    std::string name;   // "" = a stream's start point in its round, not reported
    hipStream_t stream;
    hipEvent_t ev;
    int64_t round;
  };
  bool on = false;
  bool in_round = false;   // inside ut_score_round_* (its stages share one round)
  int64_t round = 0;
  std::vector<Mark> marks;  // a stage's time = its mark - the previous mark of the round on the same stream
  std::vector<std::pair<std::string, std::pair<double, int64_t>>> totals;  // name -> (sum ms, rounds)
};

}  // namespace ut

struct ut_ctx {
  int device = 0;
  uint64_t seed = 0;
  hipStream_t stream = nullptr;      // the caller-visible stream (ut_set_stream)
  hipStream_t own_stream = nullptr;
  // internal streams: a round's hash + dedup run on `side` beside the GP
  // contractions on `stream`; an asynchronous GP fit runs on `fit_stream`
  // beside the round's proposal / hash (joined by events, never by host waits)
  hipStream_t side = nullptr;
  hipStream_t fit_stream = nullptr;
  hipEvent_t ev_fork = nullptr, ev_join = nullptr, ev_fit = nullptr, ev_prefit = nullptr;
  hipEvent_t ev_fit_x = nullptr;     // fit stream: scaled training inputs ready (K* may start)
  bool fit_pending = false;          // scoring waits on ev_fit before touching GP state
  // fp64 variance with few candidate strips: 1 = split the k loops
  // (k_gp_var_pp<true> + k_var_split_red), 0 = one item per row tile; UT_VAR_SPLIT
  int32_t var_split = 1;
  double* fit_host = nullptr;        // pinned staging of X, y, 1/ell for the asynchronous fit
  size_t fit_host_n = 0;
  // a staged fit whose device work is not enqueued yet: gp_fit_enqueue stages
  // X, y and the host-side decisions, gp_fit_flush issues the launches.  A
  // proposal (and so every scoring round) is enqueued before the staged fit,
  // so the caller's stream is not idle while the host issues the fit's ~50
  // launches; anything that reads GP state flushes first.
  struct FitJob {
    bool on = false;
    int32_t n = 0, n0 = 0, d = 0, npad = 0, dpn = 0, xr0 = 0;
    bool app = false;
    double diag = 0.0, sf2 = 1.0;
  } fit_job;
  bool fit_prefit_set = false;   // ev_prefit already recorded for fit_job (gp_fit_prefit)
  int32_t fit_defer = 1;         // UT_FIT_DEFER=0: gp_fit_enqueue issues the launches itself
  std::string err;
  ut::Space space;
  bool has_space = false;

  // population of the selected slot (ut_population_select)
  double* pop = nullptr;
  int64_t npop = 0;
  int64_t pop_cap = 0;

  // PSO state of the selected slot
  double* pso_vel = nullptr;    // [P][npop]
  double* pso_best = nullptr;   // [P][npop]
  int64_t pso_cap = 0;

  // population slots: the techniques of one bandit share a context (its GP
  // fit, history set, scratch) and keep one population each; the fields
  // above are the selected slot's, the others are parked here
  // inner digests sha256(repr(get_value)) of the selected population's
  // computed-digest params ([n_comp][npop][8]): a DE trial keeps most of its
  // target's values, so its hash reuses the target's inner digests and
  // computes only the changed ones (hash.hip launch_hash_de)
  uint32_t* pop_dig = nullptr;
  int64_t pop_dig_cap = 0;
  bool pop_dig_valid = false;
  // the cache covers members [pop_dig_lo, pop_dig_lo + pop_dig_n) only: the
  // targets of this context's candidates (a rank's shard of the global pool,
  // cand_base .. cand_base + m), not the whole replicated population
  int64_t pop_dig_lo = 0, pop_dig_n = 0;
  // member-major donor copy of the selected population ([npop + 1][ld], ld =
  // ncols rounded up to 16 columns = whole 128-B lines), primitive params
  // stored as their unit values (unit_of), the others raw: k_de gathers its
  // donors' rows from it in line pieces staged in LDS, with no unit_of left to
  // compute; row npop holds the best config of the current DE launch.  Rebuilt
  // from pop when stale, patched by replace.
  double* pop_aos = nullptr;
  int64_t pop_aos_cap = 0;
  bool pop_aos_valid = false;
  int32_t de_aos = 1;   // 0: k_de gathers donor values from the column-major population (UT_DE_AOS=0)
  // the round being enqueued holds its hash for an in-flight fit (dense fp64
  // rounds: api.hip score_round_de_impl)
  bool round_hash_hold = false;
  // the grid-stride hash kernels' workgroups per CU: > 0 at most this many, 0
  // uncapped, -1 capped while a large refit is in flight (hash.hip hash_cap);
  // UT_HASH_WG_PER_CU
  int32_t hash_wg_per_cu = -1;
  // refit: the next diagonal block factored inside the trailing update
  // (k_chol_update_diag). -1 = from 2048 padded rows on: the fit alone 6.5 ->
  // 5.7 ms at n = 4096, C3 pruned 60.1 -> 59.2 ms; at C2 (n = 1024, the fit
  // beside K*) the heavier update workgroups cost the round 0.25 ms. UT_CHOL_FUSE
  int32_t chol_fuse = -1;
  // L^-1 levels of 256 rows and more on k_trinv_big (128 x 128 tiles, glds
  // ring) instead of k_trinv_level (64 x 64 tiles, plain loads); UT_TRINV_BIG
  int32_t trinv_big = 1;
  // the diagonal blocks' inverse solved inside the Cholesky column loop
  // (gp.hip chol_diag_core<true>); UT_CHOL_MERGED
  int32_t chol_merged = 1;

  struct PopSlot {
    double* pop = nullptr;
    int64_t npop = 0, pop_cap = 0;
    double* pso_vel = nullptr;
    double* pso_best = nullptr;
    int64_t pso_cap = 0;
    uint32_t* pop_dig = nullptr;
    int64_t pop_dig_cap = 0;
    bool pop_dig_valid = false;
    int64_t pop_dig_lo = 0, pop_dig_n = 0;
    double* pop_aos = nullptr;
    int64_t pop_aos_cap = 0;
    bool pop_aos_valid = false;
  };
  std::vector<PopSlot> pop_slots;
  int32_t pop_slot = 0;

  // history set
  uint32_t* hist_keys = nullptr;   // [cap][8]
  uint32_t* hist_state = nullptr;  // [cap] 0 empty / 1 full
  int64_t hist_cap = 0;
  int64_t hist_count = 0;

  // batch dedup table
  int32_t* batch_slots = nullptr;
  int64_t batch_cap = 0;

  // GP state
  int32_t gp_n = 0, gp_d = 0;
  bool gp_ready = false;
  double* gp_Xs = nullptr;     // [n][d] scaled features
  double* gp_xnorm = nullptr;  // [n]
  double* gp_K = nullptr;      // [n][n] work / L
  double* gp_Linv = nullptr;   // [n][n]
  double* gp_T = nullptr;      // [n][n] scratch of the recursive inverse
  double* gp_y = nullptr;      // [n] standardised
  double* gp_tmp = nullptr;    // [n]
  double* gp_alpha = nullptr;  // [n]  K^-1 y
  double* gp_beta = nullptr;   // [n]  L^-1 y (mean from the variance epilogue: mu = (L^-1 k*) . beta)
  double* gp_inv_ell = nullptr;// [d]
  double* gp_stats = nullptr;  // [4]: f_best, mean, std, flag
  int32_t* gp_flag = nullptr;
  double gp_sf2 = 1.0;
  int32_t gp_prec = 64;        // precision requested for the next fit
  int32_t gp_fit_prec = 64;    // precision of the fitted factors used by scoring
  // incremental fit (gp.hip gp_fit_enqueue): 1 = a fit whose training set
  // extends the previous one's extends its factor (ut_gp_set_fit_append)
  int32_t fit_append = 1;
  int32_t gp_npad_fit = 0;     // padded size of the current factor
  double gp_diag_fit = 0.0;    // its sigma_n2 + jitter
  int32_t gp_fit_kind = 0;     // 0 = the last fit refactored, 1 = it appended rows
  bool gp_linvt_stale = false; // gp_LinvT / gp_alpha not yet written for the current factor (gp_ensure_linvt)
  int32_t* flag_host = nullptr;  // pinned readback of the previous fit's flag
  float* gp_Xs_f = nullptr;    // fp32 copies for the fp32 MFMA path
  double* gp_LinvT = nullptr;  // (L^-1)^T [k][row]: the A operand of the variance contraction
  double* gp_XsT = nullptr;    // (X/ell)^T [dpad][npad]: the A operand of the K* contraction
  // categorical K* of the current fit (cat_on): numeric-feature operands and
  // the training rows' weighted one-hot codes; c0 + c1 * matches starts the
  // fp64 accumulator (= -|x_cat - u_cat|^2 / 2)
  bool cat_on = false;         // this fit scores with the categorical K*
  bool cat_x_ok = false;       // every training row so far has one-hot ENUM / 0-1 BOOL features
  int32_t cat_enable = 1;      // UT_CAT_KSTAR
  double cat_c0 = 0.0, cat_c1 = 0.0;
  ut::DevBuf<double> gp_XsT_num;    // [dpad_num][npad]
  ut::DevBuf<double> gp_xnorm_num;  // [npad] |x_num / ell|^2
  ut::DevBuf<int8_t> gp_acat;       // [cat_k / 128][npad][128] training codes (weights 2 ENUM, 1 BOOL)
  ut::DevBuf<int8_t> bcat;         // [cat_k / 128][ldk][128] candidate codes (one-hot 0/1)
  bool ucand_cat = false;          // ucand / cnorm / bcat hold the categorical K*'s operands (encode path)
  ut::DevBuf<int8_t> pr_bcat;      // pruned scoring: the gathered candidates' codes
  float* gp_LinvT_f = nullptr;  // fp32 (L^-1)^T; in h3 mode the fp16 hi/lo planes of L^-1 [row][k]
  // int8-sliced fp64 tier (precision 8, gp_i8.hip): L^-1 as I8_S digit planes,
  // per-row scales 2^(ea_i + eb) [npad] | e_i^2 [npad] | the bound E [1]
  ut::DevBuf<int8_t> gp_i8a;
  ut::DevBuf<double> gp_i8rs;
  // precision 8's K* on the int8 MFMA (gp_kq.hip, numeric fits): digit planes
  // of the training operand and its [amax, ea]; the round's candidate planes
  // and column scales
  ut::DevBuf<int8_t> gp_x8, u8;
  ut::DevBuf<int64_t> gp_q8;
  ut::DevBuf<double> scol;
  int32_t kstar_q = 1;   // UT_KSTAR_Q=0: precision-8 K* on k_gp_kstar<int8_t> (the fp64 MFMA)
  int32_t gp_i8_eb = 0;          // K* digit scale: y = k* 2^-eb <= 0.49
  double i8_tol = 0x1p-20;       // accepted relative variance error (ut_gp_set_i8_tol)
  int64_t i8_recomputed = 0;     // candidates of the last score recomputed in fp64 (-1: all, dense)
  int32_t* gp_ctr = nullptr;   // [32] per-XCD work tickets: [0,8) variance, [8,16) K*; [16,18) max|L^-1| bits (h3)
  int32_t n_cu = 256;
  // LDS one workgroup may hold (hipDeviceAttributeMaxSharedMemoryPerBlock): the
  // categorical K*'s code-row kernels need code_rows_lds(cat_k) of it
  size_t max_lds = 65536;
  int64_t gp_cap_n = 0;

  // scratch for GP scoring / round pipeline
  ut::DevBuf<double> kst;        // [n][ld]
  ut::DevBuf<double> mu_part;    // [RT][ld]
  ut::DevBuf<double> var_part;   // [RT][ld]
  ut::DevBuf<double> cnorm;      // [ld]
  ut::DevBuf<double> ucand;      // [dpad][ld] candidate features / ell (the K* B operand)
  ut::DevBuf<double> r_values, r_feat, r_mu, r_var, r_score;
  ut::DevBuf<uint32_t> r_digest;
  ut::DevBuf<uint8_t> r_dup;
  ut::DevBuf<uint8_t> r_inval;      // GA rounds: children whose retries all reproduced a parent
  ut::DevBuf<double> tk_score[2];
  ut::DevBuf<int64_t> tk_idx[2];
  ut::DevBuf<int64_t> r_topk_idx;
  ut::DevBuf<double> perm_ws;    // [2 * perm_cols + 3 * perm_smax][ld]: GA parents + crossover scratch
  ut::DevBuf<uint32_t> perm_dig; // [n_perm][m][8] inner digests of PERM values (hash pre-pass)
  ut::DevBuf<double> r_topk_score;
  ut::DevBuf<double> r_topk_vals;   // gathered top-k rows when the caller wants digests only
  ut::DevBuf<uint32_t> r_mask;      // [ceil(n_comp / 32)][ld]: bit s = trial's cslot-s value differs from its target's
  ut::DevBuf<uint32_t> r_fresh;     // [n_comp][ld][8]: inner digests of the changed values
  ut::DevBuf<uint64_t> r_pairs;     // compacted (candidate << 20 | cslot) of the changed values
  ut::DevBuf<int64_t> r_npairs;     // [1] their count
  ut::DevBuf<uint32_t> de_xbits;    // k_de's cr-test bits when they outgrow LDS (> 2048 params)
  ut::DevBuf<uint32_t> par_dig;     // [n_comp][16]: hex inner digests of ut_hash_parent's parent row
  ut::DevBuf<uint32_t> hs_mask;     // small-m ut_hash: all-ones reuse mask [ceil(n_comp / 32)][ld]
  ut::DevBuf<uint32_t> hs_fresh;    // small-m ut_hash: every inner digest, hex [n_comp][ld][16]
  // EI-bound pruned scoring (gp.hip ut_gp_topk_pruned)
  ut::DevBuf<double> pr_mu, pr_ub, pr_score;   // [ld] exact mean, score bound, exact scores (-inf if pruned)
  ut::DevBuf<double> pr_mpart;                 // [RT][ldk] unused mean partials of the bound / survivor GEMMs
  ut::DevBuf<double> pr_kst, pr_vpart;         // survivors' K* columns [npad][lds] and variance partials
  ut::DevBuf<double> pr_ucand, pr_cnorm;       // survivors' scaled features [dpad][lds] and norms [lds]
  ut::DevBuf<int64_t> pr_idx;                  // [ld] survivor indices (+ the threshold set)
  ut::DevBuf<int64_t> pr_count;                // [1]
  ut::DevBuf<double> var_vbuf;                 // split variance: raw partial tiles [items][128][128]
  ut::DevBuf<double> app_ws;                   // split-K partials of the incremental fit [b][maxq][64][64]
  ut::DevBuf<double> pr_k2;                    // [RT][ldk] partials of |k*|^2 (the variance tail bound)
  ut::DevBuf<double> pr_f2;                    // [1] |L^-1|_F^2 (+ its block partials), then the f32
                                               // pass's sum |alpha|
  bool pr_f2_valid = false;                    // pr_f2 belongs to the current fit
  bool pr_ab_valid = false;                    // ... and its sum |alpha|
  bool pr_xf_valid = false;                    // pr_xsT_f and max |x|^2 belong to the current fit,
  bool pr_xf_cat = false;                      // ... built from this operand (numeric block or all features)
  int32_t pr_xf_dpad = -1;                     // ... with this many rows
  ut::DevBuf<float> pr_xsT_f, pr_ucand_f;      // f32 K* operands of the f32-contraction bound pass
  ut::DevBuf<double> pr_sa;                    // [RT][ldk] partials of sum |alpha_r| k*_r (f32 bound pass)
  ut::DevBuf<double> pr_gmu;                   // [RT][ldc] fp64 mean partials of recomputed columns (f32 pass)
  int32_t prune_pass = 32;                     // ut_gp_set_prune_pass: the bound pass in f32 or fp64
  ut::DevBuf<uint8_t> pr_exact;                // [ld] the stored score is the exact score
  int64_t r_ld = 0;
  int64_t r_m = 0;
  bool r_feat_valid = false;        // r_feat holds the last round's features (pruned rounds only)

  // tree-ensemble surrogate (forest.hip)
  ut_tree_node* forest_nodes = nullptr;
  int32_t* forest_roots = nullptr;
  int32_t forest_trees = 0, forest_rule = 0;
  double forest_base = 0.0, forest_scale = 1.0, forest_div = 1.0;

  // multi-GPU exchange (comm.hip): the RCCL communicator of this context's
  // rank and the packed top-k records of the all-gather / merge
  void* comm = nullptr;               // ncclComm_t
  int32_t comm_rank = 0, comm_size = 1;
  ut::DevBuf<uint64_t> cm_send, cm_recv;   // [k][W] / [R k][W] records (W = 6 + payload columns)
  ut::DevBuf<uint8_t> cm_keep;             // [R k] record survives the digest dedup
  ut::DevBuf<double> cm_pay;               // [n][5] broadcast payload (value + digest)
  ut::DevBuf<int64_t> cm_cnt;              // [2] broadcast count + agreement flag (allocated by ut_comm_init)
  // record capacity (uint64 words of cm_send / cm_recv) every rank agreed it
  // holds: the all-gather votes only when a call needs more (comm.hip)
  size_t cm_agreed_send = 0, cm_agreed_recv = 0;
  int32_t dbg_fail_alloc = 0;              // ut_debug_fail_alloc: the next N growing ensure() calls fail

  ut::Timing timing;
};

namespace ut {

int set_err(ut_ctx* c, int code, const std::string& msg);

// every device allocation of the library goes through these two (api.hip):
// the bytes held per device are what ut_device_bytes reports (a rank's HBM
// footprint in the bench line)
hipError_t dmalloc(void** p, size_t bytes);
void dfree(void* p);

// wait for every stream of the context (before freeing or reusing buffers)
inline hipError_t sync_all(ut_ctx* c) {
  hipError_t e = hipStreamSynchronize(c->stream);
  for (hipStream_t s : {c->side, c->fit_stream}) {
    if (!s) continue;
    const hipError_t e2 = hipStreamSynchronize(s);
    if (e == hipSuccess) e = e2;
  }
  return e;
}

// launches inside the scope go to stream s (the launch helpers all use c->stream)
struct StreamScope {
  ut_ctx* c;
  hipStream_t saved;
  StreamScope(ut_ctx* ctx, hipStream_t s) : c(ctx), saved(ctx->stream) { ctx->stream = s; }
  ~StreamScope() { c->stream = saved; }
};

#define UT_HIP(ctx, call)                                                                 \
  do {                                                                                    \
    hipError_t e_ = (call);                                                               \
    if (e_ != hipSuccess)                                                                 \
      return ::ut::set_err((ctx), UT_EHIP, std::string(#call) + ": " + hipGetErrorString(e_)); \
  } while (0)

#define UT_CHECK(ctx, cond, code, msg)                    \
  do {                                                    \
    if (!(cond)) return ::ut::set_err((ctx), (code), (msg)); \
  } while (0)

#define UT_LAUNCH_CHECK(ctx)                                                       \
  do {                                                                             \
    hipError_t e_ = hipGetLastError();                                             \
    if (e_ != hipSuccess)                                                          \
      return ::ut::set_err((ctx), UT_EHIP, std::string("launch: ") + hipGetErrorString(e_)); \
  } while (0)

// feature rows of the K* operands (Xs^T, U'): d rounded up to the f64 MFMA's k = 4
inline int32_t kstar_dpad(int32_t d) { return ((d + 3) / 4) * 4; }

template <class T>
int ensure(ut_ctx* c, DevBuf<T>& b, size_t n) {
  if (b.n >= n && b.p) return 0;
  if (c->dbg_fail_alloc > 0) {   // fault injection (tests): this growth fails as hipMalloc would
    --c->dbg_fail_alloc;
    return set_err(c, UT_ENOMEM, "hipMalloc: injected failure (ut_debug_fail_alloc)");
  }
  // a buffer that has to grow again (sizes that follow a growing training
  // set) gets headroom, up to 2 GiB: every regrowth costs a device-wide sync
  size_t want = n;
  if (b.p) {
    want = n + std::min(n / 4, ((size_t)2 << 30) / sizeof(T));
    hipError_t e = ut::sync_all(c);
    (void)e;
    (void)ut::dfree(b.p);
    b.p = nullptr;
    b.n = 0;
  }
  hipError_t e = ut::dmalloc((void**)&b.p, (want ? want : 1) * sizeof(T));
  if (e != hipSuccess && want > n) {   // no room for the headroom: exactly n
    (void)hipGetLastError();
    want = n;
    e = ut::dmalloc((void**)&b.p, (want ? want : 1) * sizeof(T));
  }
  if (e != hipSuccess) return set_err(c, UT_ENOMEM, std::string("hipMalloc: ") + hipGetErrorString(e));
  b.n = want;
  return 0;
}

void mark(ut_ctx* c, const char* name);
int gp_fit_enqueue(ut_ctx* c, const double* X, const double* y, int32_t n, int32_t d, const ut_gp_hyper* h);
int gp_wait_fit(ut_ctx* c);
int gp_fit_flush(ut_ctx* c);
int gp_ensure_linvt(ut_ctx* c);
int gp_fit_prefit(ut_ctx* c);

// kernel launchers implemented in the .hip translation units
int launch_population_init(ut_ctx* c, uint32_t round_);
// diff = true (DE scoring rounds): k_de also writes the DE-diff mask, pairs and
// pair count (r_mask / r_pairs / r_npairs) that launch_hash_de would derive
int launch_de(ut_ctx* c, const ut_de_params* p, uint32_t round_, int64_t cand_base, int64_t m, double* out,
              int64_t ld, bool diff = false);
int launch_pso(ut_ctx* c, const ut_pso_params* a, const double* gbest, uint32_t round_, int64_t cand_base,
               int64_t m, double* out_x, double* out_v, int64_t ld);
int launch_ga(ut_ctx* c, const ut_ga_params* a, const double* parent1, const double* parent2, uint32_t round_,
              int64_t cand_base, int64_t m, double* out, int64_t ld, uint8_t* invalid);
int launch_encode(ut_ctx* c, const double* values, int64_t ld, int64_t m, double* feat, int64_t ldf);
int launch_hash(ut_ctx* c, const double* values, int64_t ld, int64_t m, uint32_t* out);
// hash_config of DE trials of the selected population (candidate g targets
// member g % npop): inner digests of values equal to the target's come from
// the population cache (rebuilt if stale), the rest are computed once
// have_diff: the mask / pairs / count were written by k_de (launch_de diff = true)
int launch_hash_de(ut_ctx* c, const double* values, int64_t ld, int64_t m, int64_t cand_base, uint32_t* out,
                   bool have_diff = false);
// hash_config of children of one parent row (ut_hash_parent): inner digests of
// the values equal to the parent's are the parent's own
int launch_hash_parent(ut_ctx* c, const double* values, int64_t ld, int64_t m, const double* parent, uint32_t* out);
// the DE-diff buffers for m candidates (ld): r_mask, r_fresh, r_pairs, r_npairs
int ensure_de_diff(ut_ctx* c, int64_t ld);
// population cache maintenance: the rows idx[0..n) after a replace (rows
// outside the cached window are skipped)
int launch_pop_digests(ut_ctx* c, const int64_t* idx, int64_t n);
// full rebuild of the cache for the members [lo, lo + wn)
int launch_pop_digests_window(ut_ctx* c, int64_t lo, int64_t wn);
// the member-major population copy: rebuilt if stale (ensure), or the rows
// idx[0..n) patched from trial after a replace
int ensure_pop_aos(ut_ctx* c);
int launch_pop_aos_rows(ut_ctx* c, const double* trial, int64_t ld, const int64_t* idx, int64_t n);
// row `row` of the donor copy = the config `src` (device, ncols values)
int launch_aos_row(ut_ctx* c, const double* src, int64_t row);
inline int64_t pop_aos_ld(const ut_ctx* c) { return ((int64_t)c->space.ncols + 15) / 16 * 16; }
int launch_hist_insert(ut_ctx* c, const uint32_t* dig, int64_t n);
int launch_hist_rehash(ut_ctx* c, const uint32_t* okeys, const uint32_t* ostate, int64_t ocap);
int launch_dedup(ut_ctx* c, const uint32_t* dig, int64_t m, uint8_t* dup);
int launch_mask_or(ut_ctx* c, uint8_t* dst, const uint8_t* src, int64_t m);
// feat == nullptr: the candidates' scaled features and norms are already in
// c->ucand / c->cnorm (gp_encode_scaled); dup_ready: the event of the dup
// mask (the round's side stream), joined before the variance GEMM
int gp_score_impl(ut_ctx* c, const double* feat, int64_t ld, int64_t m, const ut_acq* acq, const uint8_t* dup,
                  double* mu, double* var, double* score, hipEvent_t dup_ready = nullptr);
// encode + scale in one pass into c->ucand / c->cnorm (sized for m), for gp_score_impl(feat = nullptr)
int gp_encode_scaled(ut_ctx* c, const double* values, int64_t ld, int64_t m);
int launch_encode_scaled(ut_ctx* c, const double* values, int64_t ld, int64_t m, double* u, int32_t dpad, int64_t ldu,
                         double* cn);
int topk_impl(ut_ctx* c, const double* score, const uint8_t* dup, int64_t m, int64_t cand_base, int32_t k,
              int64_t* out_idx, double* out_score);
int topk_pairs_impl(ut_ctx* c, const double* score, const int64_t* idx, int64_t n, int32_t k, int64_t* out_idx,
                    double* out_score);
// feat_ours: the features come from ut's own encoder (one-hot ENUM blocks),
// so the categorical K* may read them as codes
int gp_topk_pruned_impl(ut_ctx* c, const double* feat, int64_t ld, int64_t m, const ut_acq* acq, const uint8_t* dup,
                        int64_t cand_base, int32_t k, int32_t bound_rows, int64_t* out_idx, double* out_score,
                        ut_prune_stats* stats, hipEvent_t dup_ready = nullptr, bool feat_ours = false);
// prec: 64 (fp64 MFMA), 32 (fp32 MFMA), 16 (f16x3: fp16 hi/lo split operands,
// three fp16 MFMA products, f32 accumulate -- see gp_gemm.hip), 8 (the fp64
// tier on the int8 MFMA: six-digit planes, a per-candidate error bound and an
// fp64 recompute of the candidates it does not clear -- gp_i8.hip)
constexpr int H3_KSCALE_EXP = 14;  // K* (<= sf2) is scaled by 2^(14 - ceil(log2 sf2)) before the split
int h3_kstar_exp(double sf2);
// K*'s training operand (Xs^T, the numeric part in categorical mode) is stored
// times 256 / ln 2: the contraction then yields the exponent in 2^(1/256) units
// (sf2_exp2t_nonpos below)
constexpr double KSTAR_T_SCALE = 369.3299304675746;   // 256 / ln 2
// sf2 * exp(x) for x <= 0, table-driven: etab[j] = sf2 * 2^(j/256) built in LDS by
// each workgroup (2 KiB); about 12 VALU ops against ~32 for the library exp with
// its range checks (the epilogue shares the SIMDs with the f64 MFMAs, so every
// op counts; a 32-entry table with a degree-6 polynomial took two more FMAs).
// Max error ~2 ulp; 2^k' underflows to exactly 0 at x = -1000.
constexpr int EXP_TAB = 256;

// The K* contraction works in units of 2^(1/256): its training operand is
// Xs^T * (256 / ln 2) (KSTAR_T_SCALE, applied where Xs^T is built, k_gp_xs_t /
// k_gp_num_train), the epilogue's norms and categorical coefficients carry the
// same factor, so the accumulator is t = -|x - u|^2 / 2 * 256 / ln 2 directly
// and the exp needs no multiply and no two-step reduction: t = 256 k' + j + f
// with kf = rint(t), f = t - kf exact (|f| <= 1/2), and
// exp = 2^k' * 2^(j/256) * e^(f ln2/256) with the same degree-4 polynomial
// (|f ln2/256| <= 1.36e-3: truncation < 4e-17).  Two DP ops fewer per k*
// than sf2_exp_nonpos, whose rounding it shares to ~1 ulp.
__device__ __forceinline__ double sf2_exp2t_nonpos(double t, const double* etab) {
  constexpr double L = 0.6931471805599453 / 256.0;    // ln 2 / 256 (exact: a power-of-two division)
  constexpr double C2 = L * L / 2.0, C3 = L * L * L / 6.0, C4 = L * L * L * L / 24.0;
  const double kf = __builtin_rint(t);
  const double f = t - kf;
  double p = __builtin_fma(C4, f, C3);
  p = __builtin_fma(p, f, C2);
  p = __builtin_fma(p, f, L);
  p = __builtin_fma(p, f, 1.0);
  const int k = (int)kf;
  return __builtin_ldexp(p * etab[k & (EXP_TAB - 1)], k >> 8);
}
constexpr double KSTAR_T_MIN = -1000.0 * KSTAR_T_SCALE;   // exp(-1000): the table's 2^k' underflows to 0
// the K* contraction's categorical operands (nkc = cat_k / 128 int8 stages; 0 = none)
struct KstarCat {
  const int8_t* acat = nullptr;
  const int8_t* bcat = nullptr;
  int32_t nkc = 0;
  double c0 = 0.0, c1 = 0.0;
};
int launch_gemm_kstar(ut_ctx* c, int prec, const double* XsT, int32_t npad, const double* ucand, int32_t dpad,
                      int64_t m, void* kst, int64_t ldk, double* part, int32_t store_rows = -1,
                      const double* cn = nullptr,    // candidate norms (nullptr: c->cnorm)
                      double* part2 = nullptr,       // fp64 with part: also sum_r k*_r^2 partials
                      const KstarCat& cat = KstarCat(),
                      const double* xn = nullptr,    // training norms (nullptr: c->gp_xnorm)
                      int32_t row_tiles = -1);       // > 0: only the first row_tiles 128-row tiles
// gp_kq.hip: K* of a numeric precision-8 fit as the distance contraction on
// the int8 MFMA (digit planes of the training operand from the fit, of the
// candidates' operand per call into u8 / scol), stored as the six digit planes
// the int8 variance reads (planes = true; no mean partial, no one-hot codes).
int alloc_split_x8(ut_ctx* c, int32_t npad, int32_t K);
int launch_split_x8(ut_ctx* c, const double* XsT, int32_t K, int32_t npad);
int launch_gemm_kstar_q(ut_ctx* c, bool planes, const double* XsT, int32_t npad, const double* ucand, int32_t dpad,
                        int64_t m, void* kst, int64_t ldk, double* part, int32_t store_rows, const double* cn,
                        double* part2, const KstarCat& cat, const double* xn, DevBuf<int8_t>& u8,
                        DevBuf<double>& scol);
int launch_gemm_kstar_f32c(ut_ctx* c, const float* XsT_f, int32_t npad, const float* ucand_f, int32_t dpad,
                           int64_t m, int64_t ldk, int32_t rt0, double* part, double* part2, double* part3,
                           const KstarCat& cat, const double* xn, const double* cn);
int launch_prep_cand(ut_ctx* c, const double* feat, int64_t ld, int64_t m, int32_t d, int32_t dpad, double* u,
                     int64_t ldu, double* cn);
// categorical K*: the K* operands of the candidate side when the fit is in
// categorical mode -- numeric features / ell (dpad_num rows), their norms, and
// one-hot codes into c->bcat (from values, or from features made by ut's own
// encoder)
inline int32_t cat_dpad(const ut_ctx* c) { return kstar_dpad(c->space.n_num); }
// the candidates' 128-byte code rows of one 256-candidate workgroup, written
// coalesced: each thread sets its codes as bits in LDS (bits [256][stride],
// stride = cat_k / 32 + 1 dwords), then every 128-column block is expanded to
// bytes through an LDS image and stored as whole rows (propose.hip)
__device__ inline void store_code_rows(const uint32_t* bits, int32_t stride, int32_t nkb, uint32_t* img, int8_t* bcat,
                                int64_t ldu, int64_t i0) {
  const int t = threadIdx.x;
  for (int32_t kb = 0; kb < nkb; ++kb) {
    // this thread's 128 codes of block kb: bits 4w .. 4w + 3 -> the 4 bytes of dword w
#pragma unroll
    for (int w = 0; w < 32; ++w) {
      const uint32_t b = (bits[t * stride + kb * 4 + (w >> 3)] >> ((w & 7) * 4)) & 15u;
      img[t * 33 + w] = (b & 1u) | ((b & 2u) << 7) | ((b & 4u) << 14) | ((b & 8u) << 21);
    }
    __syncthreads();
    // the block's 256 rows of 128 bytes are contiguous in bcat: 16-byte stores in order
    uint4* dst = reinterpret_cast<uint4*>(bcat + ((int64_t)kb * ldu + i0) * 128);
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int e = q * 256 + t, r = e >> 3, c = e & 7;
      const uint32_t* src = img + r * 33 + 4 * c;
      dst[e] = make_uint4(src[0], src[1], src[2], src[3]);
    }
    __syncthreads();
  }
}

inline size_t code_rows_lds(int32_t cat_k) { return sizeof(uint32_t) * 256 * ((cat_k / 32 + 1) + 33); }
int launch_encode_scaled_cat(ut_ctx* c, const double* values, int64_t ld, int64_t m, double* u, int32_t dpad,
                             int64_t ldu, double* cn, int8_t* bcat);
int launch_prep_cand_cat(ut_ctx* c, const double* feat, int64_t ld, int64_t m, double* u, int32_t dpad, int64_t ldu,
                         double* cn, int8_t* bcat);
int launch_xs_t(ut_ctx* c, const double* Xs, int32_t npad, int32_t d, int32_t dpad, double* XsT);
int launch_gemm_var(ut_ctx* c, int prec, const void* LinvT, int64_t lda, const void* kst, int64_t ldk, int32_t npad,
                    int64_t m, double* part, const double* beta, double* mpart);
int launch_transpose(ut_ctx* c, const double* src, int32_t n, double* dst, float* dst_f);
// ---- int8-sliced fp64 tier (gp_i8.hip) ----
// six balanced 8-bit digits per operand value; tiles of the variance contraction
constexpr int I8_S = 6, I8_BM = 64, I8_BN = 64, I8_BK = 32;
constexpr int32_t I8_MAX_K = 16384;   // exact int32 group sums: K * 6 * 2^14 < 2^31
// the digit scale of K*: the smallest eb with sf2 2^-eb <= 0.49 (k* <= sf2)
inline int i8_kstar_exp(double sf2) { return ilogb(sf2 / 0.49) + 1; }
// byte offset of element (r, k) in a digit plane [K / 32][ld][32]: a 32-k piece
// of row r is 32 contiguous bytes, its 16-byte chunks swizzled by bit 3 of r
__host__ __device__ inline int64_t i8_off(int64_t r, int32_t k, int64_t ld) {
  return ((int64_t)(k >> 5) * ld + r) * 32 + ((((k >> 4) & 1) ^ (int)((r >> 3) & 1)) << 4) + (k & 15);
}
// x in [-0.49, 0.49] -> bits 0..47 = rint(x 2^48) + 0x808080808080: the fp64
// sum x + 24.5019... (24 + 0x808080808080 2^-48, exact) lies in [16, 32), so
// its ulp is 2^-48, its exponent field fixed, and its mantissa's low 48 bits
// that integer (rounded to nearest even: the offset is even); its six bytes,
// each XOR 0x80, are the balanced digits (int8) of rint(x 2^48) in base 256,
// most significant = byte 5 (bits 48.. are the exponent: ignored)
__device__ __forceinline__ uint64_t i8_biased(double x) {
  return (uint64_t)__double_as_longlong(x + 0x1.8808080808080p4);
}
// four values' biased words (lo / hi dwords) -> the six digit planes' dwords
// (byte u of plane p's dword = digit p of value u; plane 0 = most significant):
// a 4 x 4 byte transpose by v_perm_b32 (byte j of perm(a, b, s) is byte
// s_j of the pair, 0..3 = b, 4..7 = a)
typedef int32_t i8v4 __attribute__((ext_vector_type(4)));
typedef int32_t i8v16 __attribute__((ext_vector_type(16)));
__device__ __forceinline__ void i8_planes(const uint32_t (&lo)[4], const uint32_t (&hi)[4], uint32_t (&pl)[I8_S]) {
  const uint32_t t0 = __builtin_amdgcn_perm(lo[1], lo[0], 0x05010400u);   // w0.b0 w1.b0 w0.b1 w1.b1
  const uint32_t t1 = __builtin_amdgcn_perm(lo[1], lo[0], 0x07030602u);   // w0.b2 w1.b2 w0.b3 w1.b3
  const uint32_t t2 = __builtin_amdgcn_perm(lo[3], lo[2], 0x05010400u);
  const uint32_t t3 = __builtin_amdgcn_perm(lo[3], lo[2], 0x07030602u);
  const uint32_t u0 = __builtin_amdgcn_perm(hi[1], hi[0], 0x05010400u);
  const uint32_t u2 = __builtin_amdgcn_perm(hi[3], hi[2], 0x05010400u);
  pl[0] = __builtin_amdgcn_perm(u2, u0, 0x07060302u) ^ 0x80808080u;      // byte 5
  pl[1] = __builtin_amdgcn_perm(u2, u0, 0x05040100u) ^ 0x80808080u;      // byte 4
  pl[2] = __builtin_amdgcn_perm(t3, t1, 0x07060302u) ^ 0x80808080u;      // byte 3
  pl[3] = __builtin_amdgcn_perm(t3, t1, 0x05040100u) ^ 0x80808080u;      // byte 2
  pl[4] = __builtin_amdgcn_perm(t2, t0, 0x07060302u) ^ 0x80808080u;      // byte 1
  pl[5] = __builtin_amdgcn_perm(t2, t0, 0x05040100u) ^ 0x80808080u;      // byte 0
}
// fit: L^-1's planes, row scales and the error bound (c->gp_i8a, c->gp_i8rs,
// allocated beforehand by alloc_split_i8; the digit scale of K* in c->gp_i8_eb)
int alloc_split_i8(ut_ctx* c, int32_t npad);
int launch_split_i8(ut_ctx* c, int32_t n, int32_t npad);
// the variance contraction from K*'s digit planes (kst8, [6][npad/32][ldk][32]):
// part [npad / 64][ldk] column partials of |v|^2
// part / mpart: per 64-row tile the column sums of v^2 and of v beta (the mean)
int launch_gemm_var_i8(ut_ctx* c, int32_t npad, const int8_t* kst8, int64_t ldk, int64_t m, double* part,
                       double* mpart);
// L^-1 [row][k] (n x n, fp64) -> scaled fp16 hi/lo planes, blocked (h3 A operand, rows padded to 256);
// the scale exponent is derived on the device from max|L^-1| (kept in gp_ctr[16..17])
int launch_split_h3(ut_ctx* c, const double* Linv, int32_t n, _Float16* dst);
constexpr int VAR_BM = 128, VAR_BN = 256;  // variance-contraction tile (rows of L^-1 x candidates)
int launch_to_f32(ut_ctx* c, const double* src, float* dst, int64_t n);
// gp.hip: the fit kernels' issue priority (UT_FIT_SETPRIO; process-wide)
int set_fit_prio(int32_t on);
int set_fit_prio_gemm(int32_t on);   // gp_gemm.hip's fit kernels
int launch_gather_rows(ut_ctx* c, const double* values, int64_t ld, const int64_t* idx, int64_t cand_base,
                       int32_t k, double* out, int64_t ldo, const uint32_t* dig, uint32_t* out_dig);
// comm.hip: release the context's communicator (ut_ctx_destroy)
void comm_release(ut_ctx* c);

inline unsigned grid1(int64_t n, int bs) { return (unsigned)((n + bs - 1) / bs); }

}  // namespace ut
