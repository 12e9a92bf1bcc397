/*
 * uthot.h -- C ABI of libuthot.so, the gfx950 (MI355X) batch candidate
 * proposal + scoring library behind uptune_amd.
 *
 * Drop-in boundary.  The reference runs this path one configuration at a
 * time inside the Python search loop:
 *   SearchTechnique.desired_configuration()   opentuner/search/technique.py:113-121
 *   DifferentialEvolution.create_new_configuration
 *                                             opentuner/search/differentialevolution.py:105-129
 *   HybridParticle.move / op3_swarm           opentuner/search/pso.py:70-77
 *   EvolutionaryTechnique.mutation            opentuner/search/evolutionarytechniques.py:51-61
 *   ConfigurationManipulator.hash_config      opentuner/search/manipulator.py:233-243
 *   SearchDriver.get_configuration/has_results opentuner/search/driver.py:157-158,253-258
 *   ParallelTuning.unique / hash_cfg          python/uptune/api.py:254-288
 * Each entry point below replaces one of those per-candidate Python calls
 * with one batched, stream-ordered call over m candidates.
 *
 * Conventions
 *   - every function returns 0 on success or a negative UT_E* code; the
 *     message is available from ut_last_error(ctx);
 *   - pointer arguments are DEVICE pointers unless the name ends in _host;
 *   - work is enqueued on the context's HIP stream (ut_set_stream); results
 *     are valid once that stream is synchronised;
 *   - SoA value arrays are column-per-parameter: value of param p for
 *     candidate i lives at values[col(p) * ld + i] (f64 for every kind: FLOAT
 *     raw value, INT/LOGINT raw integer, POW2 raw power of two, BOOL 0/1,
 *     ENUM option index); a PERM of size S takes S consecutive columns
 *     holding its item indices in order.  col(p) = p + the sum of (size - 1)
 *     over the PERM params before p (ut_space_columns);
 *   - digests are 8 big-endian uint32 words (= sha256().digest()) per
 *     candidate, candidate-major ([m][8]);
 *   - candidate indices are GLOBAL (cand_base + i), so random streams and
 *     tie-breaks do not depend on how a pool is sharded over GPUs.
 *   - one context per host thread.
 */
#ifndef UTHOT_H
#define UTHOT_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct ut_ctx ut_ctx;

enum {
  UT_OK = 0,
  UT_EINVAL = -1,      /* bad argument */
  UT_EHIP = -2,        /* HIP runtime error */
  UT_ENOSPACE = -3,    /* ut_space_define not called */
  UT_EUNSUPPORTED = -4,
  UT_ENOTPD = -5,      /* GP kernel matrix not positive definite */
  UT_ENOMEM = -6,
  UT_ECOMM = -7        /* RCCL error (multi-GPU exchange) */
};

/* parameter kinds: manipulator.py:651-1356 (the kinds create_params builds,
 * python/uptune/api.py:179-199) */
enum {
  UT_FLOAT = 0,  /* FloatParameter        manipulator.py:703-744 */
  UT_INT = 1,    /* IntegerParameter      manipulator.py:651-700 */
  UT_LOGINT = 2, /* LogIntegerParameter   manipulator.py:778-797 (stored int, searched log2) */
  UT_POW2 = 3,   /* PowerOfTwoParameter   manipulator.py:811-836 (stored 2^e, searched e) */
  UT_BOOL = 4,   /* BooleanParameter      manipulator.py:930-996 */
  UT_ENUM = 5,   /* EnumParameter         manipulator.py:1024-1045 */
  UT_PERM = 6    /* PermutationParameter  manipulator.py:1048-1356 (n_options = size) */
};

typedef struct ut_param_desc {
  int32_t kind;        /* UT_* kind */
  int32_t sort_rank;   /* position in sorted(params, key=name)  (manipulator.py:237) */
  double lo, hi;       /* min_value, max_value of the STORED value (POW2: powers of two) */
  double u_lo, u_hi;   /* unit-encoding bounds of the SEARCHED value (get_value) as Python
                          computes them: ints widened by 0.4999 (manipulator.py:476-479);
                          LOGINT: its scaled legal_range (:792-795); POW2: exponents -+0.4999 */
  double u_span;       /* float(u_hi - u_lo) as Python computes it */
  int64_t n_options;   /* ENUM option count (BOOL: 2) */
  const char* name;    /* str(p.name) bytes, not NUL-terminated */
  int32_t name_len;
  int32_t lut_count;   /* >0: inner digests of repr(get_value) supplied in lut */
  const uint8_t* lut_host; /* lut_count * 32 bytes: sha256(repr(get_value)).digest(),
                              indexed by (value - lo) for INT and LOGINT, by
                              (exponent - log2 lo) for POW2, by option index for
                              ENUM, 0=False/1=True for BOOL */
  int32_t vtab_count;  /* LOGINT: >0 = get_value(v) = math.log(v + 1.0 - min, 2.0) for
                          v = lo .. lo+vtab_count-1, computed by the host's CPython;
                          0 = computed on the device (ut_core.h libm_log: glibc's
                          log restated bit for bit, so the same values) */
  int32_t pad;
  const double* vtab_host;
  /* PERM: repr(item) bytes of the n_options items, concatenated, and their
   * n_options + 1 offsets; the inner digest is sha256(repr(list of items)),
   * "[" + ", ".join(repr(item)) + "]" (ComplexParameter.hash_value :855-858) */
  const uint8_t* perm_repr_host;
  const int32_t* perm_repr_off_host;
} ut_param_desc;

/* permutation crossover operators (op3_cross_*, manipulator.py:1179-1353) */
enum { UT_X_NONE = 0, UT_X_OX1 = 1, UT_X_OX3 = 2, UT_X_PX = 3, UT_X_CX = 4, UT_X_PMX = 5 };

typedef struct ut_de_params {   /* differentialevolution.py:34-40,142-151 */
  double cr;                    /* crossover rate (0.9 DE, 0.2 DE-Alt) */
  int32_t n_cross;              /* forced crossovers (1), <= 4 */
  int32_t information_sharing;  /* copies of the driver's best config added to the donor pool (1);
                                   used only when best != NULL (differentialevolution.py:112-116) */
  const double* best;           /* device row [ncols]: driver.best_result's values, NULL = no result yet */
} ut_de_params;

typedef struct ut_gp_hyper {
  double sigma_f2;    /* signal variance */
  double sigma_n2;    /* noise variance added to the diagonal */
  double jitter;      /* extra diagonal jitter */
  const double* lengthscale_host; /* d entries (ARD) */
} ut_gp_hyper;

enum { UT_ACQ_EI = 0, UT_ACQ_UCB = 1 };

typedef struct ut_acq {
  int32_t kind;       /* UT_ACQ_EI or UT_ACQ_UCB */
  int32_t pad;
  double xi;          /* EI exploration offset */
  double kappa;       /* UCB: score = kappa*sigma - mu */
} ut_acq;

/* ---- context ------------------------------------------------------------ */
int ut_ctx_create(int device, uint64_t seed, ut_ctx** out);
int ut_ctx_destroy(ut_ctx* ctx);
const char* ut_last_error(ut_ctx* ctx);
/* hipStream_t to enqueue on; NULL = the device's default (null) stream.  A new
 * context starts on its own non-blocking stream. */
int ut_set_stream(ut_ctx* ctx, void* hip_stream);
int ut_sync(ut_ctx* ctx);
int ut_version(void);
/* device memory (bytes) the library currently holds on `device` in this
 * process, over all its contexts (RCCL's own buffers not included): one rank
 * per process and GPU makes this the rank's HBM footprint */
int ut_device_bytes(int32_t device, int64_t* bytes_host);

/* ---- search space (ConfigurationManipulator, manipulator.py:129-272) ---- */
/* py2_layout: 1 = OpenTuner/Python-2 hash layout (no b'' around primitive
 * inner digests; pins samples/tutorials/tuneup.opentuner.db), 0 = uptune's
 * Python-3 port (manipulator.py:240 str() of a bytes object). */
int ut_space_define(ut_ctx* ctx, int32_t n_params, const ut_param_desc* params, int32_t py2_layout);
/* outer hash message length in bytes, SHA-256 block count, GP feature width */
int ut_space_info(ut_ctx* ctx, int64_t* outer_len, int64_t* outer_blocks, int32_t* n_features);
/* number of SoA value columns (= n_params unless the space has PERMs) */
int ut_space_columns(ut_ctx* ctx, int32_t* n_columns);

/* ---- population (DifferentialEvolution.population, PSO particles) ------- */
/* op1_randomize every member on the device (manipulator.py:171-176,596-606) */
int ut_population_init(ut_ctx* ctx, int64_t npop, uint32_t round_);
int ut_population_set(ut_ctx* ctx, int64_t npop, const double* values, int64_t ld);
int ut_population_get(ut_ctx* ctx, double* values, int64_t ld);
/* population slots: every population / PSO call acts on the selected slot
 * (initially 0).  The techniques of one bandit share one context -- one GP
 * fit, one history set -- with a population each (bandittechniques.py:311-320
 * composes DE, PSO and GA over one surrogate).  slot in [0, 1024). */
int ut_population_select(ut_ctx* ctx, int32_t slot);
/* copy trial rows back into the population: pop[:, idx[j]] = trial[:, j] */
int ut_population_replace(ut_ctx* ctx, const double* trial, int64_t ld, const int64_t* idx, int64_t n);

/* ---- proposal ----------------------------------------------------------- */
/* DE/rand/1/bin: one trial per candidate; candidate g targets population
 * member g % npop (differentialevolution.py:105-129).  Donors x1, x2, x3 are
 * the first three of a shuffle of population - {target} plus
 * information_sharing copies of `best` (:109-118): three distinct pool
 * positions, so x1..x3 may all be copies of the best config.  Needs
 * npop - 1 + (best ? information_sharing : 0) >= 3. */
int ut_propose_de(ut_ctx* ctx, const ut_de_params* p, uint32_t round_, int64_t cand_base, int64_t m,
                  double* out_values, int64_t ld);

/* PSO (pso.py:11-77, HybridParticle + op3_swarm per kind).  Candidate g
 * moves particle g % npop towards gbest (device row [P]) and its own best. */
typedef struct ut_pso_params {
  double omega, phi_l, phi_g;   /* 0.5, 0.5, 0.5 (pso.py:49) */
  double sigma;                 /* Int/Pow2 gaussian noise, unit scale 0.2 (manipulator.py:661) */
  int32_t alias_pbest;          /* 1 = reference: particle.best IS the position (pso.py:46, :60) */
  int32_t enum_mode;            /* 0 = reference: enum never moves (manipulator.py:442); 1 = corrected */
  int32_t crossover;            /* PERM: UT_X_* of PSO(crossover=...) (pso.py:80-84; op3_swarm :1115-1140) */
  int32_t pad;
} ut_pso_params;
/* velocities := 0 and particle bests := positions (pso.py:59-68) */
int ut_pso_reset(ut_ctx* ctx);
int ut_propose_pso(ut_ctx* ctx, const ut_pso_params* p, const double* gbest, uint32_t round_, int64_t cand_base,
                   int64_t m, double* out_values, double* out_velocity, int64_t ld);
/* particles [cand_base, cand_base+m) take the moved positions / velocities */
int ut_pso_commit(ut_ctx* ctx, const double* values, const double* velocity, int64_t ld, int64_t cand_base,
                  int64_t m);
/* particle bests for selected particles: best[:, idx[j]] = values[:, j] */
int ut_pso_update_best(ut_ctx* ctx, const double* values, int64_t ld, const int64_t* idx, int64_t n);

/* GA family (evolutionarytechniques.py:13-158, globalGA.py:11-129). */
typedef struct ut_ga_params {
  double mutation_rate;       /* per-param mutation probability */
  double sigma;               /* NormalMutationMixin sigma (0.1) */
  double crossover_rate;      /* probability of selecting two parents */
  double crossover_strength;  /* GGA: fraction of params copied from parent 2 (0.2); 0 = GA family */
  int32_t must_mutate_count;  /* 1; <= P */
  int32_t normal;             /* 1 = NormalGreedyMutation / GGA, 0 = UniformGreedyMutation / GA */
  int32_t max_retries;        /* 10 (hash equal to a parent -> mutate again); <= 15 */
  int32_t op;                 /* RNG stream family: 4 = GA, 5 = GGA */
  int32_t crossover;          /* GA(crossover=...): UT_X_* applied to PERM params of size > 6 when two
                                 parents are selected (CrossoverMixin.crossover :123-134); UT_X_NONE else */
  int32_t pad;
} ut_ga_params;
/* parent1/parent2: device rows [P] (the global best), NULL = random parent
 * (select() without a best result).  out_invalid[i] = 1 when all retries
 * reproduced a parent (the reference returns None). */
int ut_propose_ga(ut_ctx* ctx, const ut_ga_params* p, const double* parent1, const double* parent2,
                  uint32_t round_, int64_t cand_base, int64_t m, double* out_values, int64_t ld,
                  uint8_t* out_invalid);

/* GP features of configurations: unit values (get_unit_value), BOOL 0/1,
 * ENUM one-hot, PERM position of each item / (size - 1).  out_features[f * ld_out + i]. */
int ut_encode_features(ut_ctx* ctx, const double* values, int64_t ld, int64_t m, double* out_features,
                       int64_t ld_out);

/* ---- identity + dedup (hash_config, driver.get_configuration) ----------- */
int ut_hash(ut_ctx* ctx, const double* values, int64_t ld, int64_t m, uint32_t* out_digest);
/* The same digests for DE trials of the selected population: candidate i's
 * target is member (cand_base + i) % npop (ut_propose_de).  Inner digests of
 * values bitwise equal to the target's are taken from a per-population cache
 * (built on first use, patched by ut_population_replace); only the changed
 * values are formatted and hashed.  Correct for any values (a value that does
 * not match its "target" is simply recomputed); fast when most match. */
int ut_hash_de(ut_ctx* ctx, const double* values, int64_t ld, int64_t m, int64_t cand_base, uint32_t* out_digest);
/* The same digests for GA / GGA children of one parent config (ut_propose_ga:
 * parent1, a device row of ncols values; mutation and crossover change a few
 * params, the rest are the parent's): inner digests of values bitwise equal
 * to the parent's come from the parent's own digests (computed once per call);
 * only the changed values are formatted and hashed.  Correct for any values.
 * Replaces the per-child hash_config of evolutionarytechniques.py:38-49. */
int ut_hash_parent(ut_ctx* ctx, const double* values, int64_t ld, int64_t m, const double* parent,
                   uint32_t* out_digest);
int ut_history_reset(ut_ctx* ctx, int64_t capacity);
int ut_history_add(ut_ctx* ctx, const uint32_t* digests, int64_t n);   /* device [n][8] */
int ut_history_add_host(ut_ctx* ctx, const uint32_t* digests_host, int64_t n);
/* out_dup[i] = 1 if digest i is in the history or repeats an earlier
 * (smaller index) candidate of the same batch. */
int ut_dedup(ut_ctx* ctx, const uint32_t* digests, int64_t m, uint8_t* out_dup);

/* ---- GP surrogate ------------------------------------------------------- */
/* X_host: [n][d] features, y_host: [n] objective (minimised).  Fits
 * L = chol(K + (sigma_n2 + jitter) I), L^-1, alpha on the device. */
int ut_gp_fit(ut_ctx* ctx, const double* X_host, const double* y_host, int32_t n, int32_t d,
              const ut_gp_hyper* hyper);
/* The same fit, enqueued on the context's internal fit stream without a host
 * wait: it runs beside whatever is enqueued next (e.g. the proposal and hash
 * stages of the next round), and every later scoring call waits for it on the
 * device.  X_host / y_host may be reused on return (they are staged in
 * pinned memory); the fit's launches are issued by the next call that needs
 * them -- after the proposal of ut_score_round_* / ut_propose_* (ordered
 * before it on the device), or on entry to any call that reads GP state.
 * A failed fit (not positive definite) is reported by ut_gp_stats /
 * ut_gp_fit_status, and makes every score NaN (nothing is selected). */
int ut_gp_fit_async(ut_ctx* ctx, const double* X_host, const double* y_host, int32_t n, int32_t d,
                    const ut_gp_hyper* hyper);
/* Incremental fits (default on; UT_FIT_APPEND=0 or enable=0 turns them off):
 * when a fit's training set extends the previous fit's -- its first n_old
 * rows bitwise equal to the previous X, the same hyperparameters, the same
 * padded size (n rounded up to 128) and a positive-definite previous factor --
 * the factor is extended by block rows (B = K21 L^-T, D = chol(K22 - B B^T),
 * new L^-1 rows -D^-1 B L^-1) instead of refactored: O(n^2 k) instead of
 * O(n^3).  The posterior equals the refit's to rounding.  The tuning loop's
 * per-generation refit (SharedModel.fit: the results table only grows) is
 * exactly this case.  ut_gp_last_fit_kind: 0 = the last fit refactored,
 * 1 = it appended. */
int ut_gp_set_fit_append(ut_ctx* ctx, int32_t enable);
int ut_gp_last_fit_kind(ut_ctx* ctx, int32_t* kind);
/* posterior of standardised y and the acquisition score for m candidates
 * (features [d][ld]).  mu/var/score may be NULL.  dup (may be NULL) marks
 * candidates excluded from selection (score forced to -inf). */
int ut_gp_score(ut_ctx* ctx, const double* features, int64_t ld, int64_t m, const ut_acq* acq,
                const uint8_t* dup, double* mu, double* var, double* score);
/* ut_gp_score on raw values [ncols][ld] instead of features: the encoding
 * (ut_encode_features), the 1/lengthscale scaling and |u|^2 run as one pass
 * that writes only what the K* GEMM reads, so no [d][m] feature matrix is
 * written and read back.  Same results as ut_gp_score(ut_encode_features(values))
 * for values in their parameters' domains: ENUM values are option indices in
 * [0, n_options) and BOOL values 0 or 1, as every proposal kernel writes them
 * (the reference has no other values: an out-of-range index raises in
 * EnumParameter, manipulator.py).  In categorical mode (ut_gp_kstar_mode) an
 * out-of-range ENUM value matches no option (2 / ell^2 against every training
 * row, where the dense encoding's all-zero block gives 1 / ell^2) and a BOOL
 * value other than 0 counts as 1. */
int ut_gp_score_values(ut_ctx* ctx, const double* values, int64_t ld, int64_t m, const ut_acq* acq,
                       const uint8_t* dup, double* mu, double* var, double* score);
/* Selection-exact pruned scoring + top-k (fp64 fits only; EI, or UCB with
 * kappa >= 0: scores that increase with sigma).  sigma^2 = sf2 - |L^-1 k*|^2
 * and every row of L^-1 k* adds a square, so the first `bound_rows` rows give
 * an upper bound on sigma^2, hence on the score, at a (bound_rows / n)^2
 * fraction of the variance GEMM.  The exact scores of the 1024 best bounds
 * give a threshold tau (their k-th best); only candidates whose bound reaches
 * tau get the full variance GEMM, and the top-k of those is the top-k of the
 * dense evaluation (every pruned candidate's exact score < tau <= the k-th
 * best).  out_idx/out_score [k] as ut_topk (global indices cand_base + i).
 * The mean is k* . alpha (K* epilogue), so the whole fit is waited for.  One
 * host synchronisation (the survivor count).  stats (host, may be NULL):
 * survivors, the bound rows used, tau. */
typedef struct ut_prune_stats {
  int64_t survivors;     /* candidates that got the full variance (m if the round fell back to dense) */
  int32_t bound_rows;    /* rows of L^-1 k* in the bound (a multiple of 128) */
  int32_t dense;         /* 1: too many survivors, the round ran the dense variance instead */
  double threshold;      /* tau */
} ut_prune_stats;
int ut_gp_topk_pruned(ut_ctx* ctx, const double* features, int64_t ld, int64_t m, const ut_acq* acq,
                      const uint8_t* dup, int64_t cand_base, int32_t k, int32_t bound_rows, int64_t* out_idx,
                      double* out_score, ut_prune_stats* stats_host);
/* arithmetic of the two scoring contractions (K* and L^-1 K*^T) for fits made
 * after this call: 64 = fp64 MFMA (default; 1e-5 parity), 32 = fp32 MFMA
 * (1e-3 parity), 16 = "f16x3": K* in fp64, the variance contraction as three
 * fp16 MFMA products (hi*hi + hi*lo + lo*hi) of scaled hi/lo splits of L^-1 and
 * K*, f32 accumulate (fp32-class, the same 1e-3 parity tier), 8 = the fp64
 * tier on the int8 MFMA: K* in fp64 (mean k* . alpha in fp64), the variance
 * contraction over six 8-bit digit planes of L^-1 and K* with exact int32
 * sums, each candidate's variance error bounded from the digits' truncation;
 * candidates whose bound exceeds ut_gp_set_i8_tol (relative) are recomputed
 * on the fp64 path (1e-5 parity, the fp64 tier's).  The fit itself is always
 * fp64.  Replaces the variance half of the per-candidate GP posterior the
 * reference has none of; precision 8 scores need n <= 16384. */
int ut_gp_set_precision(ut_ctx* ctx, int32_t bits);
/* ut_gp_topk_pruned's bound pass over every candidate: 32 (default) runs the
 * distance contraction past the bound rows on the f32 MFMA and k* = sf2 2^t
 * by v_exp_f32, and widens each candidate's score bound by every rounding of
 * it (|k*^ - k*| <= rho k*^ + 2^-125 sf2 with rho from the contraction length
 * and the norms; the mean within (rho + 2^-19) sum |alpha| k*^; the bound rows
 * stay fp64); the threshold set and the survivors are then scored in fp64
 * (mean k* . alpha), so the selection is the dense one.  64: the bound pass in
 * fp64 (its mean exact and reused for the survivors). */
int ut_gp_set_prune_pass(ut_ctx* ctx, int32_t bits);
/* precision 8: the largest accepted relative error of a candidate's variance
 * (default 2^-20); 0 recomputes every candidate in fp64 */
int ut_gp_set_i8_tol(ut_ctx* ctx, double tol);
/* precision 8: candidates of the last ut_gp_score / round recomputed in fp64
 * (-1: most were, and the whole round ran the fp64 contraction), and the
 * current fit's bound E on |L^-1 k* - v^| */
int ut_gp_i8_stats(ut_ctx* ctx, int64_t* recomputed_host, double* bound_host);
/* precision 8: the fit's error bounds -- E on |L^-1 k* - v^| (the variance)
 * and Emu = sum_r e_r |(L^-1 y)_r| on the mean mu^ = v^ . L^-1 y, which the
 * int8 variance epilogue computes (gp_i8.hip); 0 for other fits.  A candidate
 * is recomputed in fp64 unless its variance bound is <= tol * var and
 * Emu <= tol * sqrt(var). */
int ut_gp_i8_bounds(ut_ctx* ctx, double* E, double* Emu);
/* order everything enqueued on ctx's stream after this call behind the
 * in-flight fit (a stream wait on its event; no host wait).  Scoring that
 * needs the whole fit (pruned, fp32, f16x3) then starts with the fit done, and
 * the proposal / hash stages before it no longer share the CUs with the fit's
 * chain of small kernels. */
int ut_gp_join_fit(ut_ctx* ctx);
/* wait for the last (possibly asynchronous) fit and report whether its kernel
 * matrix was positive definite (*ok = 1) or not (*ok = 0: later scoring
 * yields NaN scores until a new fit succeeds); not an error either way */
int ut_gp_fit_status(ut_ctx* ctx, int32_t* ok);
/* the K* contraction the current fit scores with: *categorical = 1 when its
 * ENUM / BOOL one-hot blocks go through the int8 code product (one lengthscale
 * over those features, every training row one-hot there; candidates encoded
 * by the library), 0 = the dense fp64 contraction over every feature.  Both
 * give the same posterior (the categorical part of |x - u|^2 is exactly
 * 2 / ell^2 per mismatching ENUM, 1 / ell^2 per BOOL); UT_CAT_KSTAR=0 turns
 * the categorical form off. */
int ut_gp_kstar_mode(ut_ctx* ctx, int32_t* categorical);
/* f_best (min standardised y), y mean/std used for standardisation */
int ut_gp_stats(ut_ctx* ctx, double* f_best, double* y_mean, double* y_std);

/* ---- selection ---------------------------------------------------------- */
/* k largest scores, ties -> smallest global index; entries with dup[i]!=0 or
 * NaN score are never selected; missing slots get index -1. */
int ut_topk(ut_ctx* ctx, const double* score, const uint8_t* dup, int64_t m, int64_t cand_base, int32_t k,
            int64_t* out_idx, double* out_score);

/* ---- one whole round: propose(DE) -> hash -> dedup -> encode -> GP score
 *      -> top-k.  Buffers are owned by the context; results copied to the
 *      given device pointers (any may be NULL). ------------------------- */
typedef struct ut_round_out {
  int64_t* topk_idx;      /* [k] global candidate index */
  double* topk_score;     /* [k] */
  uint32_t* topk_digest;  /* [k][8] */
  double* topk_values;    /* [P][k] */
} ut_round_out;
int ut_score_round_de(ut_ctx* ctx, const ut_de_params* de, const ut_acq* acq, uint32_t round_, int64_t cand_base,
                      int64_t m, int32_t k, const ut_round_out* out);
/* A GA / GGA scoring round (UniformGreedyMutation / NormalGreedyMutation / GA /
 * GGA proposals, evolutionarytechniques.py:29-61, globalGA.py:28-48 and :68-76): the
 * children of parent1 (ut_propose_ga's parameters), hash_config of the children
 * (ut_hash_parent with parent1; ut_hash without) and dedup against the history
 * + the batch on a second stream beside the encode and the GP posterior,
 * invalid children (every retry reproduced a parent) counted as duplicates,
 * then the top-k.  The fit must be current (ut_gp_fit / _async). */
int ut_score_round_ga(ut_ctx* ctx, const ut_ga_params* ga, const double* parent1, const double* parent2,
                      const ut_acq* acq, uint32_t round_, int64_t cand_base, int64_t m, int32_t k,
                      const ut_round_out* out);
/* the same round with ut_gp_topk_pruned's selection-exact pruning in place of
 * the dense variance (fp64 fits; the round's mu/var/score buffers are not
 * filled) */
int ut_score_round_de_pruned(ut_ctx* ctx, const ut_de_params* de, const ut_acq* acq, uint32_t round_,
                             int64_t cand_base, int64_t m, int32_t k, int32_t bound_rows, const ut_round_out* out,
                             ut_prune_stats* stats_host);
/* device pointers to the last round's internal buffers (for tests/bench);
 * features is NULL: the rounds (dense and pruned) encode straight into the K*
 * operands (features / ell, norms, one-hot codes) and keep no feature matrix */
int ut_round_buffers(ut_ctx* ctx, double** values, double** features, uint32_t** digests, uint8_t** dup,
                     double** mu, double** var, double** score, int64_t* ld);

/* ---- tree-ensemble surrogate (the reference's own model family:
 *      plugins/xgbregressor.py:50-63, src/multi_stage.py:8-22) ------------- */
/* pred = (base + sum over trees of scale * leaf) / div, trees in order;
 * LE: go left iff (float)x <= threshold (sklearn), LT: iff (float)x < (float)threshold
 * (XGBoost); NaN features take default_left.  Leaves have feature < 0. */
enum { UT_SPLIT_LE = 0, UT_SPLIT_LT = 1 };
typedef struct ut_tree_node {
  int32_t feature;       /* GP feature column tested; < 0 = leaf */
  int32_t left, right;   /* child node indices (global in the node array) */
  int32_t default_left;  /* NaN goes left */
  double threshold;
  double value;          /* leaf value */
} ut_tree_node;
int ut_forest_set(ut_ctx* ctx, int32_t n_trees, const int32_t* roots_host, int64_t n_nodes,
                  const ut_tree_node* nodes_host, int32_t rule, double base, double scale, double div);
/* features [n_features][ld] (the layout ut_encode_features writes); pred and
 * score [m] may be NULL; score = sign * pred (sign -1: minimise), -inf where dup[i] */
int ut_forest_predict(ut_ctx* ctx, const double* features, int64_t ld, int64_t m, int32_t n_features,
                      const uint8_t* dup, double sign, double* pred, double* score);

/* ---- multi-GPU exchange over RCCL -------------
 * One process per GPU, one communicator per context.  Rank r scores the
 * global candidate indices [r*m, (r+1)*m) of a round; population, training
 * set, GP factor and history set are replicated.  These calls replace the
 * reference's result exchange between its parallel_factor search instances
 * (python/uptune/api.py:400-401 creates them, :547-553 api.sync injects every
 * instance's results into the others; opentuner/api.py:87-104 TuningRunManager.sync).
 * Collectives are enqueued on the context's stream (ut_set_stream) with no
 * host wait, except ut_comm_bcast_results (it returns the broadcast count)
 * and ut_comm_barrier. */
#define UT_COMM_ID_BYTES 128
/* a fresh communicator id (rank 0 creates it; the caller hands the 128 bytes
 * to every rank, e.g. over torch.distributed's store) */
int ut_comm_unique_id(uint8_t* id_host);
/* join the communicator (blocks until all nranks ranks have joined); the
 * context's device is this rank's GPU */
int ut_comm_init(ut_ctx* ctx, int32_t rank, int32_t nranks, const uint8_t* id_host);
int ut_comm_destroy(ut_ctx* ctx);
int ut_comm_info(ut_ctx* ctx, int32_t* rank, int32_t* nranks);
/* the merged top-k of every rank's local top-k (all-gather + ut_topk_merge):
 * in: idx [k] (global, -1 = empty), score [k], digest [k][8], and optionally
 * the selected rows [ncols][ld_rows] (ncols = 0: none).  out: the merged
 * idx / score / digest [k] and rows [ncols][ld_out], identical on every rank
 * (any output may be NULL).  When a call needs larger record buffers than the
 * ranks last agreed on, every rank allocates and the ranks agree on success
 * (an all-reduce MIN) before the all-gather: an allocation failure on any
 * rank returns UT_ENOMEM on every rank, none is left inside the collective. */
int ut_comm_allgather_topk(ut_ctx* ctx, int32_t k, const int64_t* idx, const double* score, const uint32_t* digest,
                           const double* rows, int64_t ld_rows, int32_t ncols, int64_t* out_idx, double* out_score,
                           uint32_t* out_digest, double* out_rows, int64_t ld_out);
/* the merge alone, on n gathered records (no communicator needed): records
 * with idx < 0 or a NaN score are empty; among records with equal digests only
 * the smallest global index survives (a configuration proposed on two shards
 * is requested once); the k best survivors by (-score, idx) fill the output in
 * that order, empty slots get idx -1, score -inf, a zero digest and zero rows. */
int ut_topk_merge(ut_ctx* ctx, int64_t n, int32_t k, const int64_t* idx, const double* score, const uint32_t* digest,
                  const double* rows, int64_t ld_rows, int32_t ncols, int64_t* out_idx, double* out_score,
                  uint32_t* out_digest, double* out_rows, int64_t ld_out);
/* the per-round history delta from `root`: objective values y [n] and digests
 * [n][8] (device buffers of capacity `cap` on every rank).  The root's n goes
 * first, so every rank learns it (*n_out_host) and takes part in the payload
 * broadcast even when its own n differs; n > cap is UT_EINVAL after the
 * collective (rows beyond cap are dropped).  No rank is left inside a
 * collective when another fails: a root whose own arguments are bad sends a
 * sentinel count and every rank returns UT_EINVAL; the ranks agree on the
 * payload allocation before the payload broadcast (UT_ENOMEM on all). */
int ut_comm_bcast_results(ut_ctx* ctx, int32_t root, int64_t n, double* y, uint32_t* digest, int64_t cap,
                          int64_t* n_out_host);
/* raw broadcast of `bytes` bytes of a device buffer from `root` */
int ut_comm_bcast(ut_ctx* ctx, void* buf, int64_t bytes, int32_t root);
/* in-place all-reduce of n doubles (device buffer) */
enum { UT_RED_SUM = 0, UT_RED_MAX = 1, UT_RED_MIN = 2 };
int ut_comm_allreduce_f64(ut_ctx* ctx, double* buf, int64_t n, int32_t op);
/* every rank's stream reaches this point (an all-reduce, then a stream sync) */
int ut_comm_barrier(ut_ctx* ctx);
/* Fault injection for tests: the next `count` device allocations of the
 * context that would grow a buffer fail with UT_ENOMEM (0 clears it). */
int ut_debug_fail_alloc(ut_ctx* ctx, int32_t count);

/* per-kernel device time (ms) of the ut_score_round_* calls since timing was
 * enabled with ut_set_timing(ctx, 1), averaged over those rounds.  Events are
 * recorded without host synchronisation; ut_stage_time synchronises once.  names: "propose", "hash",
 * "dedup", "encode", "gp_fit", "kstar", "var", "finalize", "topk" */
int ut_set_timing(ut_ctx* ctx, int32_t on);
int ut_stage_time(ut_ctx* ctx, const char* stage, double* ms);

#ifdef __cplusplus
}
#endif
#endif /* UTHOT_H */
