// forest.hip -- batched tree-ensemble inference: the reference's own surrogate
// (SURVEY.md §8(f) row 4).  The multi-stage tuner scores candidates with
// ModelBase.inference one sample at a time (python/uptune/src/multi_stage.py:8-22,
// plugins/xgbregressor.py:50-63) and ranks them (multi_stage.py:109-123); here
// one lane walks every tree of the ensemble for one candidate.
//
//   pred = (base + sum_t scale * leaf_t(x)) / div        (sum in tree order)
//     RandomForest / ExtraTrees   base 0, scale 1, div T   (ForestRegressor.predict)
//     GradientBoosting            base init_, scale lr, div 1  (predict_stages)
//     XGBoost JSON model          base base_score, scale 1, div 1
//   split rule  LE: x <= thr (sklearn: x rounded to float32 first)
//               LT: x <  thr (XGBoost: float32 compare); NaN -> default child
//
// Nodes are 32-byte records (one load per visited node); the ensemble is small
// (MBs) and stays L2 / MALL resident while lanes gather their paths.  Bound:
// latency of the dependent node loads, hidden by occupancy (few VGPRs).
#include "ut_internal.h"

namespace ut {

__global__ __launch_bounds__(256) void k_forest(const ut_tree_node* __restrict__ nodes,
                                                const int32_t* __restrict__ roots, int32_t n_trees, int32_t rule,
                                                double base, double scale, double div, int32_t n_feat,
                                                const double* __restrict__ feat, int64_t ld, int64_t m,
                                                const uint8_t* __restrict__ dup, double sign,
                                                double* __restrict__ pred, double* __restrict__ score) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= m) return;
  double acc = base;
  for (int32_t t = 0; t < n_trees; ++t) {
    int32_t nd = roots[t];
    for (int32_t depth = 0; depth < 4096; ++depth) {  // bounded: a malformed tree cannot hang the wave
      const ut_tree_node q = nodes[nd];
      if (q.feature < 0) break;
      const int32_t f = q.feature < n_feat ? q.feature : n_feat - 1;
      const double x = feat[(int64_t)f * ld + i];
      bool left;
      if (x != x) {
        left = q.default_left != 0;
      } else if (rule == UT_SPLIT_LE) {
        left = (double)(float)x <= q.threshold;
      } else {
        left = (float)x < (float)q.threshold;
      }
      nd = left ? q.left : q.right;
    }
    acc += scale * nodes[nd].value;
  }
  const double p = acc / div;
  if (pred) pred[i] = p;
  if (score) score[i] = (dup && dup[i]) ? -1.0 / 0.0 : sign * p;
}

}  // namespace ut

extern "C" int ut_forest_set(ut_ctx* c, int32_t n_trees, const int32_t* roots_host, int64_t n_nodes,
                             const ut_tree_node* nodes_host, int32_t rule, double base, double scale, double div) {
  if (!c) return UT_EINVAL;
  UT_CHECK(c, n_trees >= 1 && n_nodes >= 1 && roots_host && nodes_host, UT_EINVAL, "forest_set: empty ensemble");
  UT_CHECK(c, rule == UT_SPLIT_LE || rule == UT_SPLIT_LT, UT_EINVAL, "forest_set: bad split rule");
  UT_CHECK(c, div != 0.0, UT_EINVAL, "forest_set: div must be non-zero");
  // validate on the host: every child / root index in range (a bad index would fault on the device)
  for (int32_t t = 0; t < n_trees; ++t)
    UT_CHECK(c, roots_host[t] >= 0 && roots_host[t] < n_nodes, UT_EINVAL, "forest_set: root out of range");
  for (int64_t k = 0; k < n_nodes; ++k) {
    const ut_tree_node& q = nodes_host[k];
    if (q.feature >= 0)
      UT_CHECK(c, q.left >= 0 && q.left < n_nodes && q.right >= 0 && q.right < n_nodes, UT_EINVAL,
               "forest_set: child out of range");
  }
  UT_HIP(c, hipSetDevice(c->device));
  UT_HIP(c, ut::sync_all(c));
  if (c->forest_nodes) ut::dfree(c->forest_nodes);
  if (c->forest_roots) ut::dfree(c->forest_roots);
  c->forest_nodes = nullptr;
  c->forest_roots = nullptr;
  c->forest_trees = 0;
  UT_HIP(c, ut::dmalloc((void**)&c->forest_nodes, sizeof(ut_tree_node) * n_nodes));
  UT_HIP(c, ut::dmalloc((void**)&c->forest_roots, sizeof(int32_t) * n_trees));
  UT_HIP(c, hipMemcpy(c->forest_nodes, nodes_host, sizeof(ut_tree_node) * n_nodes, hipMemcpyHostToDevice));
  UT_HIP(c, hipMemcpy(c->forest_roots, roots_host, sizeof(int32_t) * n_trees, hipMemcpyHostToDevice));
  c->forest_trees = n_trees;
  c->forest_rule = rule;
  c->forest_base = base;
  c->forest_scale = scale;
  c->forest_div = div;
  return 0;
}

extern "C" int ut_forest_predict(ut_ctx* c, const double* features, int64_t ld, int64_t m, int32_t n_features,
                                 const uint8_t* dup, double sign, double* pred, double* score) {
  if (!c) return UT_EINVAL;
  UT_CHECK(c, c->forest_trees > 0, UT_EINVAL, "forest_predict: call ut_forest_set first");
  UT_CHECK(c, features && n_features >= 1 && ld >= m && m >= 0, UT_EINVAL, "forest_predict: bad arguments");
  if (m == 0) return 0;
  hipLaunchKernelGGL(ut::k_forest, dim3(ut::grid1(m, 256)), dim3(256), 0, c->stream, c->forest_nodes,
                     c->forest_roots, c->forest_trees, c->forest_rule, c->forest_base, c->forest_scale,
                     c->forest_div, n_features, features, ld, m, dup, sign, pred, score);
  UT_LAUNCH_CHECK(c);
  return 0;
}
