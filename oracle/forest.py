"""Tree-ensemble inference restated (TEST INFRASTRUCTURE: imported only by
tests/).  The traversal of scikit-learn's tree predict (sklearn/tree/_tree.pyx
`apply`: left iff X[i, feature] <= threshold with X converted to float32) and
the ensemble combinations of ForestRegressor.predict (sum in estimator order,
then / n_estimators) and GradientBoostingRegressor (init constant, then
raw += learning_rate * leaf per stage, predict_stages); XGBoost's documented
rule (left iff x < split_condition in float32, missing -> default_left,
base_score + sum of leaves).  Pinned by sklearn's own predict in
tests/test_forest.py; the XGBoost branch is parity unpinned (xgboost is not
installed)."""
import numpy as np

LE, LT = 0, 1


def predict(nodes, roots, rule, base, scale, div, X):
    """nodes: structured array (uptune_amd.forest.NODE_DTYPE); X [m][F] f64"""
    out = np.empty(X.shape[0])
    for i in range(X.shape[0]):
        acc = float(base)
        for r in roots:
            nd = int(r)
            while nodes["feature"][nd] >= 0:
                f = int(nodes["feature"][nd])
                x = float(X[i, f])
                if x != x:
                    left = bool(nodes["default_left"][nd])
                elif rule == LE:
                    left = float(np.float32(x)) <= float(nodes["threshold"][nd])
                else:
                    left = np.float32(x) < np.float32(nodes["threshold"][nd])
                nd = int(nodes["left"][nd] if left else nodes["right"][nd])
            acc += scale * float(nodes["value"][nd])
        out[i] = acc / div
    return out
