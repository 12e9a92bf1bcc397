"""Tree-ensemble surrogate: flattening of sklearn and
XGBoost-JSON models and the restated traversal, pinned by sklearn's predict
(CPU); the device kernel is checked in tests/test_gpu_forest.py."""
import json

import numpy as np
import pytest

from oracle import forest as of
from uptune_amd import forest as F


def _data(m=400, d=7, seed=0):
    rng = np.random.default_rng(seed)
    X = rng.uniform(size=(m, d))
    y = np.sin(6 * X[:, 0]) + X[:, 1] ** 2 - 0.5 * X[:, 2] * X[:, 3] + 0.05 * rng.standard_normal(m)
    return X, y


def _models():
    from sklearn.ensemble import ExtraTreesRegressor, GradientBoostingRegressor, RandomForestRegressor
    from sklearn.tree import DecisionTreeRegressor
    X, y = _data()
    return [DecisionTreeRegressor(max_depth=8, random_state=0).fit(X, y),
            RandomForestRegressor(n_estimators=25, max_depth=9, random_state=0).fit(X, y),
            ExtraTreesRegressor(n_estimators=20, random_state=1).fit(X, y),
            GradientBoostingRegressor(n_estimators=40, max_depth=4, learning_rate=0.07, random_state=0).fit(X, y)]


@pytest.mark.parametrize("k", range(4))
def test_flattened_sklearn_equals_predict(k):
    model = _models()[k]
    f = F.from_sklearn(model)
    Xq, _ = _data(300, 7, seed=5)
    Xq[:40] = np.round(Xq[:40], 2)     # values on (float32-rounded) thresholds
    got = of.predict(f.nodes, f.roots, f.rule, f.base, f.scale, f.div, Xq)
    np.testing.assert_array_equal(got, model.predict(Xq))


def test_xgboost_json_layout():
    # a hand-written 2-tree model in XGBoost's JSON schema (save_model format)
    tree0 = {"left_children": [1, -1, -1], "right_children": [2, -1, -1], "split_indices": [0, 0, 0],
             "split_conditions": [0.5, -1.0, 2.0], "default_left": [1, 0, 0]}
    tree1 = {"left_children": [1, 3, -1, -1, -1], "right_children": [2, 4, -1, -1, -1],
             "split_indices": [1, 2, 0, 0, 0], "split_conditions": [0.25, 0.75, 0.5, -0.125, 0.0625],
             "default_left": [0, 1, 0, 0, 0]}
    doc = {"learner": {"learner_model_param": {"base_score": "5E-1"},
                       "gradient_booster": {"model": {"trees": [tree0, tree1]}}}}
    f = F.from_xgboost_json(json.dumps(doc))
    X = np.array([[0.4, 0.1, 0.9], [0.6, 0.3, 0.0], [0.5, 0.25, 0.75], [np.nan, 0.1, 0.2]])
    got = of.predict(f.nodes, f.roots, f.rule, f.base, f.scale, f.div, X)
    # by hand: row0 -1.0 + (0.1<.25 -> node1: 0.9<.75? no -> node4 .0625); row1 2.0 + 0.5;
    # row2 (x0 == 0.5 is not < 0.5 -> right) 2.0 + (0.25 < 0.25? no -> 0.5); row3 NaN -> left -1.0 + node1 (0.2 < .75 -> -0.125)
    assert got.tolist() == [0.5 - 1.0 + 0.0625, 0.5 + 2.0 + 0.5, 0.5 + 2.0 + 0.5, 0.5 - 1.0 - 0.125]
