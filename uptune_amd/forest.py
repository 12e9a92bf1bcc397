"""Tree-ensemble surrogates on the device.

The reference's learning plugins score candidates with a tree ensemble one
sample at a time (plugins/xgbregressor.py:50-63 `XGBRegressor.predict`;
plugins/models.py:9-52 `ModelBase.inference`) and the multi-stage tuner
averages the models and ranks the pool (src/multi_stage.py:8-22 `score`,
:109-123).  Here an ensemble is flattened once into 32-byte node records
(`ut_tree_node`) and every candidate of a pool walks it on the GPU
(csrc/forest.hip), on the same features the GP uses.

Accepted models:
  * scikit-learn DecisionTreeRegressor, RandomForestRegressor,
    ExtraTreesRegressor, GradientBoostingRegressor (squared error) --
    predictions identical to `model.predict` (split on float32-rounded x);
  * an XGBoost JSON model (`Booster.save_model("m.json")`, gbtree,
    reg:squarederror), read as data -- xgboost itself is not installed here,
    so XGBoost parity is unpinned (the traversal restates its documented
    rule: left iff x < split_condition in float32, leaves in
    split_conditions, prediction = base_score + sum of leaves).
"""
from __future__ import annotations

import json
from dataclasses import dataclass
from typing import Any, List, Sequence

import numpy as np

from . import _lib as L


@dataclass
class Forest:
    """flattened ensemble: node records + tree roots + the combination rule"""
    nodes: np.ndarray      # structured [feature, left, right, default_left, threshold, value]
    roots: np.ndarray      # int32 [T]
    rule: int              # L.UT_SPLIT_LE / UT_SPLIT_LT
    base: float
    scale: float
    div: float

    @property
    def n_trees(self) -> int:
        return int(self.roots.size)


NODE_DTYPE = np.dtype([("feature", "<i4"), ("left", "<i4"), ("right", "<i4"), ("default_left", "<i4"),
                       ("threshold", "<f8"), ("value", "<f8")])


def _append_sklearn_tree(tree, out: List[np.ndarray], offset: int) -> int:
    t = tree.tree_
    n = t.node_count
    a = np.zeros(n, dtype=NODE_DTYPE)
    leaf = t.children_left < 0
    a["feature"] = np.where(leaf, -1, t.feature)
    a["left"] = np.where(leaf, 0, t.children_left + offset)
    a["right"] = np.where(leaf, 0, t.children_right + offset)
    a["default_left"] = 1
    a["threshold"] = t.threshold
    a["value"] = t.value[:, 0, 0]
    out.append(a)
    return offset + n


def from_sklearn(model) -> Forest:
    """DecisionTree / RandomForest / ExtraTrees / GradientBoosting regressors"""
    name = type(model).__name__
    parts: List[np.ndarray] = []
    roots: List[int] = []
    off = 0
    if name == "DecisionTreeRegressor":
        roots.append(off)
        _append_sklearn_tree(model, parts, off)
        return Forest(np.concatenate(parts), np.array(roots, np.int32), L.UT_SPLIT_LE, 0.0, 1.0, 1.0)
    if name in ("RandomForestRegressor", "ExtraTreesRegressor"):
        for est in model.estimators_:              # ForestRegressor.predict: sum in order, then / T
            roots.append(off)
            off = _append_sklearn_tree(est, parts, off)
        return Forest(np.concatenate(parts), np.array(roots, np.int32), L.UT_SPLIT_LE, 0.0, 1.0,
                      float(len(model.estimators_)))
    if name == "GradientBoostingRegressor":
        init = model.init_
        if not hasattr(init, "constant_"):
            raise TypeError("GradientBoostingRegressor with a non-constant init estimator")
        for est in model.estimators_[:, 0]:         # predict_stages: raw += learning_rate * leaf
            roots.append(off)
            off = _append_sklearn_tree(est, parts, off)
        return Forest(np.concatenate(parts), np.array(roots, np.int32), L.UT_SPLIT_LE,
                      float(np.asarray(init.constant_).ravel()[0]), float(model.learning_rate), 1.0)
    raise TypeError(f"unsupported model {name}")


def from_xgboost_json(doc: Any) -> Forest:
    """an XGBoost JSON model (dict, JSON text or path) -> Forest"""
    if isinstance(doc, str):
        doc = json.loads(doc) if doc.lstrip().startswith("{") else json.load(open(doc))
    learner = doc["learner"]
    base = float(learner["learner_model_param"]["base_score"])
    trees = learner["gradient_booster"]["model"]["trees"]
    parts: List[np.ndarray] = []
    roots: List[int] = []
    off = 0
    for tr in trees:
        lc = np.asarray(tr["left_children"], np.int64)
        rc = np.asarray(tr["right_children"], np.int64)
        n = lc.size
        a = np.zeros(n, dtype=NODE_DTYPE)
        leaf = lc < 0
        cond = np.asarray(tr["split_conditions"], np.float64)
        a["feature"] = np.where(leaf, -1, np.asarray(tr["split_indices"], np.int64))
        a["left"] = np.where(leaf, 0, lc + off)
        a["right"] = np.where(leaf, 0, rc + off)
        a["default_left"] = np.asarray(tr.get("default_left", [1] * n), np.int64)
        a["threshold"] = np.where(leaf, 0.0, cond)
        a["value"] = np.where(leaf, cond, 0.0)           # leaves keep their weight in split_conditions
        parts.append(a)
        roots.append(off)
        off += n
    return Forest(np.concatenate(parts), np.array(roots, np.int32), L.UT_SPLIT_LT, base, 1.0, 1.0)


def as_forest(model) -> Forest:
    if isinstance(model, Forest):
        return model
    if isinstance(model, (dict, str)):
        return from_xgboost_json(model)
    return from_sklearn(model)


class ForestScorer:
    """ModelBase-like wrapper: batch inference of one or more ensembles on the
    device; `score` averages the models like multi_stage.score (:8-22)."""

    def __init__(self, engine, models: Sequence[Any]):
        self.engine = engine
        self.forests = [as_forest(m) for m in models]
        if not self.forests:
            raise ValueError("no model")

    def predict(self, features, dup=None):
        """features: device tensor [F][m] (engine.encode) -> mean prediction [m]"""
        out = None
        for f in self.forests:
            self.engine.forest_set(f)
            p, _ = self.engine.forest_predict(features, dup=dup)
            out = p if out is None else out + p
        return out / len(self.forests)
