"""Tree-ensemble surrogate on the device (csrc/forest.hip) vs the restated
traversal (oracle/forest.py, itself pinned to sklearn's predict): bit-exact
predictions, -inf on duplicates, top-k of the ranking.  Needs a GPU."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from oracle import forest as of  # noqa: E402
from oracle import select as osel  # noqa: E402


def _engine(d):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from uptune_amd.engine import BatchEngine
    from uptune_amd.manipulator import ConfigurationManipulator, FloatParameter
    return BatchEngine(ConfigurationManipulator([FloatParameter("u%d" % k, 0.0, 1.0) for k in range(d)]))


def _fit():
    from sklearn.ensemble import GradientBoostingRegressor, RandomForestRegressor
    rng = np.random.default_rng(0)
    X = rng.uniform(size=(500, 6))
    y = np.cos(5 * X[:, 0]) + X[:, 1] * X[:, 2] + 0.05 * rng.standard_normal(500)
    return [RandomForestRegressor(n_estimators=30, max_depth=10, random_state=0).fit(X, y),
            GradientBoostingRegressor(n_estimators=60, max_depth=5, learning_rate=0.05, random_state=0).fit(X, y)]


def test_forest_predict_matches_oracle_and_sklearn():
    from uptune_amd import forest as F
    e = _engine(6)
    rng = np.random.default_rng(7)
    Xq = rng.uniform(size=(20000, 6))
    Xq[:500] = np.round(Xq[:500], 2)
    feat = torch.from_numpy(np.ascontiguousarray(Xq.T)).cuda()
    for model in _fit():
        f = F.from_sklearn(model)
        e.forest_set(f)
        pred, score = e.forest_predict(feat)
        got = pred.cpu().numpy()
        np.testing.assert_array_equal(got[:3000], of.predict(f.nodes, f.roots, f.rule, f.base, f.scale, f.div,
                                                             Xq[:3000]))
        np.testing.assert_array_equal(got, model.predict(Xq))
        np.testing.assert_array_equal(score.cpu().numpy(), -got)


def test_forest_scorer_ranking_with_dups():
    from uptune_amd.forest import ForestScorer
    e = _engine(6)
    models = _fit()
    rng = np.random.default_rng(3)
    Xq = rng.uniform(size=(5000, 6))
    feat = torch.from_numpy(np.ascontiguousarray(Xq.T)).cuda()
    dup = torch.zeros(5000, dtype=torch.uint8, device="cuda")
    dup[::7] = 1
    sc = ForestScorer(e, models)
    mean = sc.predict(feat).cpu().numpy()
    want_mean = (models[0].predict(Xq) + models[1].predict(Xq)) / 2
    np.testing.assert_array_equal(mean, want_mean)
    # minimise: score = -pred, duplicates never selected; top-k == oracle ranking
    e.forest_set(models[1])
    _, score = e.forest_predict(feat, dup=dup)
    idx, _ = e.topk(score, 64, dup=dup)
    pred = models[1].predict(Xq)
    want = osel.topk(list(-pred), 64, dup=dup.cpu().numpy().tolist())
    assert idx.cpu().numpy().tolist() == want


def test_technique_with_forest_surrogate():
    """a GPU DE technique ranking its pool with a tree ensemble instead of the GP"""
    from sklearn.ensemble import RandomForestRegressor

    from uptune_amd import technique as T
    from uptune_amd.driver import SearchDriver
    from uptune_amd.manipulator import ConfigurationManipulator, FloatParameter
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    m = ConfigurationManipulator([FloatParameter("u%d" % k, 0.0, 1.0) for k in range(6)])
    rng = np.random.default_rng(1)
    X = rng.uniform(size=(400, 6))
    y = np.sum((X - 0.7) ** 2, axis=1)
    rf = RandomForestRegressor(n_estimators=20, random_state=0).fit(X, y)
    de = T.GpuDifferentialEvolution(pool=4096, batch=4, population=256, seed=2, surrogate=rf, name="de-rf")
    d = SearchDriver(m, de, parallelism=4)
    d.main(lambda c: float(sum((c["u%d" % k] - 0.7) ** 2 for k in range(6))), test_limit=40)
    first = next(iter(d.results.values()))
    assert len(d.results) >= 40 and d.best_result.time <= first.time
    # the queued proposals are the forest's best-ranked candidates of round 0
    assert d.root_technique.engine.forest is not None
