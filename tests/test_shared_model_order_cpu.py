"""SharedModel's training-row order (technique.py SharedModel.fit): best y first
at every refit point (a new padded size of 128 rows, as gp.hip NPAD), new results
appended in arriving order in between, so the device's incremental fit still
sees a bitwise prefix.  CPU only: a stand-in engine records what gp_fit gets."""
import types

import numpy as np

from uptune_amd.technique import SharedModel


class _Engine:
    def __init__(self):
        self.spec = types.SimpleNamespace(n_features=2)
        self.fits = []

    def features_host(self, cfgs):
        return np.asarray([[c["a"], c["b"]] for c in cfgs], dtype=np.float64)

    def gp_fit(self, X, y, lengthscale, wait=True, **hyper):
        self.fits.append((np.array(X), np.array(y)))

    def gp_fit_ok(self):
        return True


class _Driver:
    def __init__(self):
        self.rows = []

    def add(self, ys, rng):
        for y in ys:
            cfg = {"a": float(rng.uniform()), "b": float(rng.uniform())}
            self.rows.append(types.SimpleNamespace(configuration=types.SimpleNamespace(data=cfg), time=float(y),
                                                   state="OK", id=len(self.rows)))

    def results_query(self):
        return self.rows


def test_rows_best_first_at_refit_appended_between():
    rng = np.random.default_rng(0)
    m = SharedModel()
    m.engine = _Engine()
    d = _Driver()
    d.add(rng.uniform(size=100), rng)
    assert m.fit(d)
    X0, y0 = m.engine.fits[-1]
    assert np.all(np.diff(y0) >= 0), "first fit: best first"
    # appends within the same padded size (<= 128 rows): prefix kept, new rows last in arriving order
    new = rng.uniform(size=8) - 1.0          # better than every earlier result
    d.add(new, rng)
    assert m.fit(d)
    X1, y1 = m.engine.fits[-1]
    assert np.array_equal(X1[:100], X0) and np.array_equal(y1[:100], y0)
    assert np.array_equal(y1[100:], new)
    # crossing 128 rows: a refit point -> re-sorted, the new best rows lead
    d.add(rng.uniform(size=30), rng)
    assert m.fit(d)
    X2, y2 = m.engine.fits[-1]
    assert len(y2) == 138 and np.all(np.diff(y2) >= 0)
    assert np.array_equal(np.sort(y2), np.sort([r.time for r in d.rows]))
    # rows and their features stay paired under the permutation
    by_y = {r.time: (r.configuration.data["a"], r.configuration.data["b"]) for r in d.rows}
    assert all(tuple(X2[i]) == by_y[y2[i]] for i in range(len(y2)))
    # no change -> no new fit
    n = len(m.engine.fits)
    assert m.fit(d) and len(m.engine.fits) == n


def test_selection_features_equal_features_host():
    """the features a round encodes beside its selections (GpuBatchTechnique._round,
    SharedModel.remember_features) are bitwise the ones features_host gives the
    results' configurations (an enum option listed twice included: proposals
    carry its first index, as encode_configs does)"""
    from _oracle_engine import OracleEngine
    from uptune_amd import technique as T
    from uptune_amd.driver import SearchDriver
    from uptune_amd.manipulator import (BooleanParameter, ConfigurationManipulator, EnumParameter, FloatParameter,
                                        IntegerParameter)

    class Counting(OracleEngine):
        rows_host = 0

        def features_host(self, cfgs):
            Counting.rows_host += len(cfgs)
            return super().features_host(cfgs)

    space = ConfigurationManipulator([FloatParameter("x", -2.0, 2.0), IntegerParameter("n", 0, 50),
                                      EnumParameter("e", ["a", "b", "a", "c"]), BooleanParameter("b")])

    def obj(c):
        return (c["x"] - 0.3) ** 2 + 0.01 * c["n"] + (-0.5 if c["e"] == "a" else 0.0) + (0.1 if c["b"] else 0.0)

    drv = SearchDriver(space, T.GpuGA(name="ga", pool=256, batch=4, population=32, seed=5, lengthscale=0.5,
                                      engine_factory=Counting), parallelism=4)
    drv.main(obj, test_limit=48, max_generations=12)
    sm = drv.root_technique.model
    assert sm.fits >= 5 and sm._n >= 24
    res = drv.results_query()[:sm._n]
    want = sm.engine.features_host([r.configuration.data for r in res])
    assert np.array_equal(sm._Xa[:sm._n].view(np.int64), want.view(np.int64))
    assert np.array_equal(sm._ya[:sm._n], [r.time for r in res])
    Counting.rows_host -= len(res)            # the check above
    assert Counting.rows_host < sm._n         # most rows came from the rounds' encodings


def test_selection_with_two_encodings_is_not_cached():
    """a selected value column that does not re-encode to the same bits (an enum
    option listed twice, at its second index) keeps no round encoding: its
    result is encoded by features_host"""
    import torch
    from _oracle_engine import OracleEngine
    from uptune_amd import technique as T
    from uptune_amd.driver import SearchDriver
    from uptune_amd.manipulator import ConfigurationManipulator, EnumParameter, FloatParameter

    class Fixed(T.GpuGA):
        def _local_round(self):
            eng = self._ensure_engine()
            rows = torch.zeros((eng.spec.ncols, 2), dtype=torch.float64)
            for ps in eng.spec.params:
                rows[ps.col] = torch.tensor([0.25, -0.5] if ps.name == "x" else [2.0, 1.0])   # e: "a" (2nd), "b"
            return rows, torch.tensor([0, 1]), torch.zeros(2, dtype=torch.float64), eng.hash(rows), rows

    space = ConfigurationManipulator([FloatParameter("x", -2.0, 2.0), EnumParameter("e", ["a", "b", "a", "c"])])
    drv = SearchDriver(space, Fixed(name="ga", pool=16, batch=2, population=8, seed=1, engine_factory=OracleEngine),
                       parallelism=2)
    t = drv.root_technique
    t._round()
    cache = t.model._feat_cache
    (c0, h0), (c1, h1) = t.queue
    assert c0["e"] == "a" and c1["e"] == "b"
    assert h0 not in cache and h1 in cache
    want = t.engine.features_host([c1])[0]
    assert np.array_equal(cache[h1].view(np.int64), want.view(np.int64))


def test_queued_selections_are_in_the_dedup_set():
    """two techniques sharing one model: the second round, run before any of the
    first round's selections is requested, selects none of them (the same
    technique twice proposes the same candidates, so without the round-time
    dedup entries the two queues would be equal)"""
    from _oracle_engine import OracleEngine
    from uptune_amd import technique as T
    from uptune_amd.driver import SearchDriver
    from uptune_amd.manipulator import ConfigurationManipulator, FloatParameter, IntegerParameter

    space = ConfigurationManipulator([FloatParameter("x", -2.0, 2.0), IntegerParameter("n", 0, 50)])
    sm = T.SharedModel(seed=4, engine_factory=OracleEngine)
    kw = dict(pool=64, batch=4, population=16, seed=4, shared=sm)
    drv = SearchDriver(space, T.MetaSearchTechnique([T.GpuGA(name="a", **kw), T.GpuGA(name="b", **kw)]),
                       parallelism=4)
    a, b = drv.root_technique.techniques
    assert a.model is b.model
    a._round()
    b._round()
    ha = {h for _, h in a.queue}
    hb = {h for _, h in b.queue}
    assert len(ha) == 4 and len(hb) == 4 and not (ha & hb)
    assert ha | hb <= a.model._hist


def test_rank_transform_fits_normal_scores():
    """y_transform="rank": the GP is fitted on Phi^-1((rank + 1/2) / n) of the
    objective in the fit's row order (order preserved, so the incumbent is the
    minimum); the rows and the append prefix are the untransformed run's"""
    from scipy.special import ndtri
    rng = np.random.default_rng(1)
    raw, rk = SharedModel(), SharedModel(y_transform="rank")
    raw.engine, rk.engine = _Engine(), _Engine()
    d = _Driver()
    d.add(10.0 ** rng.uniform(0, 14, size=100), rng)          # an objective spanning 14 decades
    for step in range(3):
        assert raw.fit(d) and rk.fit(d)
        (Xr, yr), (Xk, yk) = raw.engine.fits[-1], rk.engine.fits[-1]
        assert np.array_equal(Xr, Xk)
        n = len(yr)
        want = np.empty(n)
        want[np.argsort(yr, kind="stable")] = ndtri((np.arange(n) + 0.5) / n)
        assert np.array_equal(yk, want)
        assert np.argmin(yk) == np.argmin(yr)
        d.add(10.0 ** rng.uniform(0, 14, size=8), rng)
    try:
        SharedModel(y_transform="log")
    except ValueError:
        pass
    else:
        raise AssertionError("unknown y_transform accepted")
