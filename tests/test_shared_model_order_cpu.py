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
