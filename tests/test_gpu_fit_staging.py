"""The staged asynchronous fit (gp.hip gp_fit_enqueue / gp_fit_flush):
ut_gp_fit_async stages X, y and the host-side decisions and the fit's launches
are issued by the next call that needs them -- after a round's proposal, or on
entry to anything that reads GP state.  Every path must give what a synchronous
fit gives, bit for bit.  (The GP itself follows SharedModel's posterior, which
the reference does not have: SURVEY F2, parity against oracle/gp.py only.)"""
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from oracle import de as ode  # noqa: E402
from oracle import gp as ogp  # noqa: E402
from oracle.space import FLOAT, Param, features  # noqa: E402

pytestmark = pytest.mark.gpu


def _require_gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")


from _spaces import to_manip  # noqa: E402

HYP = dict(sigma_f2=1.0, sigma_n2=1e-6, jitter=1e-8)


def engine(space, seed=0):
    _require_gpu()
    from uptune_amd.engine import BatchEngine
    return BatchEngine(to_manip(space), device=0, seed=seed)


def dev(a):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a)).to("cuda:0")


def _data(n, d, seed):
    rng = np.random.default_rng(seed)
    X = rng.uniform(size=(n, d))
    y = np.sum((X - 0.4) ** 2, axis=1) + 0.01 * rng.standard_normal(n)
    return X, y


def _score(e, U):
    return [t.cpu().numpy() for t in e.gp_score(dev(U.T))]


@pytest.mark.parametrize("prec", [64, 8])
def test_superseded_async_fit(prec):
    """a staged fit never used is issued when the next fit is staged; scoring
    then sees the second fit only, equal to a synchronous fit of it"""
    n, d = 300, 16
    X1, y1 = _data(n, d, 1)
    X2, y2 = _data(n, d, 2)
    U = np.random.default_rng(3).uniform(size=(2000, d))
    space = [Param(f"u{k}", FLOAT, 0.0, 1.0) for k in range(d)]
    a = engine(space)
    a.gp_set_precision(prec)
    a.gp_fit(X1, y1, lengthscale=0.5, wait=False, **HYP)
    a.gp_fit(X2, y2, lengthscale=0.5, wait=False, **HYP)
    got = _score(a, U)
    b = engine(space)
    b.gp_set_precision(prec)
    b.gp_fit(X2, y2, lengthscale=0.5, **HYP)
    want = _score(b, U)
    for g, w in zip(got, want):
        np.testing.assert_array_equal(g, w)
    assert a.gp_stats() == b.gp_stats()
    mu_o, var_o = ogp.GP(X2, y2, lengthscale=0.5, **HYP).posterior(U)
    np.testing.assert_allclose(got[0], mu_o, rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(got[1], var_o, rtol=1e-5, atol=1e-8)


@pytest.mark.parametrize("prec", [64, 8])
def test_async_append_chain_without_scoring(prec):
    """appends staged back to back (each issues the one before it): the last
    is an append, and the posterior equals a fresh fit of the whole set"""
    n0, d = 500, 8
    X, y = _data(n0 + 12, d, 4)
    U = np.random.default_rng(5).uniform(size=(1500, d))
    U[:10] = X[-10:] + 1e-3
    space = [Param(f"u{k}", FLOAT, 0.0, 1.0) for k in range(d)]
    a = engine(space)
    a.gp_set_precision(prec)
    for n in (n0, n0 + 4, n0 + 8, n0 + 12):
        a.gp_fit(X[:n], y[:n], lengthscale=0.5, wait=False, **HYP)
    assert a.gp_last_fit_kind() == "append"
    got = _score(a, U)
    b = engine(space)
    b.gp_set_precision(prec)
    b.gp_fit(X, y, lengthscale=0.5, **HYP)
    want = _score(b, U)
    for g, w in zip(got, want):
        np.testing.assert_allclose(g, w, rtol=1e-10, atol=1e-12)


def test_async_fit_entry_points():
    """each entry point that reads GP state issues a staged fit first: the fit
    status, the stats, a precision change after the fit (the fit keeps the
    precision it was staged at), the join, and a fit that is not positive
    definite"""
    n, d = 256, 6
    X, y = _data(n, d, 6)
    U = np.random.default_rng(7).uniform(size=(1000, d))
    space = [Param(f"u{k}", FLOAT, 0.0, 1.0) for k in range(d)]
    ref = engine(space)
    ref.gp_set_precision(8)
    ref.gp_fit(X, y, lengthscale=0.4, **HYP)
    want = _score(ref, U)
    e = engine(space)
    e.gp_set_precision(8)
    e.gp_fit(X, y, lengthscale=0.4, wait=False, **HYP)
    assert e.gp_fit_ok()
    e.gp_fit(X, y, lengthscale=0.4, wait=False, **HYP)
    assert e.gp_stats() == ref.gp_stats()
    e.gp_fit(X, y, lengthscale=0.4, wait=False, **HYP)
    e.gp_set_precision(64)            # the staged fit was sized at precision 8
    for g, w in zip(_score(e, U), want):
        np.testing.assert_array_equal(g, w)
    e.gp_set_precision(8)
    e.gp_fit(X, y, lengthscale=0.4, wait=False, **HYP)
    e.gp_join_fit()
    for g, w in zip(_score(e, U), want):
        np.testing.assert_array_equal(g, w)
    # duplicate rows, no noise: not positive definite, reported by the status
    Xd = np.repeat(X[:64], 2, axis=0)
    e.gp_fit(Xd, np.repeat(y[:64], 2), lengthscale=0.4, sigma_f2=1.0, sigma_n2=0.0, jitter=0.0, wait=False)
    assert not e.gp_fit_ok()
    e.gp_fit(X, y, lengthscale=0.4, wait=False, **HYP)
    for g, w in zip(_score(e, U), want):
        np.testing.assert_array_equal(g, w)


@pytest.mark.parametrize("prec", [64, 8])
def test_async_fit_round_equals_sync_fit_round(prec):
    """a scoring round after ut_gp_fit_async (its fit issued after the DE
    proposal) selects exactly what the round after a synchronous fit does, and
    a stand-alone proposal issues the staged fit the same way"""
    d, npop, m, k = 12, 400, 5000, 64
    space = [Param(f"u{j}", FLOAT, -5.0, 5.0) for j in range(d)]
    pop = ode.population_init(space, npop, seed=9)
    X = features(space, pop[:, :200]).T
    y = np.sum((X - 0.5) ** 2, axis=1)
    out = []
    for wait in (True, False):
        e = engine(space, seed=9)
        e.gp_set_precision(prec)
        e.population_set(dev(pop))
        e.history_reset(0)
        e.gp_fit(X, y, lengthscale=0.6, wait=wait, **HYP)
        idx, top, dig, _ = e.score_round_de(m, k, round_=3, cand_base=0, cr=0.3)
        e.gp_fit(X, y, lengthscale=0.6, wait=wait, **HYP)
        v = e.propose_de(m, round_=4, cand_base=0)
        _, _, sc = e.gp_score(e.encode(v))
        out.append([t.cpu().numpy() for t in (idx, top, dig, sc)])
    for g, w in zip(*out):
        np.testing.assert_array_equal(g, w)
