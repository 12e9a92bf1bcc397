"""The fp64 tier on the int8 MFMA (ut_gp_set_precision(ctx, 8); gp_i8.hip).

The variance contraction |L^-1 k*|^2 runs over six balanced 8-bit digit planes
of L^-1 and K* with exact int32 group sums; every candidate's variance error
is bounded from the digits' truncation (E (2 |v^| + E), E = the fit's bound on
|L^-1 k* - v^|), and candidates whose bound exceeds the tolerance are
recomputed on the fp64 path.  These tests hold the tier to the fp64 tier's
1e-5 parity (the oracle) and check that the bound is a bound, that tol = 0 is
the fp64 path bit for bit, and that a round selects what the fp64 round does.
Needs a GPU."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

from oracle import de as ode  # noqa: E402
from oracle import gp as ogp  # noqa: E402
from oracle.space import FLOAT, Param, features  # noqa: E402

RTOL, ATOL = 1e-5, 1e-9


def _engine(space, seed=0):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from _spaces import to_manip
    from uptune_amd.engine import BatchEngine
    return BatchEngine(to_manip(space), device=0, seed=seed)


def _dev(a):
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def _problem(n, d, ell, m, seed, near=10, sf2=1.0):
    rng = np.random.default_rng(seed)
    X = rng.uniform(size=(n, d))
    y = np.sum((X - 0.4) ** 2, axis=1) + 0.01 * rng.standard_normal(n)
    U = rng.uniform(size=(m, d))
    U[:near] = X[:near] + 1e-3
    return [Param(f"u{k}", FLOAT, 0.0, 1.0) for k in range(d)], X, y, U


def _score(space, X, y, U, ell, prec, tol=None, sf2=1.0, sn2=1e-6):
    e = _engine(space)
    e.gp_set_precision(prec)
    if tol is not None:
        e.gp_set_i8_tol(tol)
    e.gp_fit(X, y, lengthscale=ell, sigma_f2=sf2, sigma_n2=sn2, jitter=1e-8)
    out = [t.cpu().numpy() for t in e.gp_score(_dev(U.T), acq=e.acq("ei"))]
    stats = e.gp_i8_stats() + (e.gp_i8_bounds()[1],) if prec == 8 else None
    e.close()
    return out, stats


@pytest.mark.parametrize("n,d,ell,sf2", [(1024, 64, 2.0, 1.0), (300, 16, 1.5, 1.0), (77, 3, 0.25, 1.0),
                                         (500, 6, 0.6, 37.0), (2000, 24, 0.8, 1e-3)])
def test_i8_bound_holds(n, d, ell, sf2):
    """with tol near 1 nothing is recomputed (except var ~ 0), so the returned
    variances and means are the int8 contraction's own: each variance is within
    the bound E (2 |v| + E) + rounding of the fp64 path's, each mean (v^ . L^-1 y
    from the int8 epilogue) within Emu + rounding of the fp64 path's, and the
    variances are within 1e-5 of the oracle wherever the default tolerance
    would have accepted them"""
    space, X, y, U = _problem(n, d, ell, 4000, n + d)
    (mu8, var8, _), (rec, E, Emu) = _score(space, X, y, U, ell, 8, tol=0.999, sf2=sf2)
    (mu64, var64, _), _ = _score(space, X, y, U, ell, 64, sf2=sf2)
    assert E > 0.0 and Emu > 0.0 and rec >= 0
    v2 = np.maximum(sf2 - var64, 0.0)
    bound = E * (2 * np.sqrt(v2) + E) + 1e-13 * sf2
    assert np.all(np.abs(var8 - var64) <= bound), float(np.max(np.abs(var8 - var64) / bound))
    mbound = Emu + 1e-12 * np.maximum(1.0, np.abs(mu64))
    assert np.all(np.abs(mu8 - mu64) <= mbound), float(np.max(np.abs(mu8 - mu64) / mbound))
    ok = bound <= 2.0 ** -20 * var64
    g = ogp.GP(X, y, lengthscale=ell, sigma_f2=sf2, sigma_n2=1e-6, jitter=1e-8)
    mu_o, var_o = g.posterior(U)
    np.testing.assert_allclose(var8[ok], var_o[ok], rtol=RTOL, atol=1e-8 * sf2)


def test_i8_tol0_is_the_fp64_path():
    """tol = 0: every candidate is recomputed (the round falls back to the whole
    fp64 contraction) -- the variance is the fp64 path's bit for bit and the
    mean its (L^-1 k*) . (L^-1 y) from the same epilogue"""
    space, X, y, U = _problem(700, 20, 0.7, 3000, 5)
    (mu8, var8, ei8), (rec, _, _) = _score(space, X, y, U, 0.7, 8, tol=0.0)
    (mu64, var64, ei64), _ = _score(space, X, y, U, 0.7, 64)
    assert rec == -1
    np.testing.assert_array_equal(var8, var64)
    np.testing.assert_allclose(mu8, mu64, rtol=1e-10, atol=1e-12)
    np.testing.assert_allclose(ei8, ei64, rtol=1e-10, atol=1e-12)


@pytest.mark.parametrize("n,d,ell,near", [(1024, 64, 0.2, 10), (1024, 64, 2.0, 40), (200, 8, 0.5, 25),
                                          (4096, 112, 1.0, 10)])
def test_i8_recompute_near_training_points(n, d, ell, near):
    """the default tolerance recomputes a few candidates (those next to training
    points, where sf2 - |v|^2 cancels) and the result is the fp64 tier's: the
    oracle within 1e-5"""
    space, X, y, U = _problem(n, d, ell, 6000, 3 * n + d, near=near)
    (mu8, var8, ei8), (rec, _, _) = _score(space, X, y, U, ell, 8)
    assert 0 <= rec <= 3000
    g = ogp.GP(X, y, lengthscale=ell, sigma_f2=1.0, sigma_n2=1e-6, jitter=1e-8)
    mu_o, var_o = g.posterior(U)
    ei_o = ogp.acquisition(mu_o, var_o, g.f_best)
    np.testing.assert_allclose(mu8, mu_o, rtol=RTOL, atol=ATOL)
    np.testing.assert_allclose(var8, var_o, rtol=RTOL, atol=1e-8)
    np.testing.assert_allclose(ei8, ei_o, rtol=RTOL, atol=1e-8)


def test_i8_round_selects_as_fp64():
    """a whole DE round (propose, hash, dedup, encode, K*, variance, EI, top-k) at
    precision 8 selects the fp64 round's candidates with the same scores, on a
    score-determined GP (ell = 2 in the 64-cube: every k* ~ 0.3)"""
    space = [Param(str(k), FLOAT, -1000.0, 1000.0) for k in range(64)]
    pop = ode.population_init(space, 1 << 15, seed=21)
    X = features(space, pop[:, :1024]).T
    y = np.sum((X - 0.5) ** 2, axis=1)
    res = {}
    for prec in (64, 8):
        e = _engine(space, seed=21)
        e.population_set(_dev(pop))
        e.gp_set_precision(prec)
        e.gp_fit(X, y, lengthscale=2.0, sigma_f2=1.0, sigma_n2=1e-6, jitter=1e-8)
        e.history_reset(0)
        idx, top, dig, _ = e.score_round_de(1 << 15, 64, round_=2, cand_base=0)
        res[prec] = (idx.cpu().numpy(), top.cpu().numpy())
        if prec == 8:
            rec, _ = e.gp_i8_stats()
            assert 0 <= rec < 100
        e.close()
    np.testing.assert_allclose(res[8][1], res[64][1], rtol=1e-7, atol=1e-12)
    s = res[64][1]
    assert np.abs(np.diff(s)).min() > 1e-6 * np.abs(s).max()   # distinct: the selection is by score
    assert res[8][0].tolist() == res[64][0].tolist()


def test_i8_rejects_too_many_training_points():
    """exact int32 digit sums need K * 6 * 2^14 < 2^31: the fit refuses n > 16384"""
    space, X, y, U = _problem(16500, 2, 0.5, 100, 1, near=0)
    e = _engine(space)
    e.gp_set_precision(8)
    from uptune_amd._lib import UthotError
    with pytest.raises(UthotError, match="16384"):
        e.gp_fit(X, y, lengthscale=0.5, sigma_f2=1.0, sigma_n2=1e-2, jitter=1e-8)
    e.close()
