"""The fit's device work replayed from captured hipGraphs (gp_fit_enqueue).

A fit whose shapes, path, hyperparameters and buffers repeat the previous
fit's is captured (two graphs, split where fp64 K* may start) and replayed
while that holds; the replay reads the newly staged X and y.  These tests
check that a replayed fit scores bit for bit as a fit launched kernel by kernel
(UT_FIT_GRAPH=0) on the same data, for every scoring precision, a categorical
space, the asynchronous fit, and that a changed signature falls back to direct
launches and re-captures.  Needs a GPU."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

from oracle import de as ode  # noqa: E402
from oracle.space import BOOL, ENUM, FLOAT, INT, Param, features  # noqa: E402


def _engine(space, seed=0):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from _spaces import to_manip
    from uptune_amd.engine import BatchEngine
    return BatchEngine(to_manip(space), device=0, seed=seed)


def _space(kind):
    if kind == "float":
        return [Param(f"u{k}", FLOAT, 0.0, 1.0) for k in range(12)]
    return [Param("x", FLOAT, -5.0, 5.0), Param("n", INT, 1, 64), Param("flag", BOOL),
            Param("mode", ENUM, options=["a", "b", "c", 4]), Param("y", FLOAT, 0.0, 1.0)]


def _data(space, n, seed):
    X = features(space, ode.population_init(space, n, seed=seed)).T
    y = np.sum((X - 0.35) ** 2, axis=1) + 0.01 * np.random.default_rng(seed).standard_normal(n)
    return X, y


def _score(e, space, cand):
    vals = torch.from_numpy(np.ascontiguousarray(cand)).cuda()
    return [t.cpu().numpy() for t in e.gp_score_values(vals, acq=e.acq("ei"))]


def _fit(e, X, y, wait=True):
    e.gp_fit(X, y, lengthscale=0.8, sigma_f2=1.0, sigma_n2=1e-6, jitter=1e-8, wait=wait)


@pytest.mark.parametrize("kind", ["float", "mixed"])
@pytest.mark.parametrize("prec", [64, 32, 16, 8])
def test_replayed_fit_equals_direct_fit(kind, prec, monkeypatch):
    space = _space(kind)
    A, B = _data(space, 1000, 1), _data(space, 1000, 2)
    cand = ode.population_init(space, 6000, seed=3)
    e = _engine(space)
    e.gp_set_precision(prec)
    _fit(e, *A)
    _fit(e, *A)
    _fit(e, *B, wait=False)           # replayed, asynchronous: the round scores behind it
    assert e.gp_fit_graph_stats() == (1, 1, 1)
    got = _score(e, space, cand)
    monkeypatch.setenv("UT_FIT_GRAPH", "0")
    f = _engine(space)
    f.gp_set_precision(prec)
    _fit(f, *B)
    assert f.gp_fit_graph_stats() == (1, 0, 0)
    want = _score(f, space, cand)
    for g, w in zip(got, want):
        np.testing.assert_array_equal(g, w)
    e.close()
    f.close()


def test_signature_change_falls_back_and_recaptures(monkeypatch):
    space = _space("float")
    A, B = _data(space, 1000, 1), _data(space, 1000, 2)
    C, D = _data(space, 700, 4), _data(space, 700, 5)
    cand = ode.population_init(space, 3000, seed=3)
    e = _engine(space)
    _fit(e, *A)
    _fit(e, *B)                      # captured
    _fit(e, *C)                      # new padded size: direct
    assert e.gp_fit_graph_stats() == (2, 1, 0)
    _fit(e, *D)                      # C's signature again: captured (replaces A's graphs)
    _fit(e, *C)                      # replayed
    assert e.gp_fit_graph_stats() == (2, 2, 1)
    got_c = _score(e, space, cand)
    _fit(e, *A)                      # a new padded size again: direct
    e.gp_fit(*B, lengthscale=0.5, sigma_f2=1.0, sigma_n2=1e-6, jitter=1e-8)   # captured (1 / ell is staged data)
    e.gp_fit(*A, lengthscale=0.3, sigma_f2=1.0, sigma_n2=1e-6, jitter=1e-8)   # replayed with a new lengthscale
    assert e.gp_fit_graph_stats() == (3, 3, 2)
    got_a = _score(e, space, cand)
    e.gp_fit(*B, lengthscale=0.3, sigma_f2=2.0, sigma_n2=1e-6, jitter=1e-8)   # sigma_f2 is a kernel argument: direct
    assert e.gp_fit_graph_stats() == (4, 3, 2)
    got_b = _score(e, space, cand)
    monkeypatch.setenv("UT_FIT_GRAPH", "0")
    f = _engine(space)
    want = []
    for (X, y), ell, sf2 in ((C, 0.8, 1.0), (A, 0.3, 1.0), (B, 0.3, 2.0)):
        f.gp_fit(X, y, lengthscale=ell, sigma_f2=sf2, sigma_n2=1e-6, jitter=1e-8)
        want += _score(f, space, cand)
    for g, w in zip(got_c + got_a + got_b, want):
        np.testing.assert_array_equal(g, w)
    e.close()
    f.close()
