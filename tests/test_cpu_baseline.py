"""The batch CPU baseline B1 (oracle/cpu_batch.*: C++/OpenMP DE + hash_config +
dedup, BLAS GP) computes exactly what the per-candidate oracle computes, so
the throughput bench.py reports for it is for the same work."""
import numpy as np
import pytest

from oracle import cpu_batch as cb
from oracle import de as ode
from oracle import gp as ogp
from oracle import hashing as oh
from oracle import select as osel
from oracle.space import FLOAT, Param


@pytest.fixture(scope="module", autouse=True)
def _built():
    cb.build()


@pytest.mark.parametrize("names", ["ints", "strs"])
def test_de_hash_matches_oracle(names):
    P = 64 if names == "ints" else 7
    space = [Param(i if names == "ints" else "p%d_%s" % (i, "xyz"[i % 3]), FLOAT, -1000.0 + i, 1000.0 - 3 * i)
             for i in range(P)]
    pop = ode.population_init(space, 300, seed=4)
    trial, dig = cb.de_hash_float(space, pop, 9, 2, 11, 500, 0.2, 1)
    np.testing.assert_array_equal(trial, ode.propose_de_vec(space, pop, 9, 2, 11, 500, 0.2, 1))
    want = [oh.hash_config(space, list(trial[:, j])) for j in range(trial.shape[1])]
    assert [bytes(d).hex() for d in dig] == want


def test_dedup_and_topk_match_oracle():
    rng = np.random.default_rng(2)
    dig = rng.integers(0, 4, size=(3000, 32), dtype=np.uint8)        # many repeats
    hist = dig[100:130].copy()
    hx = [bytes(d).hex() for d in dig]
    assert cb.dedup(dig, hist).tolist() == osel.dedup(hx, {bytes(h).hex() for h in hist})
    s = np.round(rng.normal(size=5000), 1)                            # ties
    s[::7] = -np.inf
    s[3] = np.nan
    want = [i for i in osel.topk(list(s), 100) if i >= 0 and np.isfinite(s[i])]
    assert cb.topk(s, 100).tolist() == want


def test_c2_round_selection_matches_oracle():
    space = [Param(i, FLOAT, -1000.0, 1000.0) for i in range(16)]
    pop = ode.population_init(space, 2048, seed=1)
    rng = np.random.default_rng(4)
    X = rng.uniform(size=(200, 16))
    y = np.sum((X - 0.4) ** 2, axis=1)
    gp = ogp.GP(X, y, lengthscale=0.5)
    sel, trial, dig, dup, ei = cb.c2_round(space, pop, gp, 1, 3, 2048, 32)
    want_t = ode.propose_de_vec(space, pop, 1, 3, 0, 2048, 0.2, 1)
    np.testing.assert_array_equal(trial, want_t)
    from oracle.space import features
    mu, var = gp.posterior(features(space, want_t).T)
    wei = ogp.acquisition(mu, var, gp.f_best)
    np.testing.assert_allclose(ei, wei, rtol=1e-9, atol=1e-12)
    assert sel.tolist() == osel.topk(list(wei), 32)
