"""Full-size rounds of the bench's other two workloads, checked through
size-independent properties and the oracle at the selected indices:

  C3 (BASELINE configs[2] per GPU): the HPL-64 mixed space
     (samples/hpl/hpl.py:44-56 padded to 64 params), m = 2^21 DE-Alt
     candidates, GP n = 4096 -- dense and EI-bound pruned (256 rows);
  C4 (configs[3]): the gcc-options space (339 params,
     samples/gcc-options/tune_gcc.py:259-287), m = 2^22 GA proposals from the
     best recorded config, dedup against the 3,680 recorded configurations.

For the k selected candidates of a round:
  * their values are the oracle's proposals at those global indices
    (differentialevolution.py:105-129 / evolutionarytechniques.py:29-61 as
    restated in oracle/de.py, oracle/ga.py);
  * their digests are the oracle's hash_config (manipulator.py:233-243), and
    none of them is in the recorded history (driver.py:157-158 dedup);
  * their scores are the oracle GP's EI within 1e-5 (fp64);
  * C3: the pruned round selects exactly what the dense round selects, and no
    candidate of a random sample of the others has a larger oracle EI than the
    k-th selected one (a score-determined selection).
"""
import hashlib
import os
import time

import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from _spaces import oracle_space  # noqa: E402
from oracle import de as ode  # noqa: E402
from oracle import ga as oga  # noqa: E402
from oracle import gp as ogp  # noqa: E402
from oracle import hashing as oh  # noqa: E402
from oracle.space import features, from_f64  # noqa: E402

K = 256


def _require_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _hashes(space, vals):
    """oracle hash_config of SoA columns, inner digests memoised per (param, value)"""
    order = sorted(range(len(space)), key=lambda i: space[i].name)
    cache, out = {}, []
    for c in range(vals.shape[1]):
        parts = []
        for i, j in enumerate(order):
            key = (j, vals[j, c])
            hv = cache.get(key)
            if hv is None:
                hv = cache[key] = str(oh.hash_value(space[j], from_f64(space[j], vals[j, c]))).encode()
            parts += [str(space[j].name).encode(), hv, str(i).encode(), b"|"]
        out.append(hashlib.sha256(b"".join(parts)).hexdigest())
    return out


def _check_selection(space, idx, top, dig, vals, want_vals, hist_hex, X, y, ell, jitter):
    from uptune_amd.engine import digests_to_hex
    ii = idx.cpu().numpy()
    assert np.all(ii >= 0) and len(set(ii.tolist())) == len(ii)
    t = top.cpu().numpy()
    assert np.all(np.diff(t) <= 0)
    got = vals.cpu().numpy()
    np.testing.assert_array_equal(got, want_vals)              # the oracle's proposals at those indices
    hx = digests_to_hex(dig)
    assert hx == _hashes(space, want_vals)                     # hash_config
    assert not (set(hx) & hist_hex)                            # none was evaluated before
    g = ogp.GP(X, y, lengthscale=ell, sigma_f2=1.0, sigma_n2=1e-6, jitter=jitter)
    mu, var = g.posterior(features(space, want_vals).T)
    ei = ogp.acquisition(mu, var, g.f_best)
    np.testing.assert_allclose(t, ei, rtol=1e-5, atol=1e-12)
    return g, ei


@pytest.fixture(scope="module")
def c3():
    _require_gpu()
    from uptune_amd import spaces
    from uptune_amd.engine import BatchEngine
    manip = spaces.hpl64()
    space = oracle_space(manip)
    m, n = 1 << 21, 4096
    tr = ode.population_init(space, n, 101)
    X = features(space, tr).T.copy()
    y = np.sum((X - 0.3) ** 2, axis=1)
    hist = _hashes(space, tr)
    e = BatchEngine(manip, device=0, seed=1)
    e.population_init(m)
    e.history_reset(2 * n)
    e.history_add(hist)
    return dict(e=e, space=space, m=m, n=n, X=X, y=y, hist=set(hist))


def test_c3_full_size_round_dense_and_pruned(c3):
    e, space, m = c3["e"], c3["space"], c3["m"]
    t0 = time.time()
    e.gp_fit(c3["X"], c3["y"], lengthscale=1.0, sigma_f2=1.0, sigma_n2=1e-6)
    rnd = 4
    idx, top, dig, vals = e.score_round_de(m, K, round_=rnd, cand_base=0, cr=0.2, n_cross=1, acq=e.acq("ei"))
    pi, pt, pd, pv, st = e.score_round_de_pruned(m, K, round_=rnd, cand_base=0, cr=0.2, n_cross=1,
                                                 acq=e.acq("ei"), bound_rows=256)
    e.sync()
    # pruned = dense, candidate for candidate (selection-exact bound)
    assert pi.cpu().tolist() == idx.cpu().tolist()
    np.testing.assert_array_equal(pt.cpu().numpy(), top.cpu().numpy())
    assert torch.equal(pd, dig) and torch.equal(pv, vals)
    assert 0 < st["survivors"] < m
    want = ode.propose_de_at(space, idx.cpu().numpy(), m, 1, rnd, 0.2, 1)
    g, ei = _check_selection(space, idx, top, dig, vals, want, c3["hist"], c3["X"], c3["y"], 1.0, 0.0)
    # score-determined: a random sample of the others never beats the k-th
    rng = np.random.default_rng(7)
    chosen = set(idx.cpu().tolist())
    samp = np.array([j for j in rng.choice(m, 4096, replace=False) if j not in chosen])
    mu, var = g.posterior(features(space, ode.propose_de_at(space, samp, m, 1, rnd, 0.2, 1)).T)
    ei_s = ogp.acquisition(mu, var, g.f_best)
    assert ei_s.max() <= ei.min() * (1 + 1e-5)
    assert len(np.unique(top.cpu().numpy())) == K              # distinct scores decide the order
    print(f"C3 full-size round: {time.time() - t0:.1f} s, survivors {st['survivors']}")


@pytest.fixture(scope="module")
def c4(golden_dir):
    _require_gpu()
    from uptune_amd import spaces
    from uptune_amd.engine import BatchEngine
    manip = spaces.gcc()
    space = oracle_space(manip)
    z = np.load(os.path.join(golden_dir, "gcc_history.npz"))
    hist, qor = z["values"], z["qor"]
    e = BatchEngine(manip, device=0, seed=44)
    e.history_reset(0)
    e.history_add(e.hash(torch.from_numpy(np.ascontiguousarray(hist)).cuda()))
    ok_rows = np.flatnonzero(np.isfinite(qor))[:1024]
    X = features(space, hist[:, ok_rows]).T.copy()
    y = qor[ok_rows].astype(np.float64)
    return dict(e=e, space=space, hist=hist, X=X, y=y, best=hist[:, int(np.argmin(qor))].copy(),
                hist_hex=set(_hashes(space, hist)))


def test_c4_full_size_ga_round(c4):
    """the bench's C4 step at m = 2^22: GA mutation 0.1 from the best recorded
    config -> ut_hash_parent -> dedup -> ut_gp_score_values -> top-k"""
    e, space = c4["e"], c4["space"]
    m, rnd, base = 1 << 22, 6, 0
    t0 = time.time()
    e.gp_fit(c4["X"], c4["y"], lengthscale=2.0, sigma_f2=1.0, sigma_n2=1e-6, jitter=1e-8)
    vals, invalid = e.propose_ga(m, parent1=c4["best"], round_=rnd, cand_base=base, mutation_rate=0.1)
    dig = e.hash_parent(vals, c4["best"])
    dup = torch.maximum(e.dedup(dig), invalid)
    _, _, score = e.gp_score_values(vals, acq=e.acq("ei"), dup=dup)
    idx, top = e.topk(score, K, dup=dup, cand_base=base)
    loc = idx - base
    sel_vals, sel_dig = vals[:, loc].contiguous(), dig[loc].contiguous()
    assert int(invalid[loc].sum()) == 0 and int(dup[loc].sum()) == 0
    n_dup = int(dup.sum())
    want, winv = oga.propose_ga_vec(space, c4["best"], None, 44, rnd, 0, 0, mutation_rate=0.1,
                                    g=idx.cpu().numpy())
    assert not winv.any()
    _check_selection(space, idx, top, sel_dig, sel_vals, want, c4["hist_hex"], c4["X"], c4["y"], 2.0, 1e-8)
    print(f"C4 full-size round: {time.time() - t0:.1f} s, {n_dup} duplicates / invalid of {m}")
