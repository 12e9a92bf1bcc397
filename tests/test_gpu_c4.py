"""C4 (BASELINE.json configs[3]): the gcc-options space -- 339 params: -O in
[0, 3], 184 flags {on, off, default}, 154 --params with the integer ranges
tune_gcc.py:264-282 derives from samples/gcc-options/params.def
(tests/golden/make_golden.py params_def_ranges) -- under GA and PSO proposal
rounds, with dedup against ALL 3,680 recorded configurations of
samples/gcc-options/matmul-record.csv (tests/golden/gcc_history.npz).

Bit-exact vs the oracle: proposed values, invalid masks, hash_config digests
(also of the 3,680 recorded configs), dedup masks; GP-EI on the recorded qor
within 1e-5 and the selected top-k equal to the oracle's.
"""
import hashlib
import os

import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from _spaces import oracle_space  # noqa: E402
from oracle import ga as oga  # noqa: E402
from oracle import gp as ogp  # noqa: E402
from oracle import hashing as oh  # noqa: E402
from oracle import pso as opso  # noqa: E402
from oracle import select as osel  # noqa: E402
from oracle.space import features, from_f64  # noqa: E402

M = 20000


def _require_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


class _Hasher:
    """oracle hash_config with the inner digests memoised per (param, value):
    hash_value depends on the value alone (manipulator.py:456-459, :855-858)"""

    def __init__(self, space):
        self.space = space
        self.order = sorted(range(len(space)), key=lambda i: space[i].name)
        self.names = [str(space[j].name).encode() for j in self.order]
        self.cache = {}

    def __call__(self, vals):
        out = []
        for c in range(vals.shape[1]):
            col = vals[:, c]
            parts = []
            for i, j in enumerate(self.order):
                key = (j, col[j])
                hv = self.cache.get(key)
                if hv is None:
                    hv = str(oh.hash_value(self.space[j], from_f64(self.space[j], col[j]))).encode()
                    self.cache[key] = hv
                parts += [self.names[i], hv, str(i).encode(), b"|"]
            out.append(hashlib.sha256(b"".join(parts)).hexdigest())
        return out


@pytest.fixture(scope="module")
def c4(golden_dir):
    _require_gpu()
    from uptune_amd import spaces
    from uptune_amd.engine import BatchEngine, digests_to_hex
    manip = spaces.gcc()
    space = oracle_space(manip)
    z = np.load(os.path.join(golden_dir, "gcc_history.npz"))
    hist, qor = z["values"], z["qor"]
    # the params.def ranges (not recorded min..max): e.g. -O [0, 3], align-threshold [25, 400]
    rng = {p.name: (p.lo, p.hi) for p in space}
    assert rng["-O"] == (0, 3) and rng["align-threshold"] == (25, 400) and rng["l1-cache-line-size"] == (2, 8)
    assert sum(1 for p in space if p.kind == 5) == 184 and len(space) == 339
    e = BatchEngine(manip, device=0, seed=44)
    H = _Hasher(space)
    hv = torch.from_numpy(np.ascontiguousarray(hist)).cuda()
    hd = e.hash(hv)
    hist_hex = H(hist)
    assert digests_to_hex(hd) == hist_hex           # all 3,680 recorded configs
    e.history_reset(0)
    e.history_add(hd)
    best = int(np.argmin(qor))
    return dict(e=e, space=space, hist=hist, qor=qor, H=H, hist_hex=set(hist_hex), best=hist[:, best].copy(),
                second=hist[:, int(np.argsort(qor)[1])].copy())


def _score_and_check(c4, vals, dup, k=64):
    """device GP-EI on the recorded qor vs the oracle; top-k equality"""
    e, space = c4["e"], c4["space"]
    n = 1024
    ok_rows = np.flatnonzero(np.isfinite(c4["qor"]))[:n]   # 149 recorded runs failed (qor = inf)
    X = features(space, c4["hist"][:, ok_rows]).T
    y = c4["qor"][ok_rows].astype(np.float64)
    e.gp_fit(X, y, lengthscale=2.0, sigma_f2=1.0, sigma_n2=1e-6, jitter=1e-8)
    feat = e.encode(torch.from_numpy(np.ascontiguousarray(vals)).cuda())
    np.testing.assert_array_equal(feat.cpu().numpy(), features(space, vals))
    dupt = torch.from_numpy(np.asarray(dup, dtype=np.uint8)).cuda()
    mu, var, score = e.gp_score(feat, acq=e.acq("ei"), dup=dupt)
    g = ogp.GP(X, y, lengthscale=2.0, sigma_f2=1.0, sigma_n2=1e-6, jitter=1e-8)
    wmu, wvar = g.posterior(features(space, vals).T)
    ei = ogp.acquisition(wmu, wvar, g.f_best)
    np.testing.assert_allclose(mu.cpu().numpy(), wmu, rtol=1e-5, atol=1e-9)
    np.testing.assert_allclose(var.cpu().numpy(), wvar, rtol=1e-5, atol=1e-9)
    ok = np.asarray(dup) == 0
    np.testing.assert_allclose(score.cpu().numpy()[ok], ei[ok], rtol=1e-5, atol=1e-9)
    idx, top = e.topk(score, k, dup=dupt)
    want = osel.topk(list(np.where(ok, ei, -np.inf)), k, dup=list(dup))
    s = np.sort(ei[ok])[::-1][:k + 1]
    if np.abs(np.diff(s)).min() > 1e-6 * max(1.0, abs(s).max()):      # distinct scores: exact selection
        assert idx.cpu().numpy().tolist() == want


@pytest.mark.parametrize("mutation_rate,crossover_rate,two", [(0.01, 0.5, False), (0.05, 0.8, True),
                                                              (0.1, 0.8, False)])
def test_c4_ga_round(c4, mutation_rate, crossover_rate, two):
    """UniformGreedyMutation / GA(crossover_rate) from the best recorded config
    (GreedySelectionMixin.select; evolutionarytechniques.py:29-61,:72-96)"""
    e, space = c4["e"], c4["space"]
    p2 = c4["second"] if two else None
    vals, inv = e.propose_ga(M, parent1=c4["best"], parent2=p2, round_=3, cand_base=17,
                             mutation_rate=mutation_rate, crossover_rate=crossover_rate)
    wv, winv = oga.propose_ga_vec(space, c4["best"], p2, 44, 3, 17, M, mutation_rate=mutation_rate,
                                  crossover_rate=crossover_rate)
    np.testing.assert_array_equal(vals.cpu().numpy(), wv)
    np.testing.assert_array_equal(inv.cpu().numpy().astype(bool), winv)
    from uptune_amd.engine import digests_to_hex
    # the batch also carries 512 recorded configs (they must come out as
    # duplicates of the history) and repeats of its own first 64 proposals
    pick = np.random.default_rng(1).choice(c4["hist"].shape[1], 512, replace=False)
    allv = np.ascontiguousarray(np.concatenate([wv, c4["hist"][:, pick], wv[:, :64]], axis=1))
    dig = e.hash(torch.from_numpy(allv).cuda())
    hx = digests_to_hex(dig)
    assert hx == c4["H"](allv)
    # the bench's C4 step hashes through ut_hash_parent (parent1's inner digests reused)
    assert digests_to_hex(e.hash_parent(torch.from_numpy(allv).cuda(), c4["best"])) == hx
    dup = e.dedup(dig)
    wdup = osel.dedup(hx, c4["hist_hex"])
    assert dup.cpu().numpy().tolist() == wdup
    assert all(wdup[M:])                                 # recorded configs + in-batch repeats
    full = np.maximum(np.asarray(wdup), np.concatenate([winv, np.ones(576, dtype=bool)]).astype(np.int64))
    _score_and_check(c4, allv, full)


@pytest.mark.parametrize("two", [False, True])
def test_score_round_ga_equals_separate_calls(c4, two):
    """ut_score_round_ga (the bench's C4 step: hash + dedup on a second stream
    beside encode + GP) selects what the separate calls select -- propose_ga,
    hash_parent, dedup with the invalid children, gp_score_values, topk -- with
    the same scores and digests, and its selections' digests are the oracle's"""
    e, space = c4["e"], c4["space"]
    n, k, m = 1024, 64, 50000
    ok_rows = np.flatnonzero(np.isfinite(c4["qor"]))[:n]
    X = features(space, c4["hist"][:, ok_rows]).T
    y = c4["qor"][ok_rows].astype(np.float64)
    p2 = c4["second"] if two else None
    kw = dict(mutation_rate=0.05, crossover_rate=0.5 if two else 0.0)
    e.gp_fit(X, y, lengthscale=2.0, sigma_f2=1.0, sigma_n2=1e-6, jitter=1e-8)
    acq = e.acq("ei")
    idx, top, dig, vals = e.score_round_ga(m, k, parent1=c4["best"], parent2=p2, round_=5, cand_base=100, acq=acq,
                                           **kw)
    v2, inv = e.propose_ga(m, parent1=c4["best"], parent2=p2, round_=5, cand_base=100, **kw)
    d2 = e.hash_parent(v2, c4["best"])
    dup = torch.maximum(e.dedup(d2), inv)
    _, _, score = e.gp_score_values(v2, acq=acq, dup=dup)
    i2, t2 = e.topk(score, k, dup=dup, cand_base=100)
    assert idx.cpu().tolist() == i2.cpu().tolist()
    np.testing.assert_array_equal(top.cpu().numpy(), t2.cpu().numpy())
    sel = (i2 - 100).cpu().numpy()
    np.testing.assert_array_equal(dig.cpu().numpy(), d2[sel].cpu().numpy())
    np.testing.assert_array_equal(vals.cpu().numpy(), v2[:, sel].cpu().numpy())
    from uptune_amd.engine import digests_to_hex
    assert digests_to_hex(dig) == c4["H"](vals.cpu().numpy())


def test_c4_pso_round(c4):
    """PSO (pso.py:23-77) over a swarm of recorded configs toward the best one;
    Enum flags keep the reference quirk (enum_mode 0: never move)"""
    e, space = c4["e"], c4["space"]
    npop = 3680
    pop = np.ascontiguousarray(c4["hist"])
    e.population_set(torch.from_numpy(pop).cuda())
    e.pso_reset()
    x, v = e.propose_pso(c4["best"], npop, round_=2)
    wx, wv = opso.propose_pso_vec(space, pop, np.zeros_like(pop), pop, c4["best"], 44, 2, 0, npop)
    np.testing.assert_array_equal(x.cpu().numpy(), wx)
    np.testing.assert_array_equal(v.cpu().numpy(), wv)
    from uptune_amd.engine import digests_to_hex
    dig = e.hash(x)
    hx = digests_to_hex(dig)
    assert hx == c4["H"](wx)
    dup = e.dedup(dig).cpu().numpy().tolist()
    assert dup == osel.dedup(hx, c4["hist_hex"])
    _score_and_check(c4, wx, dup, k=32)


def test_c4_second_history_raytracer(c4, golden_dir):
    """the second recorded history of the same space
    (samples/gcc-options/raytracer-record.csv, 2,269 configs:
    tests/golden/gcc_raytracer_history.npz): every recorded config hashes on
    the device as the oracle hashes it (the committed oracle digests of its
    first rows too); deduplicated against the matmul history the mask is the
    oracle's set membership; then both histories together are the dedup set
    of a GA round from the raytracer's best config, scored by a GP on the
    raytracer's recorded qor"""
    e, space, H = c4["e"], c4["space"], c4["H"]
    from uptune_amd.engine import digests_to_hex
    z = np.load(os.path.join(golden_dir, "gcc_raytracer_history.npz"))
    rv, rq = z["values"], z["qor"]
    assert rv.shape == (339, 2269)
    dig = e.hash(torch.from_numpy(np.ascontiguousarray(rv)).cuda())
    hx = digests_to_hex(dig)
    assert hx[:len(z["hashes_py3"])] == list(z["hashes_py3"])
    assert hx == H(rv)
    dup = e.dedup(dig).cpu().numpy().tolist()
    assert dup == osel.dedup(hx, c4["hist_hex"])      # matmul history + repeats inside the raytracer record
    # a fresh engine: both recorded histories are the dedup set
    from uptune_amd import spaces
    from uptune_amd.engine import BatchEngine
    e2 = BatchEngine(spaces.gcc(), device=0, seed=45)
    e2.history_reset(0)
    e2.history_add(e.hash(torch.from_numpy(np.ascontiguousarray(c4["hist"])).cuda()))
    e2.history_add(dig)
    best = rv[:, int(np.argmin(rq))].copy()
    vals, inv = e2.propose_ga(M, parent1=best, round_=5, cand_base=3, mutation_rate=0.05)
    wv, winv = oga.propose_ga_vec(space, best, None, 45, 5, 3, M, mutation_rate=0.05)
    np.testing.assert_array_equal(vals.cpu().numpy(), wv)
    np.testing.assert_array_equal(inv.cpu().numpy().astype(bool), winv)
    allv = np.ascontiguousarray(np.concatenate([wv, rv[:, :100], c4["hist"][:, :100]], axis=1))
    d2 = e2.hash_parent(torch.from_numpy(allv).cuda(), best)
    h2 = digests_to_hex(d2)
    assert h2 == H(allv)
    m2 = e2.dedup(d2).cpu().numpy().tolist()
    assert m2 == osel.dedup(h2, c4["hist_hex"] | set(hx))
    assert all(m2[M:])
    ok = np.flatnonzero(np.isfinite(rq))[:1024]
    X = features(space, rv[:, ok]).T
    y = rq[ok].astype(np.float64)
    e2.gp_fit(X, y, lengthscale=2.0, sigma_f2=1.0, sigma_n2=1e-6, jitter=1e-8)
    mu, var, score = e2.gp_score_values(torch.from_numpy(allv).cuda(), acq=e2.acq("ei"),
                                        dup=torch.tensor(m2, dtype=torch.uint8, device="cuda"))
    g = ogp.GP(X, y, lengthscale=2.0, sigma_f2=1.0, sigma_n2=1e-6, jitter=1e-8)
    wmu, wvar = g.posterior(features(space, allv).T)
    np.testing.assert_allclose(mu.cpu().numpy(), wmu, rtol=1e-5, atol=1e-9)
    np.testing.assert_allclose(var.cpu().numpy(), wvar, rtol=1e-5, atol=1e-9)
    e2.close()
