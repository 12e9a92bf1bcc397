"""Device path (libuthot.so through the C ABI) vs the oracle.  Needs a GPU.

Tolerances: bit-exact for values, digests, dedup masks and selected
indices; GP mu / var / EI within 1e-5 relative (fp64 path, BASELINE.json
north_star) with an absolute floor of 1e-9 for quantities that are ~0.
"""
import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

from oracle import de as ode  # noqa: E402
from oracle import gp as ogp  # noqa: E402
from oracle import hashing as oh  # noqa: E402
from oracle import select as osel  # noqa: E402
from oracle.space import BOOL, ENUM, FLOAT, INT, Param, features, from_f64  # noqa: E402

RTOL = 1e-5
ATOL = 1e-9


def _require_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


from _spaces import oracle_space, to_manip  # noqa: E402


def engine(space, seed=0, py2=False):
    _require_gpu()
    from uptune_amd.engine import BatchEngine
    return BatchEngine(to_manip(space), device=0, seed=seed, py2_layout=py2)


def dev(a):
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def hexes(d):
    from uptune_amd.engine import digests_to_hex
    return digests_to_hex(d)


def mixed_space():
    return [Param("x", FLOAT, -5.0, 5.0), Param("n", INT, 1, 64), Param("flag", BOOL),
            Param("mode", ENUM, options=["a", "b", "c", 4]), Param("y", FLOAT, 0.0, 1.0),
            Param("big", INT, -100000, 2000000)]


def r64_space():
    return [Param(d, FLOAT, -1000.0, 1000.0) for d in range(64)]


def oracle_hashes(space, vals):
    return [oh.hash_config(space, [from_f64(p, vals[i, j]) for i, p in enumerate(space)])
            for j in range(vals.shape[1])]


# --------------------------------------------------------------------------- hash
def test_hash_tutorial_db_py2(golden_dir):
    d = json.load(open(os.path.join(golden_dir, "tutorial_db_hashes.json")))
    space = [Param("BLOCK_SIZE", INT, 1, 10)]
    e = engine(space, py2=True)
    vals = np.array([[float(r["BLOCK_SIZE"]) for r in d["rows"]]])
    got = hexes(e.hash(dev(vals)))
    assert got == [r["hash"] for r in d["rows"]]


def test_hash_r64_golden_and_random(golden_dir):
    z = np.load(os.path.join(golden_dir, "r64_hashes.npz"))
    e = engine(r64_space())
    assert e.space_info()[:2] == (4588, 72)
    assert hexes(e.hash(dev(z["values"]))) == list(z["hashes"])
    rng = np.random.default_rng(5)
    vals = rng.uniform(-1000, 1000, size=(64, 2000))
    vals[:, :50] = np.round(vals[:, :50], rng.integers(0, 6))  # short reprs
    vals[3, 60:80] = rng.uniform(-1e-4, 1e-4, 20)               # exponent form
    assert hexes(e.hash(dev(vals))) == oracle_hashes(r64_space(), vals)


def test_hash_gcc_space(golden_dir):
    d = json.load(open(os.path.join(golden_dir, "gcc_space.json")))
    vals = np.load(os.path.join(golden_dir, "gcc_rows.npz"))["values"]
    space = []
    for ptype, name, rng in d["params"]:
        space.append(Param(name, ENUM, options=list(rng)) if ptype == "EnumParameter" else
                     Param(name, INT, rng[0], rng[1]))
    e = engine(space)
    assert e.space_info()[:2] == (30178, 472)
    got = hexes(e.hash(dev(vals)))
    assert got[:64] == d["hashes_py3"]
    assert got == oracle_hashes(space, vals)


def test_hash_mixed_and_py2():
    space = mixed_space()
    pop = ode.population_init(space, 3000, seed=3)
    for py2 in (False, True):
        e = engine(space, py2=py2)
        got = hexes(e.hash(dev(pop)))
        want = [oh.hash_config(space, [from_f64(p, pop[i, j]) for i, p in enumerate(space)], py2=py2)
                for j in range(pop.shape[1])]
        assert got == want


# --------------------------------------------------------------------------- proposal
def test_population_init_matches_oracle():
    space = mixed_space()
    e = engine(space, seed=11)
    e.population_init(1000, round_=2)
    got = e.population_get().cpu().numpy()
    np.testing.assert_array_equal(got, ode.population_init(space, 1000, seed=11, round_=2))


@pytest.mark.parametrize("cr,n_cross", [(0.5, 1), (0.2, 1), (0.9, 2), (0.0, 0)])
def test_de_matches_oracle(cr, n_cross):
    space = mixed_space()
    e = engine(space, seed=21)
    pop = ode.population_init(space, 257, seed=4)
    e.population_set(dev(pop))
    got = e.propose_de(4000, round_=7, cand_base=123, cr=cr, n_cross=n_cross).cpu().numpy()
    want = ode.propose_de_vec(space, pop, seed=21, round_=7, cand_base=123, m=4000, cr=cr, n_cross=n_cross)
    np.testing.assert_array_equal(got, want)


@pytest.mark.parametrize("npop,share", [(30, 1), (30, 0), (4, 3), (257, 2)])
def test_de_information_sharing_matches_oracle(npop, share):
    """donor pool = population - {target} + [best] * information_sharing
    (differentialevolution.py:110-118), the reference's 30-member population
    included; the best row is a device row passed per call"""
    space = mixed_space()
    e = engine(space, seed=22)
    pop = ode.population_init(space, npop, seed=5)
    best = ode.population_init(space, 1, seed=77)[:, 0]
    e.population_set(dev(pop))
    got = e.propose_de(3000, round_=2, cand_base=9, cr=0.5, n_cross=1, best=best,
                       information_sharing=share).cpu().numpy()
    want = ode.propose_de_vec(space, pop, 22, 2, 9, 3000, 0.5, 1, best=best, information_sharing=share)
    np.testing.assert_array_equal(got, want)
    if share:   # the best config's values do reach the trials
        assert not np.array_equal(got, ode.propose_de_vec(space, pop, 22, 2, 9, 3000, 0.5, 1))


def test_de_information_sharing_perm():
    space = perm_space()
    e = engine(space, seed=24)
    pop = ode.population_init(space, 30, seed=6)
    best = ode.population_init(space, 1, seed=88)[:, 0]
    e.population_set(dev(pop))
    got = e.propose_de(2000, round_=3, cand_base=1, cr=0.5, n_cross=2, best=best).cpu().numpy()
    np.testing.assert_array_equal(got, ode.propose_de_vec(space, pop, 24, 3, 1, 2000, 0.5, 2, best=best))


def test_de_argument_errors():
    """population < 4 (the donor pool of DE/rand/1 needs 3 members besides the
    target) and a negative information_sharing are rejected, never launched"""
    from uptune_amd._lib import UthotError
    space = mixed_space()
    e = engine(space, seed=1)
    with pytest.raises(UthotError):
        e.population_set(dev(ode.population_init(space, 3, seed=1)))
    e.population_set(dev(ode.population_init(space, 4, seed=1)))
    best = ode.population_init(space, 1, seed=2)[:, 0]
    with pytest.raises(UthotError):
        e.propose_de(10, best=best, information_sharing=-1)
    e.propose_de(10, best=best, information_sharing=0)


@pytest.mark.parametrize("which", ["mixed", "r64", "hpl", "perm"])
def test_hash_de_reuses_population_digests(which):
    """ut_hash_de (inner digests of values equal to the target member's taken
    from the population cache) == ut_hash == the oracle, for DE trials, for
    unrelated values, after ut_population_replace (cache patched per row) and
    after ut_pso_commit (cache rebuilt)"""
    space = {"mixed": mixed_space, "r64": r64_space, "hpl": hpl_space, "perm": perm_space}[which]()
    e = engine(space, seed=31)
    e.population_init(3000, round_=1)
    pop = e.population_get().cpu().numpy()
    m, base = 5000, 1234
    trial = e.propose_de(m, round_=2, cand_base=base, cr=0.2)
    want = oracle_hashes(space, trial.cpu().numpy()) if which != "perm" else _row_hashes(space, trial.cpu().numpy())
    assert hexes(e.hash_de(trial, base)) == want
    assert hexes(e.hash(trial)) == want
    # unrelated values (nothing matches a target): every digest is recomputed
    other = torch.from_numpy(ode.population_init(space, 700, seed=99)).cuda()
    assert hexes(e.hash_de(other, 0)) == hexes(e.hash(other))
    # replace some members, then trials of the new population
    rows = torch.tensor([0, 5, 1233 % 3000, 2999], device="cuda")
    e.population_replace(other[:, :4].contiguous(), rows)
    trial2 = e.propose_de(m, round_=3, cand_base=base, cr=0.2)
    assert hexes(e.hash_de(trial2, base)) == hexes(e.hash(trial2))
    if which == "r64":   # PSO commit moves positions: the cache is rebuilt
        e.pso_reset()
        x, v = e.propose_pso(pop[:, 0].copy(), 3000, round_=1)
        e.pso_commit(x, v)
        trial3 = e.propose_de(m, round_=4, cand_base=0, cr=0.2)
        assert hexes(e.hash_de(trial3, 0)) == hexes(e.hash(trial3))


@pytest.mark.parametrize("which", ["r64", "hpl"])
def test_hash_de_shard_window(which):
    """ut_hash_de caches the inner digests of the calling shard's targets only
    (members [cand_base, cand_base + m)): a call for another shard rebuilds the
    window, ut_population_replace patches the rows inside it and skips the
    others, and every digest still equals ut_hash's"""
    space = {"r64": r64_space, "hpl": hpl_space}[which]()
    e = engine(space, seed=37)
    e.population_init(4000, round_=1)
    other = torch.from_numpy(ode.population_init(space, 8, seed=98)).cuda()
    for r, (base, m) in enumerate([(1000, 1000), (1000, 600), (2500, 1000), (1200, 300), (3900, 200)]):
        trial = e.propose_de(m, round_=r, cand_base=base, cr=0.2)
        assert hexes(e.hash_de(trial, base)) == hexes(e.hash(trial)), (base, m)
        if r == 2:   # rows inside ([2500, 3500)) and outside the cached window
            e.population_replace(other[:, :4].contiguous(), torch.tensor([2600, 10, 3499, 3600], device="cuda"))
            trial = e.propose_de(m, round_=9, cand_base=base, cr=0.2)
            assert hexes(e.hash_de(trial, base)) == hexes(e.hash(trial))


@pytest.mark.parametrize("which", ["r64", "hpl"])
def test_hash_capped_grid(which):
    """the grid-stride hash kernels with their grids capped at one workgroup
    per CU (UT_HASH_WG_PER_CU=1: what a round does while a large refit runs,
    at 4) give the digests of the full grids, for ut_hash_de and ut_hash"""
    space = {"r64": r64_space, "hpl": hpl_space}[which]()
    m, base = 200000, 0
    outs = []
    old = os.environ.get("UT_HASH_WG_PER_CU")
    try:
        for cap in ("0", "1"):
            os.environ["UT_HASH_WG_PER_CU"] = cap
            e = engine(space, seed=39)
            e.population_init(m, round_=1)
            trial = e.propose_de(m, round_=2, cand_base=base, cr=0.2)
            outs.append((e.hash_de(trial, base).cpu(), e.hash(trial).cpu()))
            e.close()
    finally:
        if old is None:
            os.environ.pop("UT_HASH_WG_PER_CU", None)
        else:
            os.environ["UT_HASH_WG_PER_CU"] = old
    (a_de, a), (b_de, b) = outs
    assert torch.equal(a_de, a) and torch.equal(b_de, b) and torch.equal(a, b)


def test_hash_small_m_of_a_wide_array():
    """a few columns of a wide SoA array (ld much larger than m): the small-m
    path sizes its scratch by m, not by ld, and the digests equal
    those of a contiguous copy"""
    space = r64_space()
    e = engine(space, seed=5)
    wide = torch.from_numpy(ode.population_init(space, 1 << 20, seed=4)).cuda()   # [64][2^20]: ld = 2^20
    assert hexes(e.hash(wide, m=100)) == hexes(e.hash(wide[:, :100].contiguous()))


def test_de_golden(golden_dir):
    z = np.load(os.path.join(golden_dir, "de_mixed.npz"))
    e = engine(mixed_space(), seed=11)
    e.population_set(dev(z["pop"]))
    got = e.propose_de(48, round_=3, cand_base=5, cr=0.5, n_cross=1).cpu().numpy()
    np.testing.assert_array_equal(got, z["trial"])


def test_de_r64_large():
    space = r64_space()
    e = engine(space, seed=1)
    e.population_init(1 << 16)
    pop = e.population_get().cpu().numpy()
    np.testing.assert_array_equal(pop, ode.population_init(space, 1 << 16, seed=1))
    got = e.propose_de(1 << 16, round_=1, cr=0.2).cpu().numpy()
    np.testing.assert_array_equal(got, ode.propose_de_vec(space, pop, 1, 1, 0, 1 << 16, 0.2, 1))


def test_encode_features():
    space = mixed_space()
    e = engine(space)
    pop = ode.population_init(space, 500, seed=8)
    got = e.encode(dev(pop)).cpu().numpy()
    np.testing.assert_array_equal(got, features(space, pop))


# --------------------------------------------------------------------------- dedup
def test_dedup_matches_oracle():
    space = [Param("a", INT, 0, 20), Param("b", ENUM, options=["x", "y"]), Param("c", BOOL)]
    e = engine(space, seed=2)
    pop = ode.population_init(space, 5000, seed=2)  # 84 distinct configs -> many in-batch dups
    d = e.hash(dev(pop))
    hx = hexes(d)
    hist = hx[3000:3010]
    e.history_reset(16)
    e.history_add(hist)
    got = e.dedup(d).cpu().numpy().tolist()
    assert got == osel.dedup(hx, set(hist))
    # growth path of the history table keeps earlier entries
    e.history_add(hexes(e.hash(dev(ode.population_init(space, 3000, seed=99)))))
    got2 = e.dedup(d).cpu().numpy()
    assert got2.sum() >= sum(got)


def test_dedup_unique_large():
    space = r64_space()
    e = engine(space, seed=3)
    e.population_init(1 << 15)
    vals = e.population_get()
    vals = torch.cat([vals, vals[:, :100]], dim=1).contiguous()
    d = e.hash(vals)
    e.history_reset(0)
    dup = e.dedup(d).cpu().numpy()
    assert dup[: 1 << 15].sum() == 0 and dup[1 << 15:].sum() == 100


# --------------------------------------------------------------------------- GP
def _close(got, want, rtol=RTOL, atol=ATOL):
    np.testing.assert_allclose(got, want, rtol=rtol, atol=atol)


def test_gp_small_golden(golden_dir):
    z = np.load(os.path.join(golden_dir, "gp_small.npz"))
    space = [Param(f"u{k}", FLOAT, 0.0, 1.0) for k in range(5)]
    e = engine(space)
    e.gp_fit(z["X"], z["y"], lengthscale=0.3, sigma_f2=1.0, sigma_n2=1e-6, jitter=1e-8)
    fb, mean, sd = e.gp_stats()
    assert abs(fb - float(z["f_best"])) < 1e-12
    U = dev(z["U"].T)
    mu, var, ei = e.gp_score(U, acq=e.acq("ei"))
    _close(mu.cpu().numpy(), z["mu"])
    _close(var.cpu().numpy(), z["var"])
    _close(ei.cpu().numpy(), z["ei"])
    _, _, ucb = e.gp_score(U, acq=e.acq("ucb", kappa=2.0))
    _close(ucb.cpu().numpy(), z["ucb"])


@pytest.mark.parametrize("prec", [64, 32, 16, 8])
@pytest.mark.parametrize("n,d,ell", [(1024, 64, 0.2), (200, 8, 0.5), (77, 3, 0.25), (300, 16, 1.5), (4096, 112, 1.0)])
def test_gp_vs_oracle(n, d, ell, prec):
    """fp64 and the int8-sliced fp64 tier (precision 8): 1e-5 relative; fp32
    MFMA / f16x3 variance contraction: 1e-3 relative
    (north star), absolute floor 1e-5 (variance near training points is a
    cancellation).  K* and mu stay fp64 in both lower tiers: the first ten
    candidates sit 1e-3 from training points, where |x/ell|^2 ~ 500 and a K*
    exponent taken from an f32-accumulated x.u loses ~1e-4 of var (measured with
    an f16x3 K*, not kept)."""
    rng = np.random.default_rng(n + d)
    X = rng.uniform(size=(n, d))
    y = np.sum((X - 0.4) ** 2, axis=1) + 0.01 * rng.standard_normal(n)
    U = rng.uniform(size=(3000, d))
    U[:10] = X[:10] + 1e-3
    space = [Param(f"u{k}", FLOAT, 0.0, 1.0) for k in range(d)]
    e = engine(space)
    e.gp_set_precision(prec)
    e.gp_fit(X, y, lengthscale=ell, sigma_f2=1.0, sigma_n2=1e-6, jitter=1e-8)
    g = ogp.GP(X, y, lengthscale=ell, sigma_f2=1.0, sigma_n2=1e-6, jitter=1e-8)
    mu_o, var_o = g.posterior(U)
    ei_o = ogp.acquisition(mu_o, var_o, g.f_best)
    mu, var, ei = e.gp_score(dev(U.T))
    if prec in (64, 8):
        _close(mu.cpu().numpy(), mu_o)
        _close(var.cpu().numpy(), var_o, atol=1e-8)
        _close(ei.cpu().numpy(), ei_o, atol=1e-8)
    else:
        # fp32 var contraction: 1e-3 relative, absolute floor 1e-5 (var near
        # training points is sf2 - |L^-1 k*|^2, a cancellation in fp32)
        _close(mu.cpu().numpy(), mu_o)                     # K* and mu stay fp64
        _close(var.cpu().numpy(), var_o, rtol=1e-3, atol=1e-5)
        _close(ei.cpu().numpy(), ei_o, rtol=1e-3, atol=1e-5)


@pytest.mark.parametrize("sf2,ell,sn2,tier", [(1e-3, 0.4, 1e-9, True), (37.0, 0.6, 1e-4, True),
                                              (2.0, 2.0, 1e-6, False)])
def test_gp_f16x3_scaling(sf2, ell, sn2, tier):
    """f16x3 operand scales: sigma_f2 far from 1 (K* scale 2^(14 - ilogb sf2)) and a
    long lengthscale (near-singular K, large |L^-1| entries: the device-side max
    sets L^-1's scale).  The fp32-tier bound (relative to sf2) where the problem is
    conditioned for it; in the near-singular case (ell = 2 on the unit 6-cube,
    every var ~1e-6, sf2 - |L^-1 k*|^2 cancels to ~1e-6 relative) neither 32-bit
    tier meets 1e-5 absolute, and f16x3 is held to the fp32-MFMA path's own error."""
    rng = np.random.default_rng(int(sf2 * 1000) + 7)
    n, d = 500, 6
    X = rng.uniform(size=(n, d))
    y = np.sin(3 * X).sum(axis=1) + 0.01 * rng.standard_normal(n)
    U = rng.uniform(size=(2000, d))
    U[:20] = X[:20] + 1e-3
    space = [Param(f"u{k}", FLOAT, 0.0, 1.0) for k in range(d)]
    g = ogp.GP(X, y, lengthscale=ell, sigma_f2=sf2, sigma_n2=sn2, jitter=1e-8)
    mu_o, var_o = g.posterior(U)
    got = {}
    for prec in (32, 16):
        e = engine(space)
        e.gp_set_precision(prec)
        e.gp_fit(X, y, lengthscale=ell, sigma_f2=sf2, sigma_n2=sn2, jitter=1e-8)
        mu, var, _ = e.gp_score(dev(U.T))
        got[prec] = var.cpu().numpy()
        _close(mu.cpu().numpy(), mu_o)
    err = {p: np.max(np.abs(v - var_o)) / sf2 for p, v in got.items()}
    if tier:
        _close(got[16], var_o, rtol=1e-3, atol=1e-5 * sf2)
    # f16x3 stays within a small factor of the fp32-MFMA path's own error
    assert err[16] <= max(4 * err[32], 1e-7), err


@pytest.mark.parametrize("prec", [64, 32, 16, 8])
@pytest.mark.parametrize("n0,steps,d", [(130, [120], 8), (1000, [4], 64), (513, [1] * 7 + [3], 16),
                                        (40, [4] * 6, 7), (700, [60, 60, 60], 32)])
def test_gp_fit_append_equals_refit(n0, steps, d, prec):
    """incremental fits (ut_gp_set_fit_append): a training set that grows by
    appended rows extends the factor by block rows; the posterior equals a
    fresh full fit's (fp64: 1e-10 relative) and the oracle's at the tier's
    tolerance, over chains of appends inside and across 64-row blocks"""
    rng = np.random.default_rng(n0 + d)
    n1 = n0 + sum(steps)
    X = rng.uniform(size=(n1, d))
    y = np.sum((X - 0.4) ** 2, axis=1) + 0.01 * rng.standard_normal(n1)
    U = rng.uniform(size=(3000, d))
    U[:10] = X[n1 - 10:] + 1e-3          # next to appended rows
    space = [Param(f"u{k}", FLOAT, 0.0, 1.0) for k in range(d)]
    e = engine(space)
    e.gp_set_precision(prec)
    n = n0
    e.gp_fit(X[:n], y[:n], lengthscale=0.5, sigma_f2=1.0, sigma_n2=1e-6, jitter=1e-8)
    assert e.gp_last_fit_kind() == "refit"
    for s in steps:
        n += s
        e.gp_fit(X[:n], y[:n], lengthscale=0.5, sigma_f2=1.0, sigma_n2=1e-6, jitter=1e-8)
        want = "append" if (n + 127) // 128 == (n - s + 127) // 128 else "refit"
        assert e.gp_last_fit_kind() == want, (n, s)
    mu, var, ei = [t.cpu().numpy() for t in e.gp_score(dev(U.T))]
    f = engine(space)
    f.gp_set_precision(prec)
    f.gp_fit(X, y, lengthscale=0.5, sigma_f2=1.0, sigma_n2=1e-6, jitter=1e-8)
    mu_f, var_f, ei_f = [t.cpu().numpy() for t in f.gp_score(dev(U.T))]
    assert e.gp_stats() == f.gp_stats()
    g = ogp.GP(X, y, lengthscale=0.5, sigma_f2=1.0, sigma_n2=1e-6, jitter=1e-8)
    mu_o, var_o = g.posterior(U)
    ei_o = ogp.acquisition(mu_o, var_o, g.f_best)
    if prec in (64, 8):
        _close(mu, mu_f, rtol=1e-10, atol=1e-12)
        _close(var, var_f, rtol=1e-10, atol=1e-12)
        _close(mu, mu_o)
        _close(var, var_o, atol=1e-8)
        _close(ei, ei_o, atol=1e-8)
    else:
        _close(mu, mu_o)
        _close(var, var_o, rtol=1e-3, atol=1e-5)
        _close(ei, ei_o, rtol=1e-3, atol=1e-5)


@pytest.mark.parametrize("m,n", [(300, 4096), (3000, 1024), (100, 300)])
def test_gp_var_split_equals_unsplit(monkeypatch, m, n):
    """few candidate strips: the fp64 variance splits each row tile's k loop
    over workgroups (k_gp_var_pp<true> + k_var_split_red, the survivor /
    threshold passes of pruned scoring); it equals the one-item-per-row-tile
    contraction (UT_VAR_SPLIT=0) to rounding"""
    rng = np.random.default_rng(m + n)
    d = 16
    X = rng.uniform(size=(n, d))
    y = np.sin(3 * X).sum(axis=1)
    U = rng.uniform(size=(m, d))
    U[:5] = X[:5] + 1e-3
    space = [Param(f"u{k}", FLOAT, 0.0, 1.0) for k in range(d)]
    out = {}
    for split in ("1", "0"):
        monkeypatch.setenv("UT_VAR_SPLIT", split)
        e = engine(space)
        e.gp_fit(X, y, lengthscale=0.5, sigma_f2=1.0, sigma_n2=1e-6, jitter=1e-8)
        out[split] = [t.cpu().numpy() for t in e.gp_score(dev(U.T))]
    for a, b in zip(out["1"], out["0"]):
        _close(a, b, rtol=1e-11, atol=1e-13)
    g = ogp.GP(X, y, lengthscale=0.5, sigma_f2=1.0, sigma_n2=1e-6, jitter=1e-8)
    mu_o, var_o = g.posterior(U)
    _close(out["1"][0], mu_o)
    _close(out["1"][1], var_o, atol=1e-8)


def test_gp_fit_append_conditions():
    """an append is taken only for a bitwise prefix with the same
    hyperparameters and a positive-definite previous factor; the pruned
    scoring after an append uses the new factor's |L^-1|_F^2"""
    rng = np.random.default_rng(3)
    d = 6
    X = rng.uniform(size=(300, d))
    y = np.sin(4 * X).sum(axis=1)
    space = [Param(f"u{k}", FLOAT, 0.0, 1.0) for k in range(d)]
    e = engine(space)
    hy = dict(lengthscale=0.4, sigma_f2=1.0, sigma_n2=1e-6, jitter=1e-8)
    e.gp_fit(X[:260], y[:260], **hy)
    e.gp_fit(X[:270], y[:270], **hy)
    assert e.gp_last_fit_kind() == "append"
    e.gp_fit(X[:280], y[:280], **dict(hy, lengthscale=0.41))          # lengthscale changed
    assert e.gp_last_fit_kind() == "refit"
    e.gp_fit(X[:285], y[:285], **dict(hy, lengthscale=0.41, jitter=1e-7))   # noise changed
    assert e.gp_last_fit_kind() == "refit"
    X2 = X.copy()
    X2[3, 2] += 1e-12                                                   # not a prefix
    e.gp_fit(X2[:290], y[:290], **dict(hy, lengthscale=0.41, jitter=1e-7))
    assert e.gp_last_fit_kind() == "refit"
    e.gp_set_fit_append(False)
    e.gp_fit(X2[:295], y[:295], **dict(hy, lengthscale=0.41, jitter=1e-7))
    assert e.gp_last_fit_kind() == "refit"
    e.gp_set_fit_append(True)
    e.gp_fit(X2[:300], y[:300], **dict(hy, lengthscale=0.41, jitter=1e-7))
    assert e.gp_last_fit_kind() == "append"
    # a failed (not positive definite) factor is never extended
    Xd = np.repeat(X[:1], 300, axis=0)
    e.gp_fit(Xd[:260], y[:260], lengthscale=0.4, sigma_f2=1.0, sigma_n2=0.0, jitter=0.0, wait=False)
    e.gp_fit(Xd[:270], y[:270], lengthscale=0.4, sigma_f2=1.0, sigma_n2=0.0, jitter=0.0, wait=False)
    assert e.gp_last_fit_kind() == "refit"
    # pruned top-k after appends equals the dense top-k
    e.gp_fit(X[:200], y[:200], **hy)
    feat = dev(rng.uniform(size=(d, 20000)))
    e.gp_topk_pruned(feat, 16, bound_rows=128)
    e.gp_fit(X[:250], y[:250], **hy)
    assert e.gp_last_fit_kind() == "append"
    idx, top, st = e.gp_topk_pruned(feat, 16, bound_rows=128)
    _, _, score = e.gp_score(feat)
    i2, t2 = e.topk(score, 16)
    _close(top.cpu().numpy(), t2.cpu().numpy(), rtol=1e-9, atol=1e-12)
    assert idx.cpu().numpy().tolist() == i2.cpu().numpy().tolist()


# --------------------------------------------------------------------------- top-k
def test_topk_matches_oracle():
    e = engine([Param("x", FLOAT, 0.0, 1.0)])
    rng = np.random.default_rng(0)
    # power-of-two k with several re-merge passes (sorted-list fast path), and
    # k that are not powers of two (full network every pass)
    for m, k in [(10, 4), (5000, 256), (100000, 1000), (2048 * 3 + 7, 17), (1 << 20, 256), (600001, 64),
                 (300000, 1024)]:
        s = np.round(rng.standard_normal(m), 2)  # many ties
        s[::97] = np.nan
        dup = (rng.uniform(size=m) < 0.1).astype(np.uint8)
        idx, top = e.topk(dev(s), k, dup=dev(dup), cand_base=1000)
        want = osel.topk(list(s), k, dup=list(dup), cand_base=1000)
        assert idx.cpu().numpy().tolist() == want


# --------------------------------------------------------------------------- round
def _round_oracle(space, pop, seed, round_, cand_base, m, cr, X, y, ell, hist, k):
    trial = ode.propose_de_vec(space, pop, seed, round_, cand_base, m, cr, 1)
    hx = oracle_hashes(space, trial)
    dup = osel.dedup(hx, set(hist))
    g = ogp.GP(X, y, lengthscale=ell, sigma_f2=1.0, sigma_n2=1e-6, jitter=1e-8)
    mu, var = g.posterior(features(space, trial).T)
    ei = ogp.acquisition(mu, var, g.f_best)
    return trial, hx, dup, ei


def test_score_round_de_small():
    space = mixed_space()
    seed, m, k = 5, 6000, 64
    e = engine(space, seed=seed)
    pop = ode.population_init(space, 512, seed=seed)
    e.population_set(dev(pop))
    rng = np.random.default_rng(1)
    X = features(space, pop[:, :100]).T
    y = rng.standard_normal(100)
    e.gp_fit(X, y, lengthscale=0.7, sigma_f2=1.0, sigma_n2=1e-6, jitter=1e-8)
    hist = oracle_hashes(space, pop[:, :300])
    e.history_reset(300)
    e.history_add(hist)
    idx, top, dig, vals = e.score_round_de(m, k, round_=2, cand_base=0, cr=0.2)
    trial, hx, dup, ei = _round_oracle(space, pop, seed, 2, 0, m, 0.2, X, y, 0.7, hist, k)
    (pv, pf, pd, pdup, pmu, pvar, psc), ld = e.round_buffers()
    assert ld >= m and psc
    e.sync()
    idx_l = idx.cpu().numpy().tolist()
    # selected rows: values and digests are bit-exact with the oracle
    for j, g in enumerate(idx_l):
        assert g >= 0 and not dup[g]
        np.testing.assert_array_equal(vals[:, j].cpu().numpy(), trial[:, g])
        assert hexes(dig[j:j + 1])[0] == hx[g]
    # selection = oracle top-k of the oracle scores wherever scores are distinct
    want = osel.topk(list(ei), k, dup=dup)
    top_o = np.asarray([ei[g] for g in want])
    _close(top.cpu().numpy(), top_o, atol=1e-8)
    gaps = np.abs(np.diff(np.sort(np.asarray(ei)[np.asarray(dup) == 0])[::-1][: k + 1]))
    if gaps.min() > 1e-6:
        assert idx_l == want


def test_score_round_de_best_row_digests():
    """the scoring round's fused DE-diff (k_de writes the changed-value mask and
    pairs the hash reuses) with the best config in the donor pool, before and
    after a population replace: every selected row's values and digest equal
    the oracle's trial and hash_config"""
    space = mixed_space()
    seed, npop, m, k = 31, 300, 4000, 1024
    e = engine(space, seed=seed)
    pop = ode.population_init(space, npop, seed=seed)
    e.population_set(dev(pop))
    X = features(space, pop[:, :100]).T
    e.gp_fit(X, np.sum((X - 0.5) ** 2, axis=1), lengthscale=0.7, sigma_f2=1.0, sigma_n2=1e-6, jitter=1e-8)
    e.history_reset(0)
    best = ode.population_init(space, 1, seed=5)[:, 0]
    for rnd, base in ((4, 7), (5, 4007)):
        idx, top, dig, vals = e.score_round_de(m, k, round_=rnd, cand_base=base, cr=0.5, best=best,
                                               information_sharing=3)
        trial = ode.propose_de_vec(space, pop, seed, rnd, base, m, 0.5, 1, best=best, information_sharing=3)
        e.sync()
        idx_l = idx.cpu().numpy().tolist()
        sel = [g - base for g in idx_l]
        assert all(0 <= j < m for j in sel)
        np.testing.assert_array_equal(vals.cpu().numpy(), trial[:, sel])
        assert hexes(dig) == oracle_hashes(space, trial[:, sel])
        # accept the first 64 selections into the population (rows 0..63): the
        # next round reuses the patched inner-digest cache
        rows = np.arange(64)
        e.population_replace(vals[:, :64].contiguous(), dev(rows.astype(np.int64)))
        pop = pop.copy()
        pop[:, rows] = trial[:, sel[:64]]


def test_sharding_invariance():
    """top-k over a pool split into shards (global candidate indices) and
    merged equals the single-shot top-k -- the multi-GPU contract."""
    space = r64_space()
    e = engine(space, seed=9)
    e.population_init(4096)
    rng = np.random.default_rng(2)
    X = rng.uniform(size=(256, 64))
    y = rng.standard_normal(256)
    e.gp_fit(X, y, lengthscale=2.0)
    k, m = 32, 8192
    i_full, s_full, _, _ = e.score_round_de(m, k, round_=1, cand_base=0)
    parts = []
    for base in (0, 3000, 6000):
        mm = min(3000, m - base)
        i_p, s_p, _, _ = e.score_round_de(mm, k, round_=1, cand_base=base)
        parts += list(zip(s_p.cpu().numpy().tolist(), i_p.cpu().numpy().tolist()))
    parts = [p for p in parts if p[1] >= 0]
    parts.sort(key=lambda t: (-t[0], t[1]))
    assert [p[1] for p in parts[:k]] == i_full.cpu().numpy().tolist()


def test_full_size_round_properties():
    """C2 at full size (m = 2^20, n = 1024, d = 64): size-independent checks."""
    space = r64_space()
    m, n, k = 1 << 20, 1024, 256
    e = engine(space, seed=1)
    e.population_init(m)
    rng = np.random.default_rng(0)
    X = rng.uniform(size=(n, 64))
    xs = X * 2000.0 - 1000.0
    y = np.sum(100.0 * (xs[:, 1:] - xs[:, :-1] ** 2) ** 2 + (xs[:, :-1] - 1.0) ** 2, axis=1)
    e.gp_fit(X, y, lengthscale=0.2, sigma_f2=1.0, sigma_n2=1e-6)
    e.history_reset(0)
    idx, top, dig, vals = e.score_round_de(m, k, round_=0, cand_base=0, cr=0.2)
    idx = idx.cpu().numpy()
    top = top.cpu().numpy()
    assert np.all(idx >= 0) and len(set(idx.tolist())) == k
    assert np.all(np.diff(top) <= 0)
    v = vals.cpu().numpy()
    # digests of the selected rows recomputed by the oracle
    assert hexes(dig) == oracle_hashes(space, v)
    # their scores recomputed by the oracle GP
    g = ogp.GP(X, y, lengthscale=0.2, sigma_f2=1.0, sigma_n2=1e-6)
    mu, var = g.posterior(features(space, v).T)
    ei = ogp.acquisition(mu, var, g.f_best)
    _close(top, ei, atol=1e-8)
    # and the rows are exactly the DE trials the oracle proposes for those indices
    pop = e.population_get().cpu().numpy()
    sub = ode.propose_de_vec(space, pop, 1, 0, 0, m, 0.2, 1)[:, idx]
    np.testing.assert_array_equal(v, sub)


# --------------------------------------------------------------------------- PSO / GA
@pytest.mark.parametrize("alias,enum_mode", [(True, 0), (False, 1)])
def test_pso_matches_oracle(alias, enum_mode):
    from oracle import pso as opso
    space = mixed_space()
    e = engine(space, seed=31)
    pop = ode.population_init(space, 700, seed=6)
    e.population_set(dev(pop))
    e.pso_reset()
    vel = np.zeros_like(pop)
    gbest = pop[:, 17].copy()
    x, v = e.propose_pso(gbest, 700, round_=4, alias_pbest=alias, enum_mode=enum_mode)
    wx, wv = opso.propose_pso_vec(space, pop, vel, pop, gbest, 31, 4, 0, 700, enum_mode=enum_mode)
    np.testing.assert_array_equal(x.cpu().numpy(), wx)
    np.testing.assert_array_equal(v.cpu().numpy(), wv)
    # second generation from committed state (non-zero velocities)
    e.pso_commit(x, v)
    x2, v2 = e.propose_pso(gbest, 1400, round_=5, cand_base=0, alias_pbest=alias, enum_mode=enum_mode)
    pb = wx if alias else pop
    wx2, wv2 = opso.propose_pso_vec(space, wx, wv, pb, gbest, 31, 5, 0, 1400, enum_mode=enum_mode)
    np.testing.assert_array_equal(x2.cpu().numpy(), wx2)
    np.testing.assert_array_equal(v2.cpu().numpy(), wv2)


@pytest.mark.parametrize("kw", [
    dict(mutation_rate=0.1),                                             # UniformGreedyMutation / ga-base
    dict(mutation_rate=0.3, normal=True, sigma=0.1),                     # NormalGreedyMutation(0.3)
    dict(mutation_rate=0.1, normal=True, crossover_rate=0.5, crossover_strength=0.2, op=5),   # GGA
    dict(mutation_rate=0.01, crossover_rate=0.8),                        # GA(crossover=...)
])
def test_ga_matches_oracle(kw):
    from oracle import ga as oga
    space = mixed_space() + [Param("z%d" % i, INT, 0, 3) for i in range(8)]
    e = engine(space, seed=41)
    pop = ode.population_init(space, 8, seed=9)
    best = pop[:, 0].copy()
    for p1, p2 in [(best, None), (None, None), (best, pop[:, 1].copy())]:
        got, inv = e.propose_ga(3000, parent1=p1, parent2=p2, round_=2, cand_base=11, **kw)
        want, winv = oga.propose_ga_vec(space, p1, p2, 41, 2, 11, 3000, **kw)
        np.testing.assert_array_equal(got.cpu().numpy(), want)
        np.testing.assert_array_equal(inv.cpu().numpy().astype(bool), winv)


def test_ga_retry_gives_up_on_tiny_space():
    """A 1-value space can never differ from its parent: every candidate is
    invalid after max_retries (the reference returns None, :45-49)."""
    from oracle import ga as oga
    space = [Param("only", INT, 5, 5), Param("b", ENUM, options=["x"])]
    e = engine(space, seed=1)
    got, inv = e.propose_ga(100, parent1=np.array([5.0, 0.0]), mutation_rate=0.5)
    assert inv.cpu().numpy().all()
    _, winv = oga.propose_ga_vec(space, np.array([5.0, 0.0]), None, 1, 0, 0, 100, mutation_rate=0.5)
    assert winv.all()


# --------------------------------------------------------------------------- scaled kinds (C3 HPL-64)
def hpl_space():
    from uptune_amd import spaces
    return oracle_space(spaces.hpl64())


def _non_cr_log_ints(golden_dir):
    """integers x in [2^22, 2^31) where CPython's math.log(x) is NOT the
    correctly rounded log -- the arguments a correctly rounded device log got
    wrong in round 1 (tests/golden/make_libm_log_cases.py)"""
    with open(os.path.join(golden_dir, "libm_log_non_cr.json")) as f:
        return json.load(f)["ints"]


def test_hpl_population_de_encode_hash():
    space = hpl_space()
    e = engine(space, seed=13)
    e.population_init(4000, round_=1)
    pop = e.population_get().cpu().numpy()
    np.testing.assert_array_equal(pop, ode.population_init(space, 4000, seed=13, round_=1))
    got = e.propose_de(6000, round_=3, cand_base=77, cr=0.5, n_cross=2).cpu().numpy()
    want = ode.propose_de_vec(space, pop, 13, 3, 77, 6000, 0.5, 2)
    np.testing.assert_array_equal(got, want)
    np.testing.assert_array_equal(e.encode(dev(got)).cpu().numpy(), features(space, got))
    # hashes bit-exact everywhere, including logint_3 (range 2^30: no host
    # table, the device's libm_log restatement)
    hx = hexes(e.hash(dev(got)))
    want_h = oracle_hashes(space, got)
    bad = [j for j in range(got.shape[1]) if hx[j] != want_h[j]]
    assert bad == []


def test_logint_large_range_bit_exact(golden_dir):
    """LogIntegerParameter over [0, 2^31) (no host table): get_value =
    math.log(v + 1.0 - min, 2.0) restated on the device (ut_core.h libm_log)
    is bit-identical to THIS box's CPython on random values and on integers
    where libm's log is not correctly rounded; digests and unit features
    follow (manipulator.py:784-787, :456-459)."""
    from oracle.space import LOGINT
    space = [Param("big_log", LOGINT, 0, (1 << 31) - 1), Param("f", FLOAT, 0.0, 1.0)]
    e = engine(space, seed=3)
    assert e.spec.params[0].vtab is None
    rng = np.random.default_rng(11)
    xs = _non_cr_log_ints(golden_dir) + [int(v) for v in rng.integers(1, (1 << 31) - 1, 4000)]
    vals = np.zeros((2, len(xs)))
    vals[0] = [x - 1 for x in xs]          # v + 1.0 - min = x
    vals[1] = rng.uniform(size=len(xs))
    assert hexes(e.hash(dev(vals))) == oracle_hashes(space, vals)
    np.testing.assert_array_equal(e.encode(dev(vals)).cpu().numpy(), features(space, vals))


@pytest.mark.parametrize("alias,enum_mode", [(True, 0), (False, 1)])
def test_hpl_pso_matches_oracle(alias, enum_mode):
    from oracle import pso as opso
    space = hpl_space()
    e = engine(space, seed=17)
    pop = ode.population_init(space, 900, seed=3)
    e.population_set(dev(pop))
    e.pso_reset()
    gbest = pop[:, 5].copy()
    x, v = e.propose_pso(gbest, 900, round_=2, alias_pbest=alias, enum_mode=enum_mode)
    wx, wv = opso.propose_pso_vec(space, pop, np.zeros_like(pop), pop, gbest, 17, 2, 0, 900, enum_mode=enum_mode)
    np.testing.assert_array_equal(x.cpu().numpy(), wx)
    np.testing.assert_array_equal(v.cpu().numpy(), wv)
    e.pso_commit(x, v)
    x2, v2 = e.propose_pso(gbest, 900, round_=3, alias_pbest=alias, enum_mode=enum_mode)
    wx2, wv2 = opso.propose_pso_vec(space, wx, wv, wx if alias else pop, gbest, 17, 3, 0, 900, enum_mode=enum_mode)
    np.testing.assert_array_equal(x2.cpu().numpy(), wx2)
    np.testing.assert_array_equal(v2.cpu().numpy(), wv2)


@pytest.mark.parametrize("kw", [dict(mutation_rate=0.2), dict(mutation_rate=0.3, normal=True, sigma=0.1),
                                dict(mutation_rate=0.1, normal=True, crossover_rate=0.5, crossover_strength=0.2,
                                     op=5)])
def test_hpl_ga_matches_oracle(kw):
    from oracle import ga as oga
    space = hpl_space()
    e = engine(space, seed=19)
    pop = ode.population_init(space, 4, seed=2)
    for p1, p2 in [(pop[:, 0].copy(), None), (None, None), (pop[:, 0].copy(), pop[:, 1].copy())]:
        got, inv = e.propose_ga(2000, parent1=p1, parent2=p2, round_=1, cand_base=3, **kw)
        want, winv = oga.propose_ga_vec(space, p1, p2, 19, 1, 3, 2000, **kw)
        np.testing.assert_array_equal(got.cpu().numpy(), want)
        np.testing.assert_array_equal(inv.cpu().numpy().astype(bool), winv)


# --------------------------------------------------------------------------- permutations
def perm_space():
    from uptune_amd import spaces
    return oracle_space(spaces.perm_mixed())


def _row_hashes(space, vals):
    from oracle.space import row_values
    return [oh.hash_config(space, row_values(space, vals, j)) for j in range(vals.shape[1])]


def test_perm_population_de_encode_hash():
    space = perm_space()
    e = engine(space, seed=23)
    e.population_init(3000, round_=1)
    pop = e.population_get().cpu().numpy()
    np.testing.assert_array_equal(pop, ode.population_init(space, 3000, seed=23, round_=1))
    got = e.propose_de(2500, round_=4, cand_base=11, cr=0.5, n_cross=2).cpu().numpy()
    np.testing.assert_array_equal(got, ode.propose_de_vec(space, pop, 23, 4, 11, 2500, 0.5, 2))
    np.testing.assert_array_equal(e.encode(dev(got)).cpu().numpy(), features(space, got))
    assert hexes(e.hash(dev(got))) == _row_hashes(space, got)
    # config dicts round trip through the host codec, and hash the same on the host path
    cfgs = e.decode(dev(got[:, :20]))
    assert isinstance(cfgs[0]["tour"], list) and sorted(cfgs[0]["tour"]) == [100 + 7 * k for k in range(40)]
    assert e.hash_configs(cfgs) == _row_hashes(space, got[:, :20])


@pytest.mark.parametrize("xop", ["op3_cross_OX1", "op3_cross_OX3", "op3_cross_PX", "op3_cross_CX",
                                 "op3_cross_PMX"])
def test_perm_pso_matches_oracle(xop):
    from oracle import perm as opm
    from oracle import pso as opso
    space = perm_space()
    e = engine(space, seed=29)
    pop = ode.population_init(space, 600, seed=8)
    e.population_set(dev(pop))
    e.pso_reset()
    gbest = pop[:, 7].copy()
    x, v = e.propose_pso(gbest, 600, round_=2, alias_pbest=True, crossover=xop)
    wx, wv = opso.propose_pso_vec(space, pop, np.zeros_like(pop), pop, gbest, 29, 2, 0, 600,
                                  crossover=opm.XNAMES[xop])
    np.testing.assert_array_equal(x.cpu().numpy(), wx)
    np.testing.assert_array_equal(v.cpu().numpy(), wv)
    # non-aliased bests: pso_best holds the reset positions while the positions move
    e.pso_commit(x, v)
    x2, v2 = e.propose_pso(gbest, 600, round_=3, alias_pbest=False, crossover=xop)
    wx2, wv2 = opso.propose_pso_vec(space, wx, wv, pop, gbest, 29, 3, 0, 600, crossover=opm.XNAMES[xop])
    np.testing.assert_array_equal(x2.cpu().numpy(), wx2)
    np.testing.assert_array_equal(v2.cpu().numpy(), wv2)


@pytest.mark.parametrize("xop", ["op3_cross_OX1", "op3_cross_OX3", "op3_cross_PX", "op3_cross_CX",
                                 "op3_cross_PMX"])
@pytest.mark.parametrize("normal", [False, True])
def test_perm_ga_matches_oracle(xop, normal):
    from oracle import ga as oga
    from oracle import perm as opm
    space = perm_space()
    e = engine(space, seed=31)
    pop = ode.population_init(space, 4, seed=6)
    kw = dict(mutation_rate=0.2, crossover_rate=0.8, normal=normal)
    for p1, p2 in [(pop[:, 0].copy(), pop[:, 1].copy()), (None, None), (pop[:, 2].copy(), None)]:
        got, inv = e.propose_ga(1500, parent1=p1, parent2=p2, round_=2, cand_base=5, crossover=xop, **kw)
        want, winv = oga.propose_ga_vec(space, p1, p2, 31, 2, 5, 1500, crossover=opm.XNAMES[xop], **kw)
        np.testing.assert_array_equal(got.cpu().numpy(), want)
        np.testing.assert_array_equal(inv.cpu().numpy().astype(bool), winv)


def test_perm_gga_matches_oracle():
    from oracle import ga as oga
    space = perm_space()
    e = engine(space, seed=37)
    pop = ode.population_init(space, 4, seed=7)
    kw = dict(mutation_rate=0.1, normal=True, crossover_rate=0.5, crossover_strength=0.2, op=5)
    got, inv = e.propose_ga(1500, parent1=pop[:, 0].copy(), parent2=pop[:, 3].copy(), round_=1, **kw)
    want, winv = oga.propose_ga_vec(space, pop[:, 0].copy(), pop[:, 3].copy(), 37, 1, 0, 1500, **kw)
    np.testing.assert_array_equal(got.cpu().numpy(), want)
    np.testing.assert_array_equal(inv.cpu().numpy().astype(bool), winv)


def test_perm_score_round():
    """whole DE round on a permutation space: selection == oracle's"""
    from oracle.space import features as ofeat
    space = perm_space()
    e = engine(space, seed=41)
    e.population_init(4096)
    pop = e.population_get().cpu().numpy()
    rng = np.random.default_rng(3)
    Xv = ode.population_init(space, 200, seed=77)
    X = ofeat(space, Xv).T
    y = rng.normal(size=200)
    e.gp_fit(X, y, lengthscale=0.7, sigma_f2=1.0, sigma_n2=1e-4, jitter=1e-8)
    e.history_reset(0)
    idx, top, dig, vals = e.score_round_de(4096, 32, round_=1, cr=0.3)
    trial = ode.propose_de_vec(space, pop, 41, 1, 0, 4096, 0.3, 1)
    g = ogp.GP(X, y, lengthscale=0.7, sigma_f2=1.0, sigma_n2=1e-4, jitter=1e-8)
    mu, var = g.posterior(ofeat(space, trial).T)
    ei = ogp.acquisition(mu, var, g.f_best)
    dup = osel.dedup(_row_hashes(space, trial), set())
    want = osel.topk(list(ei), 32, dup=dup)
    idx_l = idx.cpu().numpy().tolist()
    _close(top.cpu().numpy(), np.asarray([ei[g] for g in want]), atol=1e-8)
    np.testing.assert_array_equal(vals.cpu().numpy(), trial[:, idx_l])
    gaps = np.abs(np.diff(np.sort(np.asarray(ei)[np.asarray(dup) == 0])[::-1][:33]))
    if gaps.min() > 1e-6:
        assert idx_l == want


# --------------------------------------------------------------------------- EI-bound pruning
@pytest.mark.parametrize("prune_pass", [32, 64])
@pytest.mark.parametrize("acq,bound_rows", [("ei", 128), ("ei", 384), ("ucb", 256)])
def test_gp_topk_pruned_equals_dense(acq, bound_rows, prune_pass):
    """ut_gp_topk_pruned: the top-k of a non-degenerate GP --
    training points drawn from the population the candidates come from, so
    many candidates sit near training data and their bound is loose -- equals
    the dense device top-k and the oracle's; the survivors are a strict subset.
    Both bound passes: f32 contraction and k* with every rounding bounded (32,
    the default) and fp64"""
    space = mixed_space()
    e = engine(space, seed=8)
    e.gp_set_prune_pass(prune_pass)
    pop = ode.population_init(space, 4096, seed=8)
    e.population_set(dev(pop))
    n = 640
    X = features(space, pop[:, :n]).T
    rng = np.random.default_rng(4)
    y = np.sum((X - 0.3) ** 2, axis=1) + 0.05 * rng.standard_normal(n)
    e.gp_fit(X, y, lengthscale=0.6, sigma_f2=1.0, sigma_n2=1e-6, jitter=1e-8)
    m, k = 20000, 64
    trial = e.propose_de(m, round_=1, cr=0.5)
    feat = e.encode(trial)
    dup = torch.zeros(m, dtype=torch.uint8, device="cuda")
    dup[::97] = 1
    a = e.acq(acq, xi=0.0, kappa=2.0)
    idx, top, st = e.gp_topk_pruned(feat, k, acq=a, dup=dup, cand_base=5, bound_rows=bound_rows)
    _, _, score = e.gp_score(feat, acq=a, dup=dup)
    i2, t2 = e.topk(score, k, dup=dup, cand_base=5)
    assert 0 < st["survivors"] < m and not st["dense"] and st["bound_rows"] >= bound_rows
    g = ogp.GP(X, y, lengthscale=0.6, sigma_f2=1.0, sigma_n2=1e-6, jitter=1e-8)
    mu, var = g.posterior(features(space, trial.cpu().numpy()).T)
    sc = ogp.acquisition(mu, var, g.f_best, kind=acq, kappa=2.0)
    sc = np.where(dup.cpu().numpy() != 0, -np.inf, sc)
    want = [5 + i for i in sorted(range(m), key=lambda i: (-sc[i], i))[:k]]
    gaps = np.abs(np.diff(np.sort(sc[np.isfinite(sc)])[::-1][:k + 1]))
    _close(top.cpu().numpy(), t2.cpu().numpy(), rtol=1e-9, atol=1e-12)
    if gaps.min() > 1e-9:
        assert idx.cpu().numpy().tolist() == i2.cpu().numpy().tolist() == want


def test_gp_topk_pruned_degenerate_exact_ties():
    """far-away candidates (k* ~ 0 everywhere): every score is the same.  The
    tail bound |L^-1|_F^2 |k*|^2 proves each candidate's variance from the first
    row tile (exact flag), so ties are broken by index in the pruning itself:
    exactly k survivors, and the dense top-k"""
    space = r64_space()
    e = engine(space, seed=3)
    e.population_init(8192)
    rng = np.random.default_rng(7)
    X = rng.uniform(size=(1024, 64))
    y = rng.standard_normal(1024)
    e.gp_fit(X, y, lengthscale=0.2)
    vals = e.propose_de(8192, round_=1)
    feat = e.encode(vals)
    for prune_pass in (32, 64):   # the f32 pass pins these scores too (k*^ flushes to 0 within its bound)
        e.gp_set_prune_pass(prune_pass)
        for base in (0, 1000):
            idx, top, st = e.gp_topk_pruned(feat, 32, bound_rows=128, cand_base=base)
            _, _, score = e.gp_score(feat)
            i2, t2 = e.topk(score, 32, cand_base=base)
            assert idx.cpu().numpy().tolist() == i2.cpu().numpy().tolist() == list(range(base, base + 32))
            assert not st["dense"] and st["survivors"] == 32, (prune_pass, st)


def test_gp_topk_pruned_dense_fallback():
    """every candidate at the same training point: identical scores whose
    variance the tail bound cannot pin (k* ~ sf2), so every bound reaches the
    threshold, the round falls back to the dense variance, and the selection
    is still the dense top-k (the smallest indices)"""
    space = r64_space()
    e = engine(space, seed=3)
    rng = np.random.default_rng(9)
    X = rng.uniform(size=(512, 64))
    y = rng.standard_normal(512)
    e.gp_fit(X, y, lengthscale=0.5)
    feat = dev(np.repeat(X[5:6].T, 4096, axis=1))
    idx, top, st = e.gp_topk_pruned(feat, 16, bound_rows=128)
    _, _, score = e.gp_score(feat)
    i2, t2 = e.topk(score, 16)
    assert idx.cpu().numpy().tolist() == i2.cpu().numpy().tolist() == list(range(16))
    assert st["dense"] and st["survivors"] == 4096, st


def test_score_round_de_pruned_equals_dense_round():
    """the whole DE round with pruning (ut_score_round_de_pruned) selects the
    same candidates, scores, digests and rows as the dense round"""
    space = mixed_space()
    e = engine(space, seed=12)
    pop = ode.population_init(space, 8192, seed=12)
    e.population_set(dev(pop))
    n = 512
    X = features(space, pop[:, :n]).T
    y = np.sum((X - 0.6) ** 2, axis=1)
    e.gp_fit(X, y, lengthscale=0.6, sigma_f2=1.0, sigma_n2=1e-6, jitter=1e-8)
    e.history_reset(0)
    e.history_add(e.hash(dev(pop[:, :n])))
    a = e.score_round_de(8192, 48, round_=3, cand_base=100, cr=0.3)
    b = e.score_round_de_pruned(8192, 48, round_=3, cand_base=100, cr=0.3, bound_rows=128)
    st = b[4]
    assert 0 < st["survivors"] < 8192 and not st["dense"]
    sa, sb = a[1].cpu().numpy(), b[1].cpu().numpy()
    _close(sb, sa, rtol=1e-9, atol=1e-12)
    if np.abs(np.diff(sa)).min() > 1e-9:
        assert a[0].cpu().numpy().tolist() == b[0].cpu().numpy().tolist()
        assert hexes(a[2]) == hexes(b[2])
        np.testing.assert_array_equal(a[3].cpu().numpy(), b[3].cpu().numpy())


@pytest.mark.parametrize("prec", [64, 8])
def test_repeated_same_shape_categorical_fits(prec):
    """a replayed fit graph once failed its PD check on the third
    same-shape categorical fit of one engine.  The fit is launched kernel by
    kernel now; three same-shape categorical fits with DIFFERENT data in one
    engine (every signature the same, every buffer reused) must each give the
    oracle's posterior -- no fit state survives from the previous fit."""
    _require_gpu()
    space = hpl_space()
    e = engine(space, seed=5)
    e.gp_set_precision(prec)
    n, m = 512, 3000
    cand = ode.population_init(space, m, seed=6)
    for rep in range(3):
        tr = ode.population_init(space, n, seed=100 + rep)
        X = features(space, tr).T
        y = np.sum((X - 0.3 - 0.1 * rep) ** 2, axis=1)
        e.gp_fit(X, y, lengthscale=1.0, sigma_f2=1.0, sigma_n2=1e-6, jitter=1e-8)
        assert e.gp_kstar_mode() == "categorical"
        mu, var, score = [t.cpu().numpy() for t in e.gp_score_values(dev(cand), acq=e.acq("ei"))]
        g = ogp.GP(X, y, lengthscale=1.0, sigma_f2=1.0, sigma_n2=1e-6, jitter=1e-8)
        wmu, wvar = g.posterior(features(space, cand).T)
        np.testing.assert_allclose(mu, wmu, rtol=RTOL, atol=ATOL)
        np.testing.assert_allclose(var, wvar, rtol=RTOL, atol=ATOL)
        np.testing.assert_allclose(score, ogp.acquisition(wmu, wvar, g.f_best), rtol=RTOL, atol=ATOL)


@pytest.mark.parametrize("order", ["feat_first", "round_first"])
def test_pruned_entry_points_share_one_categorical_fit(order):
    """the f32 bound pass caches an f32 copy of the training operand
    per fit.  In categorical mode the feature entry (ut_gp_topk_pruned: every
    feature, dense K*) and the fused DE round (ut_score_round_de_pruned: the
    numeric block + one-hot codes) take different operands; run both on ONE
    fit, in either order, and each must equal its dense counterpart."""
    _require_gpu()
    space = hpl_space()
    e = engine(space, seed=21)
    e.gp_set_prune_pass(32)
    pop = ode.population_init(space, 8192, seed=21)
    e.population_set(dev(pop))
    n = 512
    X = features(space, pop[:, :n]).T
    y = np.sum((X - 0.4) ** 2, axis=1)
    e.gp_fit(X, y, lengthscale=1.0, sigma_f2=1.0, sigma_n2=1e-6, jitter=1e-8)
    assert e.gp_kstar_mode() == "categorical"
    e.history_reset(0)
    trial = e.propose_de(8192, round_=5, cr=0.3)
    feat = e.encode(trial)

    def feat_entry():
        idx, top, st = e.gp_topk_pruned(feat, 32, bound_rows=128)
        _, _, score = e.gp_score(feat)
        i2, t2 = e.topk(score, 32)
        _close(top.cpu().numpy(), t2.cpu().numpy(), rtol=1e-9, atol=1e-12)
        if np.abs(np.diff(t2.cpu().numpy())).min() > 1e-9:
            assert idx.cpu().numpy().tolist() == i2.cpu().numpy().tolist()

    def round_entry():
        a = e.score_round_de(8192, 32, round_=3, cand_base=0, cr=0.3)
        b = e.score_round_de_pruned(8192, 32, round_=3, cand_base=0, cr=0.3, bound_rows=128)
        sa, sb = a[1].cpu().numpy(), b[1].cpu().numpy()
        _close(sb, sa, rtol=1e-9, atol=1e-12)
        if np.abs(np.diff(sa)).min() > 1e-9:
            assert a[0].cpu().numpy().tolist() == b[0].cpu().numpy().tolist()

    for f in ((feat_entry, round_entry, feat_entry) if order == "feat_first" else
              (round_entry, feat_entry, round_entry)):
        f()


@pytest.mark.parametrize("which", ["mixed", "r64", "hpl", "perm"])
def test_hash_parent_reuses_parent_digests(which):
    """ut_hash_parent (inner digests of values equal to the parent's taken from
    the parent's own) == ut_hash == the oracle, for GA / GGA children of that
    parent, for two-parent crossovers, and for values unrelated to the parent"""
    space = {"mixed": mixed_space, "r64": r64_space, "hpl": hpl_space, "perm": perm_space}[which]()
    e = engine(space, seed=41)
    e.population_init(64, round_=1)
    pop = e.population_get().cpu().numpy()
    p1, p2 = pop[:, 3].copy(), pop[:, 7].copy()
    for kw in ({"mutation_rate": 0.1}, {"mutation_rate": 0.05, "normal": True, "op": 5},
               {"mutation_rate": 0.1, "crossover_rate": 0.5, "crossover_strength": 0.2}):
        kids, _ = e.propose_ga(4000, parent1=p1, parent2=p2 if "crossover_rate" in kw else None, round_=2,
                               cand_base=17, **kw)
        want = hexes(e.hash(kids))
        assert hexes(e.hash_parent(kids, p1)) == want
        vals = kids.cpu().numpy()
        sub = slice(0, 300)
        ref = oracle_hashes(space, vals[:, sub]) if which != "perm" else _row_hashes(space, vals[:, sub])
        assert want[sub] == ref
    other = torch.from_numpy(ode.population_init(space, 500, seed=98)).cuda()
    assert hexes(e.hash_parent(other, p1)) == hexes(e.hash(other))
    # the parent itself and an empty batch
    assert hexes(e.hash_parent(torch.from_numpy(p1.reshape(-1, 1).copy()).cuda(), p1)) == \
        hexes(e.hash(torch.from_numpy(p1.reshape(-1, 1).copy()).cuda()))


@pytest.mark.parametrize("which", ["mixed", "hpl", "perm"])
def test_de_donor_copy_follows_population_changes(which):
    """k_de gathers its donors from a member-major unit-value copy of the
    population: after every way the population changes (replace: rows patched;
    set, PSO commit, re-init: rebuilt; slot switch: the slot's own copy; the
    best config row rewritten per call) the trials still equal the oracle's on
    the population as it is then"""
    space = {"mixed": mixed_space, "hpl": hpl_space, "perm": perm_space}[which]()
    e = engine(space, seed=51)
    e.population_init(500, round_=1)
    best = None

    def check(rnd, share=0):
        pop = e.population_get().cpu().numpy()
        got = e.propose_de(3000, round_=rnd, cand_base=7, cr=0.3, best=best, information_sharing=share).cpu().numpy()
        want = ode.propose_de_vec(space, pop, 51, rnd, 7, 3000, 0.3, 1, best=best if share else None,
                                  information_sharing=share)
        np.testing.assert_array_equal(got, want)

    check(1)
    other = ode.population_init(space, 500, seed=77)
    e.population_replace(dev(other[:, :40]), torch.arange(100, 140, device="cuda"))   # rows patched
    check(2)
    best = other[:, 3].copy()
    check(3, share=2)                                  # the best row of the copy
    best = other[:, 9].copy()
    check(4, share=1)                                  # ... rewritten per call
    best = None
    e.population_set(dev(other))                       # rebuilt
    check(5)
    if which != "perm":
        e.pso_reset()
        x, v = e.propose_pso(other[:, 0].copy(), 500, round_=1)
        e.pso_commit(x, v)                             # positions moved: rebuilt
        check(6)
    e.population_select(1)                             # another slot, its own population and copy
    e.population_init(300, round_=4)
    check(7)
    e.population_select(0)
    check(8)
    e.population_init(500, round_=9)                   # re-init: rebuilt
    check(9)


def _wide_space(P):
    kinds = [lambda i: Param("f%d" % i, FLOAT, -3.0, 7.5), lambda i: Param("i%d" % i, INT, -50, 900),
             lambda i: Param("b%d" % i, BOOL), lambda i: Param("e%d" % i, ENUM, options=["on", "off", "default"])]
    return [kinds[i % 4](i) for i in range(P)]


@pytest.mark.parametrize("P,aos", [(339, "1"), (339, "0"), (61, "1"), (2100, "1")])
def test_de_wide_spaces(P, aos, monkeypatch):
    """k_de on wide spaces: 339 params (the C4 gcc shape; a column count that is
    no multiple of the 8-column staging group or the 16-column row pitch) and 61
    (< one group of 64), through the member-major donor copy and, with
    UT_DE_AOS=0, the column-major gather; 2100 params (> 2048: the cr-test bits
    spill to the global scratch and the column-major path is taken)"""
    monkeypatch.setenv("UT_DE_AOS", aos)
    space = _wide_space(P)
    e = engine(space, seed=61)
    e.population_init(97, round_=1)
    pop = e.population_get().cpu().numpy()
    best = ode.population_init(space, 1, seed=5)[:, 0]
    m = 600 if P > 1000 else 2500
    for rnd, cr, n_cross, share in ((2, 0.1, 1, 0), (3, 0.6, 4, 2)):
        got = e.propose_de(m, round_=rnd, cand_base=11, cr=cr, n_cross=n_cross, best=best,
                           information_sharing=share).cpu().numpy()
        want = ode.propose_de_vec(space, pop, 61, rnd, 11, m, cr, n_cross, best=best if share else None,
                                  information_sharing=share)
        np.testing.assert_array_equal(got, want)


@pytest.mark.parametrize("which,prec", [("mixed", 64), ("hpl", 64), ("mixed", 32), ("hpl", 32), ("mixed", 16),
                                        ("hpl", 16)])
def test_gp_score_values_equals_score_of_encoded(which, prec):
    """ut_gp_score_values (encode + 1/ell scaling fused into the K* operand
    pass) == ut_gp_score(ut_encode_features(values)), and == the oracle's
    posterior within the precision's tier (fp64: RTOL; fp32 / f16x3: 1e-3)"""
    space = {"mixed": mixed_space, "hpl": hpl_space}[which]()
    e = engine(space, seed=71)
    e.gp_set_precision(prec)
    pop = ode.population_init(space, 3000, seed=12)
    F = features(space, pop)
    d = F.shape[0]
    rng = np.random.default_rng(3)
    X = features(space, ode.population_init(space, 200, seed=13)).T.copy()
    y = rng.normal(size=200)
    ell = rng.uniform(0.5, 2.0, size=d)
    e.gp_fit(X, y, lengthscale=ell, sigma_f2=1.0, sigma_n2=1e-6, jitter=1e-8)
    dup = np.zeros(3000, np.uint8)
    dup[::17] = 1
    vals, dupd = dev(pop), dev(dup)
    mu0, var0, s0 = e.gp_score(e.encode(vals), dup=dupd)
    mu1, var1, s1 = e.gp_score_values(vals, dup=dupd)
    # the two entry points share the K* / variance kernels: equal to rounding
    # of the fused encode (fp64) or of the reduced-precision contractions
    same = 1e-12 if prec == 64 else 1e-6
    for a, b in ((mu0, mu1), (var0, var1), (s0, s1)):
        np.testing.assert_allclose(b.cpu().numpy(), a.cpu().numpy(), rtol=same, atol=same)
    mu, var = ogp.GP(X, y, lengthscale=ell, sigma_f2=1.0, sigma_n2=1e-6, jitter=1e-8).posterior(F.T)
    tol = (RTOL, ATOL) if prec == 64 else (1e-3, 1e-3)
    np.testing.assert_allclose(mu1.cpu().numpy(), mu, rtol=tol[0], atol=tol[1])
    np.testing.assert_allclose(var1.cpu().numpy(), var, rtol=tol[0], atol=tol[1])


def test_chol_fused_refit_bitwise_and_not_pd():
    """the fused refit (k_chol_update_diag factors the next diagonal block
    inside the trailing update; default from 2048 padded rows) gives bitwise
    the factor of the unfused chain (UT_CHOL_FUSE=0 vs 1: the posterior and
    EI of a batch are bitwise equal), and a kernel matrix that is not positive
    definite in a block the fused kernel factors is flagged (gp_fit_ok() is
    False, every score NaN, nothing selected) -- ADVICE r3"""
    _require_gpu()
    rng = np.random.default_rng(41)
    n, d = 2200, 6
    X = rng.uniform(size=(n, d))
    y = np.sum((X - 0.4) ** 2, axis=1)
    U = torch.from_numpy(np.ascontiguousarray(rng.uniform(size=(d, 3000)))).cuda()
    U[:, :5] = torch.from_numpy(np.ascontiguousarray(X[:5].T)).cuda()
    space = [Param("f%d" % i, FLOAT, 0.0, 1.0) for i in range(d)]
    old = os.environ.get("UT_CHOL_FUSE")
    outs = []
    try:
        for fuse in ("0", "1"):
            os.environ["UT_CHOL_FUSE"] = fuse
            e = engine(space, seed=2)
            e.gp_fit(X, y, lengthscale=0.3, sigma_f2=1.0, sigma_n2=1e-6, jitter=1e-8)
            outs.append([t.cpu() for t in e.gp_score(U, acq=e.acq("ei"))])
            e.close()
        for a, b in zip(*outs):
            assert torch.equal(a, b)
        # not PD from block row 2100 on: rows 2100.. repeat rows 0..99 (the Schur
        # complement there is ~0) and the diagonal carries -0.5
        X2 = X.copy()
        X2[2100:] = X[:100]
        os.environ["UT_CHOL_FUSE"] = "1"
        e = engine(space, seed=2)
        e.gp_fit(X2, y, lengthscale=0.05, sigma_f2=1.0, sigma_n2=-0.5, jitter=0.0, wait=False)
        _, _, score = e.gp_score(U, acq=e.acq("ei"))       # enqueued behind the failing fit: NaN
        idx, _ = e.topk(score, 8)
        assert torch.isnan(score).all()
        assert idx.cpu().tolist() == [-1] * 8
        assert not e.gp_fit_ok()
        from uptune_amd._lib import UthotError
        with pytest.raises(UthotError):                     # no usable fit until a new one succeeds
            e.gp_score(U, acq=e.acq("ei"))
        # the same matrix with its duplicates removed is PD on the fused path
        e.gp_fit(X2[:2100], y[:2100], lengthscale=0.05, sigma_f2=1.0, sigma_n2=-0.5, jitter=0.0, wait=False)
        assert e.gp_fit_ok()
        e.close()
    finally:
        if old is None:
            os.environ.pop("UT_CHOL_FUSE", None)
        else:
            os.environ["UT_CHOL_FUSE"] = old


def test_trinv_big_bitwise():
    """k_trinv_big (L^-1 levels of 256 rows and up on 128 x 128 tiles) gives
    bitwise the inverse of k_trinv_level's 64 x 64 tiles (UT_TRINV_BIG=0 vs 1:
    the posterior and EI of a batch are bitwise equal), with a ragged last
    pair (npad 2304: level 2048 pairs 2048 rows with 256), and the posterior
    matches the oracle"""
    _require_gpu()
    rng = np.random.default_rng(43)
    n, d = 2200, 6
    X = rng.uniform(size=(n, d))
    y = np.sum((X - 0.4) ** 2, axis=1)
    U = torch.from_numpy(np.ascontiguousarray(rng.uniform(size=(d, 3000)))).cuda()
    U[:, :5] = torch.from_numpy(np.ascontiguousarray(X[:5].T)).cuda()
    space = [Param("f%d" % i, FLOAT, 0.0, 1.0) for i in range(d)]
    old = os.environ.get("UT_TRINV_BIG")
    outs = []
    try:
        for big in ("0", "1"):
            os.environ["UT_TRINV_BIG"] = big
            e = engine(space, seed=2)
            e.gp_fit(X, y, lengthscale=0.3, sigma_f2=1.0, sigma_n2=1e-6, jitter=1e-8)
            outs.append([t.cpu() for t in e.gp_score(U, acq=e.acq("ei"))])
            e.close()
    finally:
        if old is None:
            os.environ.pop("UT_TRINV_BIG", None)
        else:
            os.environ["UT_TRINV_BIG"] = old
    for a, b in zip(*outs):
        assert torch.equal(a, b)
    mu, var = ogp.GP(X, y, lengthscale=0.3, sigma_f2=1.0, sigma_n2=1e-6, jitter=1e-8).posterior(U.cpu().numpy().T)
    np.testing.assert_allclose(outs[1][0].numpy(), mu, rtol=RTOL, atol=ATOL)
    np.testing.assert_allclose(outs[1][1].numpy(), var, rtol=RTOL, atol=ATOL)


@pytest.mark.parametrize("n", [300, 2200])
def test_chol_merged_bitwise(n):
    """the diagonal blocks' inverse solved inside the Cholesky column loop
    (UT_CHOL_MERGED=1, the default) gives bitwise the factor and inverse of the
    separate substitution sweep (=0): unfused k_chol_diag at n = 300, the
    fused k_chol_update_diag at n = 2200 (posterior and EI bitwise equal),
    and an appended fit on top of each matches its refit within RTOL"""
    _require_gpu()
    rng = np.random.default_rng(47)
    d = 6
    X = rng.uniform(size=(n + 40, d))
    y = np.sum((X - 0.4) ** 2, axis=1)
    U = torch.from_numpy(np.ascontiguousarray(rng.uniform(size=(d, 2000)))).cuda()
    space = [Param("f%d" % i, FLOAT, 0.0, 1.0) for i in range(d)]
    old = os.environ.get("UT_CHOL_MERGED")
    outs = []
    try:
        for merged in ("0", "1"):
            os.environ["UT_CHOL_MERGED"] = merged
            e = engine(space, seed=2)
            e.gp_fit(X[:n], y[:n], lengthscale=0.3, sigma_f2=1.0, sigma_n2=1e-6, jitter=1e-8)
            full = [t.cpu() for t in e.gp_score(U, acq=e.acq("ei"))]
            e.gp_fit(X, y, lengthscale=0.3, sigma_f2=1.0, sigma_n2=1e-6, jitter=1e-8)   # appended rows
            outs.append((full, [t.cpu() for t in e.gp_score(U, acq=e.acq("ei"))]))
            e.close()
    finally:
        if old is None:
            os.environ.pop("UT_CHOL_MERGED", None)
        else:
            os.environ["UT_CHOL_MERGED"] = old
    for a, b in zip(outs[0][0], outs[1][0]):
        assert torch.equal(a, b)
    mu, var = ogp.GP(X, y, lengthscale=0.3, sigma_f2=1.0, sigma_n2=1e-6, jitter=1e-8).posterior(U.cpu().numpy().T)
    for app in (outs[0][1], outs[1][1]):
        np.testing.assert_allclose(app[0].numpy(), mu, rtol=RTOL, atol=ATOL)
        np.testing.assert_allclose(app[1].numpy(), var, rtol=RTOL, atol=ATOL)


@pytest.mark.parametrize("which", ["hpl", "gcc", "mixed", "perm"])
@pytest.mark.parametrize("prec", [64, 32, 16, 8])
def test_categorical_kstar_equals_dense(which, prec):
    """The categorical K* (ENUM / BOOL one-hot blocks as an int8 code product on
    v_mfma_i32_16x16x64_i8, the other features on the fp64 contraction) gives
    the dense contraction's posterior: ut_gp_score_values (categorical, the
    library's own encoding) against ut_gp_score on the same candidates' feature
    matrix (dense), and the oracle GP.  fp64 within 1e-9 relative / 1e-10
    absolute of the dense path (only the fp summation order of the distances
    differs; the mean's cancellation magnifies it near mu = 0), lower tiers at
    their 1e-3 tolerance against the oracle."""
    _require_gpu()
    from uptune_amd import spaces
    space = {"hpl": hpl_space, "mixed": mixed_space, "perm": perm_space,
             "gcc": lambda: oracle_space(spaces.gcc())}[which]()
    e = engine(space, seed=9)
    e.gp_set_precision(prec)
    n, m = (700, 5000) if which != "gcc" else (400, 3000)
    tr = ode.population_init(space, n, seed=8)
    X = features(space, tr).T
    y = np.sum((X - 0.35) ** 2, axis=1)
    ell = {"hpl": 1.0, "gcc": 2.0, "mixed": 0.7, "perm": 0.9}[which]
    e.gp_fit(X, y, lengthscale=ell, sigma_f2=1.0, sigma_n2=1e-6, jitter=1e-8)
    assert e.gp_kstar_mode() == "categorical"
    cand = ode.population_init(space, m, seed=7)
    cand[:, :20] = tr[:, :20]                  # candidates on training points (var ~ 0)
    vals = dev(cand)
    mu_c, var_c, sc_c = [t.cpu().numpy() for t in e.gp_score_values(vals, acq=e.acq("ei"))]
    mu_d, var_d, sc_d = [t.cpu().numpy() for t in e.gp_score(e.encode(vals), acq=e.acq("ei"))]
    g = ogp.GP(X, y, lengthscale=ell, sigma_f2=1.0, sigma_n2=1e-6, jitter=1e-8)
    wmu, wvar = g.posterior(features(space, cand).T)
    ei = ogp.acquisition(wmu, wvar, g.f_best)
    if prec in (64, 8):
        np.testing.assert_allclose(mu_c, mu_d, rtol=1e-9, atol=1e-10)
        np.testing.assert_allclose(var_c, var_d, rtol=1e-9, atol=1e-10)
        np.testing.assert_allclose(sc_c, sc_d, rtol=1e-9, atol=1e-10)
        tol = dict(rtol=RTOL, atol=ATOL)
        np.testing.assert_allclose(mu_c, wmu, **tol)
        np.testing.assert_allclose(var_c, wvar, **tol)
        np.testing.assert_allclose(sc_c, ei, **tol)
    else:
        # the fp32 / f16x3 variance of a candidate ON a training point is a
        # cancellation 1 - (1 - 1e-6) in f32: the tier's error there is the
        # dense path's too, so the categorical K* must be as good as dense
        # (its K* differs from dense only in fp64 summation order, below the
        # f32 rounding of the stored K*)
        def err(a, b):
            return float(np.max(np.abs(a - b) / (1e-5 + 1e-3 * np.abs(b))))
        for got, dense, want in ((mu_c, mu_d, wmu), (var_c, var_d, wvar), (sc_c, sc_d, ei)):
            assert err(got, want) <= max(1.0, 1.25 * err(dense, want)), (err(got, want), err(dense, want))


def test_categorical_kstar_too_many_options_is_dense():
    """the candidates' code rows of an ENUM with thousands of options
    need more LDS than one workgroup holds (code_rows_lds(cat_k) > the device's
    hipDeviceAttributeMaxSharedMemoryPerBlock); the fit then scores with the
    dense contraction instead of failing at launch, and the posterior is the
    oracle's"""
    _require_gpu()
    space = [Param("big", ENUM, options=list(range(5000))), Param("x", FLOAT, 0.0, 1.0), Param("b", BOOL)]
    e = engine(space, seed=5)
    tr = ode.population_init(space, 300, seed=5)
    X = features(space, tr).T
    y = np.sum((X - 0.3) ** 2, axis=1)
    e.gp_fit(X, y, lengthscale=1.0, sigma_f2=1.0, sigma_n2=1e-6, jitter=1e-8)
    assert e.gp_kstar_mode() == "dense"
    cand = ode.population_init(space, 1500, seed=6)
    cand[:, :5] = tr[:, :5]
    mu, var, _ = [t.cpu().numpy() for t in e.gp_score_values(dev(cand), acq=e.acq("ei"))]
    g = ogp.GP(X, y, lengthscale=1.0, sigma_f2=1.0, sigma_n2=1e-6, jitter=1e-8)
    wmu, wvar = g.posterior(features(space, cand).T)
    np.testing.assert_allclose(mu, wmu, rtol=RTOL, atol=ATOL)
    np.testing.assert_allclose(var, wvar, rtol=RTOL, atol=1e-8)


def test_categorical_kstar_fallbacks():
    """the dense contraction when the categorical form does not apply: a
    training row whose ENUM block is not one-hot, per-feature lengthscales
    that differ inside the categorical features, UT_CAT_KSTAR=0 -- the
    posterior is the oracle's either way; a later fit with clean rows goes back
    to the categorical form, and an appended fit re-checks only its new rows"""
    _require_gpu()
    space = hpl_space()
    e = engine(space, seed=4)
    tr = ode.population_init(space, 300, seed=3)
    X = features(space, tr).T
    y = np.sum((X - 0.5) ** 2, axis=1)
    cand = dev(ode.population_init(space, 2000, seed=2))
    F = X.shape[1]

    def check(Xf, ell):
        g = ogp.GP(Xf, y[:Xf.shape[0]], lengthscale=ell, sigma_f2=1.0, sigma_n2=1e-6, jitter=1e-8)
        mu, var = g.posterior(features(space, cand.cpu().numpy()).T)
        m2, v2, _ = e.gp_score_values(cand, acq=e.acq("ei"))
        np.testing.assert_allclose(m2.cpu().numpy(), mu, rtol=RTOL, atol=ATOL)
        np.testing.assert_allclose(v2.cpu().numpy(), var, rtol=RTOL, atol=ATOL)

    Xb = X.copy()
    enum_p = next(p for p in e.spec.params if p.kind == 5)
    enum_col = enum_p.feat_col
    Xb[7, enum_col] = 0.5                       # not one-hot
    e.gp_fit(Xb, y, lengthscale=1.0, sigma_f2=1.0, sigma_n2=1e-6, jitter=1e-8)
    assert e.gp_kstar_mode() == "dense"
    check(Xb, 1.0)
    ell = np.ones(F)
    ell[enum_col + 1] = 1.5                     # two lengthscales inside the categorical features
    e.gp_fit(X, y, lengthscale=ell, sigma_f2=1.0, sigma_n2=1e-6, jitter=1e-8)
    assert e.gp_kstar_mode() == "dense"
    check(X, ell)
    e.gp_fit(X[:200], y[:200], lengthscale=1.0, sigma_f2=1.0, sigma_n2=1e-6, jitter=1e-8)
    assert e.gp_kstar_mode() == "categorical"
    check(X[:200], 1.0)
    e.gp_fit(X[:250], y[:250], lengthscale=1.0, sigma_f2=1.0, sigma_n2=1e-6, jitter=1e-8)   # appends
    assert e.gp_last_fit_kind() == "append" and e.gp_kstar_mode() == "categorical"
    check(X[:250], 1.0)
    Xc = X.copy()
    Xc[280, enum_col:enum_col + enum_p.n_feat] = 0.0   # an all-zero block in an appended row
    e.gp_fit(Xc, y, lengthscale=1.0, sigma_f2=1.0, sigma_n2=1e-6, jitter=1e-8)
    assert e.gp_kstar_mode() == "dense"
    check(Xc, 1.0)
    e.close()
    old = os.environ.get("UT_CAT_KSTAR")
    os.environ["UT_CAT_KSTAR"] = "0"
    try:
        e2 = engine(space, seed=4)
        e2.gp_fit(X, y, lengthscale=1.0, sigma_f2=1.0, sigma_n2=1e-6, jitter=1e-8)
        assert e2.gp_kstar_mode() == "dense"
        e2.close()
    finally:
        if old is None:
            os.environ.pop("UT_CAT_KSTAR", None)
        else:
            os.environ["UT_CAT_KSTAR"] = old
