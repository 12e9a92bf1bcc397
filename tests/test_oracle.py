"""The oracle against the reference's own data and standard KATs (CPU)."""
import hashlib
import json
import os
import random

import numpy as np

from oracle import de as ode
from oracle import gp as ogp
from oracle import hashing as oh
from oracle import philox as ph
from oracle import select as osel
from oracle.space import BOOL, ENUM, FLOAT, INT, Param, from_f64, get_unit_value, set_unit_value


def test_tutorial_db_hashes_pin_layout(golden_dir):
    """9 Configuration.hash values stored by the reference's tutorial run
    (samples/tutorials/tuneup.opentuner.db) are reproduced exactly by the
    Python-2 outer-message layout."""
    d = json.load(open(os.path.join(golden_dir, "tutorial_db_hashes.json")))
    space = [Param("BLOCK_SIZE", INT, 1, 10)]
    assert len(d["rows"]) == 9
    for r in d["rows"]:
        assert oh.hash_config(space, [r["BLOCK_SIZE"]], py2=True) == r["hash"]
    # and the py3 layout (uptune's port) differs only by the b'' wrapper
    msg = oh.outer_message(space, [3])
    assert msg.startswith(b"BLOCK_SIZEb'") and msg.endswith(b"'0|")


def test_py3_layout_matches_reference_expression():
    """str(bytes) wrapper of manipulator.py:240/459 under Python 3"""
    inner = hashlib.sha256(repr(2.5).encode("utf-8")).hexdigest().encode()
    m = hashlib.sha256()
    m.update(str("x").encode())
    m.update(str(inner).encode())
    m.update(str(0).encode())
    m.update(b"|")
    assert oh.hash_config([Param("x", FLOAT, 0.0, 5.0)], [2.5]) == m.hexdigest()


def test_sha256_fips_vectors():
    assert hashlib.sha256(b"abc").hexdigest() == "ba7816bf8f01cfea414140de5dae2223b00361a396177a9cb410ff61f20015ad"
    assert hashlib.sha256(b"").hexdigest() == "e3b0c44298fc1c149afbf4c8996fb92427ae41e4649b934ca495991b7852b855"


def test_philox_random123_kats():
    cases = [((0, 0, 0, 0), (0, 0), (0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8)),
             ((0xffffffff,) * 4, (0xffffffff,) * 2, (0x408f276d, 0x41c83b0e, 0xa20bc7c6, 0x6d5451fd)),
             ((0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344), (0xa4093822, 0x299f31d0),
              (0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1))]
    for c, k, want in cases:
        got = ph.philox4x32_10(*c, *k)
        assert tuple(int(x) for x in got) == want


def test_mulhi64():
    rng = random.Random(0)
    a = [rng.getrandbits(64) for _ in range(200)]
    b = [rng.getrandbits(63) + 1 for _ in range(200)]
    got = ph.mulhi64(np.array(a, dtype=np.uint64), np.array(b, dtype=np.uint64))
    assert [int(x) for x in got] == [(x * y) >> 64 for x, y in zip(a, b)]


def test_unit_value_roundtrip_int():
    p = Param("n", INT, 1, 10)
    for v in range(1, 11):
        u = get_unit_value(p, v)
        assert set_unit_value(p, u, None) == v


def _space():
    return [Param("x", FLOAT, -5.0, 5.0), Param("n", INT, 1, 64), Param("flag", BOOL),
            Param("mode", ENUM, options=["a", "b", "c", 4]), Param("y", FLOAT, 0.0, 1.0),
            Param("big", INT, -100000, 2000000)]


def test_de_scalar_equals_vectorised():
    space = _space()
    pop = ode.population_init(space, 16, seed=11)
    trial = ode.propose_de_vec(space, pop, seed=11, round_=3, cand_base=5, m=48, cr=0.5, n_cross=1)
    pop_cfgs = [[from_f64(p, pop[j, i]) for j, p in enumerate(space)] for i in range(16)]
    for i in range(48):
        cfg = ode.propose_de_scalar(space, pop_cfgs, 11, 3, 5 + i, 0.5, 1)
        assert [from_f64(p, trial[j, i]) for j, p in enumerate(space)] == cfg


def test_de_golden(golden_dir):
    z = np.load(os.path.join(golden_dir, "de_mixed.npz"))
    space = _space()
    pop = ode.population_init(space, 16, seed=11)
    np.testing.assert_array_equal(pop, z["pop"])
    trial = ode.propose_de_vec(space, pop, seed=11, round_=3, cand_base=5, m=48, cr=0.5, n_cross=1)
    np.testing.assert_array_equal(trial, z["trial"])


def test_de_invariants():
    space = _space()
    pop = ode.population_init(space, 64, seed=1)
    trial = ode.propose_de_vec(space, pop, seed=1, round_=0, cand_base=0, m=256, cr=0.2, n_cross=1)
    assert np.all((trial[0] >= -5.0) & (trial[0] <= 5.0))
    assert np.all(trial[1] == np.round(trial[1])) and np.all((trial[1] >= 1) & (trial[1] <= 64))
    assert set(np.unique(trial[2])) <= {0.0, 1.0}
    assert set(np.unique(trial[3])) <= {0.0, 1.0, 2.0, 3.0}
    # donors are distinct and differ from the target
    t, d1, d2, d3 = ode.donors(np.arange(4096, dtype=np.uint64), 7, seed=9, round_=2)
    st = np.stack([t, d1, d2, d3])
    assert all(len(set(st[:, i])) == 4 for i in range(st.shape[1]))
    assert st.min() >= 0 and st.max() < 7
    # at least one param changes per trial (n_cross=1) unless the forced op is a no-op
    forced = ode.forced_mask(np.arange(256, dtype=np.uint64), len(space), 1, 1, 0)
    assert np.all(forced.sum(axis=0) == 1)


def test_de_information_sharing():
    """donor pool = population - {target} + [best] * information_sharing
    (differentialevolution.py:110-118): the scalar restatement (written like the
    reference, over config lists) equals the vectorised one; without a best
    result the pool is the population alone and the trials are unchanged; with
    a 30-member population the best is among the 3 donors 3/30 of the time."""
    space = _space()
    pop = ode.population_init(space, 30, seed=12)
    best = ode.population_init(space, 1, seed=99)[:, 0]
    pop_cfgs = [[from_f64(p, pop[j, i]) for j, p in enumerate(space)] for i in range(30)]
    best_cfg = [from_f64(p, best[j]) for j, p in enumerate(space)]
    for share in (1, 3):
        trial = ode.propose_de_vec(space, pop, 12, 4, 7, 64, 0.6, 1, best=best, information_sharing=share)
        for i in range(64):
            cfg = ode.propose_de_scalar(space, pop_cfgs, 12, 4, 7 + i, 0.6, 1, best_cfg=best_cfg,
                                        information_sharing=share)
            assert [from_f64(p, trial[j, i]) for j, p in enumerate(space)] == cfg
    np.testing.assert_array_equal(ode.propose_de_vec(space, pop, 12, 4, 7, 64, 0.6, 1, best=None),
                                  ode.propose_de_vec(space, pop, 12, 4, 7, 64, 0.6, 1))
    np.testing.assert_array_equal(ode.propose_de_vec(space, pop, 12, 4, 7, 64, 0.6, 1, best=best,
                                                     information_sharing=0),
                                  ode.propose_de_vec(space, pop, 12, 4, 7, 64, 0.6, 1))
    g = np.arange(200000, dtype=np.uint64)
    t, d1, d2, d3 = ode.donors(g, 30, seed=3, round_=1, share=1)
    st = np.stack([d1, d2, d3])
    frac = np.mean((st < 0).any(axis=0))
    assert abs(frac - 3.0 / 30.0) < 0.004, frac
    assert np.all((st < 0).sum(axis=0) <= 1)                   # one best copy: at most one best donor
    assert np.all((st != t) | (st < 0))
    # share = 5 copies: distinct POSITIONS, so several donors may be the best
    _, e1, e2, e3 = ode.donors(g[:20000], 4, seed=3, round_=1, share=5)
    assert np.any((np.stack([e1, e2, e3]) < 0).sum(axis=0) == 3)


def test_r64_hash_golden(golden_dir):
    z = np.load(os.path.join(golden_dir, "r64_hashes.npz"))
    space = [Param(d, FLOAT, -1000.0, 1000.0) for d in range(64)]
    vals = z["values"]
    for j in range(vals.shape[1]):
        assert oh.hash_config(space, list(vals[:, j])) == z["hashes"][j]
    # outer message length is constant: 4588 bytes for R64
    assert len(oh.outer_message(space, list(vals[:, 0]))) == 4588


def test_gcc_hash_golden(golden_dir):
    d = json.load(open(os.path.join(golden_dir, "gcc_space.json")))
    vals = np.load(os.path.join(golden_dir, "gcc_rows.npz"))["values"]
    space = []
    for ptype, name, rng in d["params"]:
        if ptype == "EnumParameter":
            space.append(Param(name, ENUM, options=list(rng)))
        else:
            space.append(Param(name, INT, rng[0], rng[1]))
    assert len(space) == 339
    for j, h in enumerate(d["hashes_py3"][:16]):
        cfg = [from_f64(p, vals[i, j]) for i, p in enumerate(space)]
        assert oh.hash_config(space, cfg) == h
    assert len(oh.outer_message(space, cfg)) == 30178


def test_gp_golden(golden_dir):
    z = np.load(os.path.join(golden_dir, "gp_small.npz"))
    g = ogp.GP(z["X"], z["y"], lengthscale=0.3, sigma_f2=1.0, sigma_n2=1e-6, jitter=1e-8)
    mu, var = g.posterior(z["U"])
    np.testing.assert_allclose(mu, z["mu"], rtol=1e-12, atol=1e-12)
    np.testing.assert_allclose(var, z["var"], rtol=1e-9, atol=1e-12)
    # posterior at training points: small variance, mean ~ ys
    assert np.all(var[:4] < 1e-4)
    np.testing.assert_allclose(mu[:4], g.ys[:4], atol=1e-3)


def test_ei_properties():
    mu = np.array([0.0, -1.0, 1.0, 0.0])
    var = np.array([1.0, 1.0, 1.0, 0.0])
    ei = ogp.acquisition(mu, var, f_best=0.0)
    assert ei[1] > ei[0] > ei[2] > 0
    assert ei[3] == 0.0


def test_topk_and_dedup_semantics():
    s = [0.5, 0.9, 0.9, float("nan"), 0.1, 0.9]
    assert osel.topk(s, 3) == [1, 2, 5]
    assert osel.topk(s, 3, dup=[0, 1, 0, 0, 0, 0]) == [2, 5, 0]
    assert osel.topk(s, 8, cand_base=10)[-2:] == [-1, -1]
    assert osel.dedup(["a", "b", "a", "c"], history={"c"}) == [0, 0, 1, 1]


# ---------------------------------------------------------------- scaled kinds
def _scaled_space():
    from oracle.space import LOGINT, POW2
    return [Param("li", LOGINT, 1, 1000), Param("li0", LOGINT, 0, 1 << 30), Param("p2", POW2, 1, 1 << 20),
            Param("x", FLOAT, -5.0, 5.0), Param("p2s", POW2, 256, 256), Param("n", INT, -3, 40)]


def test_logint_pow2_reference_semantics():
    """get_value / legal_range / unit round trip of LogIntegerParameter and
    PowerOfTwoParameter (manipulator.py:778-836), written out from the source"""
    import math
    from oracle.space import LOGINT, POW2, scale
    li = Param("li", LOGINT, 1, 1000)
    lo, hi = li.legal_range()
    assert lo == math.log(1.0 - 0.4999 + 1.0 - 1.0, 2.0) and hi == math.log(1000.0 + 0.4999 + 1.0 - 1.0, 2.0)
    for v in range(1, 1001):
        assert scale(li, v) == math.log(v + 1.0 - 1.0, 2.0)
        assert set_unit_value(li, get_unit_value(li, v), None) == v
    p2 = Param("p2", POW2, 1, 1 << 20)
    assert p2.legal_range() == (0, 20)
    for e in range(21):
        assert scale(p2, 1 << e) == e
        assert set_unit_value(p2, get_unit_value(p2, 1 << e), None) == 1 << e
    # hash_value = sha256(repr(get_value)): a float for LogInteger, the exponent for PowerOfTwo
    h = hashlib.sha256(repr(math.log(7 + 1.0 - 1.0, 2.0)).encode()).hexdigest().encode()
    assert oh.hash_value(li, 7, py2=True) == h.decode()
    assert oh.hash_value(p2, 1 << 13, py2=True) == hashlib.sha256(b"13").hexdigest()


def test_scaled_kinds_de_scalar_equals_vectorised():
    space = _scaled_space()
    pop = ode.population_init(space, 32, seed=5)
    trial = ode.propose_de_vec(space, pop, seed=5, round_=2, cand_base=9, m=64, cr=0.7, n_cross=1)
    pop_cfgs = [[from_f64(p, pop[j, i]) for j, p in enumerate(space)] for i in range(32)]
    for i in range(64):
        cfg = ode.propose_de_scalar(space, pop_cfgs, 5, 2, 9 + i, 0.7, 1)
        assert [from_f64(p, trial[j, i]) for j, p in enumerate(space)] == cfg
    # stored values stay legal: ints in range, powers of two
    assert np.all((trial[0] >= 1) & (trial[0] <= 1000)) and np.all(trial[0] == np.round(trial[0]))
    assert np.all(np.frexp(trial[2])[0] == 0.5) and np.all(trial[4] == 256.0)


def test_scaled_kinds_pso_ga_legal():
    from oracle import ga as oga
    from oracle import pso as opso
    space = _scaled_space()
    pop = ode.population_init(space, 64, seed=6)
    x, v = opso.propose_pso_vec(space, pop, np.zeros_like(pop), pop, pop[:, 3], seed=6, round_=1, cand_base=0, m=64)
    y, inv = oga.propose_ga_vec(space, pop[:, 0], None, seed=6, round_=1, cand_base=0, m=64, mutation_rate=0.3,
                                normal=True)
    for out in (x, y):
        assert np.all((out[0] >= 1) & (out[0] <= 1000)) and np.all(out[0] == np.round(out[0]))
        assert np.all((out[1] >= 0) & (out[1] <= 1 << 30))
        assert np.all(np.frexp(out[2])[0] == 0.5) and np.all((out[2] >= 1) & (out[2] <= 1 << 20))


def test_de_at_equals_vectorised():
    """propose_de_at (the bench's parity check: only the members a trial reads)
    equals the full vectorised round at those global indices, on the HPL-64
    mixed space and a permutation space"""
    from tests._spaces import oracle_space
    from uptune_amd import spaces
    for manip in (spaces.hpl64(), spaces.perm_mixed()):
        space = oracle_space(manip)
        npop, m = 300, 700
        pop = ode.population_init(space, npop, 5)
        full = ode.propose_de_vec(space, pop, 5, 3, 0, m, 0.2, 1)
        g = np.array([0, 1, 299, 300, 301, 512, 699])
        assert np.array_equal(ode.propose_de_at(space, g, npop, 5, 3, 0.2, 1), full[:, g])
        mem = np.array([0, 1, 299, 7])
        assert np.array_equal(ode.population_init(space, npop, 5, members=mem), pop[:, mem])


def test_raytracer_history_fixture(golden_dir):
    """the second C4 history (samples/gcc-options/raytracer-record.csv decoded
    into the gcc_space.json space): values inside the params.def ranges, and
    the committed digests are the oracle's hash_config of its first rows"""
    import json
    z = np.load(os.path.join(golden_dir, "gcc_raytracer_history.npz"))
    sp = json.load(open(os.path.join(golden_dir, "gcc_space.json")))
    v = z["values"]
    assert v.shape == (len(sp["params"]), 2269) and z["qor"].shape == (2269,)
    from oracle.space import ENUM, INT, Param, from_f64
    from oracle import hashing as oh
    space = [Param(n, ENUM, options=["on", "off", "default"]) if k == "EnumParameter" else Param(n, INT, *r)
             for k, n, r in sp["params"]]
    for j, p in enumerate(space):
        if p.kind == INT:
            assert p.lo <= v[j].min() and v[j].max() <= p.hi
        else:
            assert set(np.unique(v[j])) <= {0.0, 1.0, 2.0}
    for c in range(8):
        assert oh.hash_config(space, [from_f64(p, v[i, c]) for i, p in enumerate(space)]) == z["hashes_py3"][c]
