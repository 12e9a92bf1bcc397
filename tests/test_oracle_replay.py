"""The reference-ordered restatements (oracle/replay.py: HybridParticle.move,
pso.py:70-77; EvolutionaryTechnique / GGA desired_configuration,
evolutionarytechniques.py:29-61, globalGA.py:28-85) fed the build's counter
draws reproduce the batch oracles (oracle/pso.py, oracle/ga.py) -- and hence
the device kernels the GPU parity tests pin to them -- candidate for candidate.
The batch forms therefore follow the reference's control flow; they differ
only in where their random numbers come from.  The same restatements also run
on CPython's MT19937 stream (MTDraws), consuming it in the reference's order.
"""
import random

import numpy as np
import pytest

from oracle import ga as oga
from oracle import perm as pm
from oracle import philox as ph
from oracle import pso as opso
from oracle import replay as rp
from oracle.space import ENUM, PERM, columns, from_f64, to_f64, width  # noqa: F401
from tests._spaces import oracle_space


def _spaces():
    from uptune_amd import spaces
    return {"hpl64": oracle_space(spaces.hpl64()), "perm": oracle_space(spaces.perm_mixed())}


def _row(space, soa, j):
    """stored values of column j (PERM: item-index lists)"""
    starts, _ = columns(space)
    return [[int(a) for a in soa[c:c + width(p), j]] if p.kind == PERM else from_f64(p, soa[c, j])
            for p, c in zip(space, starts)]


def _soa_col(space, row):
    out = []
    for p, v in zip(space, row):
        out.extend([float(a) for a in v] if p.kind == PERM else [to_f64(p, v)])
    return np.array(out)


@pytest.mark.parametrize("name", ["hpl64", "perm"])
def test_pso_move_scalar_equals_batch(name):
    space = _spaces()[name]
    rng = np.random.default_rng(4)
    seed, rnd, npop, m = 17, 5, 40, 120
    from oracle import de as ode
    pos = ode.population_init(space, npop, seed)
    pbest = ode.population_init(space, npop, seed + 1)
    gbest = ode.population_init(space, 1, seed + 2)[:, 0]
    vel = np.zeros_like(pos)
    starts, _ = columns(space)
    for p, c in zip(space, starts):
        if p.kind not in (PERM, ENUM):
            vel[c] = rng.normal(size=npop) * 0.3
    for xop in (pm.X_OX1, pm.X_OX3, pm.X_PX, pm.X_PMX, pm.X_CX):
        wx, wv = opso.propose_pso_vec(space, pos, vel, pbest, gbest, seed, rnd, 3, m, crossover=xop)
        for j in range(m):
            g = 3 + j
            t = g % npop
            vin = [0.0 if p.kind == PERM else float(vel[c, t]) for p, c in zip(space, starts)]
            x, v = rp.pso_move_scalar(space, _row(space, pos, t), vin, _row(space, pbest, t),
                                      _row(space, gbest[:, None], 0), rp.CounterDraws(seed, g, rnd, ph.OP_PSO),
                                      xchoice=xop)
            np.testing.assert_array_equal(_soa_col(space, x), wx[:, j])
            for p, c, vv in zip(space, starts, v):
                if p.kind != PERM:
                    assert float(vv) == wv[c, j], (p.name, j)


GA_CASES = [
    dict(mutation_rate=0.1),
    dict(mutation_rate=0.3, must_mutate_count=2),
    dict(mutation_rate=0.05, normal=True, sigma=0.1),
    dict(mutation_rate=0.1, crossover_rate=0.5, crossover_strength=0.2, normal=True),        # GGA
    dict(mutation_rate=0.1, crossover_rate=0.8, crossover=pm.X_OX3),                         # GA(crossover)
    dict(mutation_rate=0.1, crossover_rate=0.8, crossover=pm.X_PMX, max_retries=2),
    dict(mutation_rate=0.1, crossover_rate=0.8, crossover=pm.X_OX1),
    dict(mutation_rate=0.1, crossover_rate=0.8, crossover=pm.X_PX),
    dict(mutation_rate=0.1, crossover_rate=0.8, crossover=pm.X_CX),
]


@pytest.mark.parametrize("case", range(len(GA_CASES)))
@pytest.mark.parametrize("name", ["hpl64", "perm"])
@pytest.mark.parametrize("with_best", [True, False])
def test_ga_scalar_equals_batch(name, case, with_best):
    space = _spaces()[name]
    kw = dict(GA_CASES[case])
    from oracle import de as ode
    seed, rnd, m = 29, 3, 80
    best = ode.population_init(space, 2, seed + 5)
    p1 = best[:, 0] if with_best else None
    p2 = best[:, 1] if with_best and kw.get("crossover_rate", 0) > 0 else None
    op = ph.OP_GGA if kw.get("crossover_strength", 0) > 0 else ph.OP_GA
    want, winv = oga.propose_ga_vec(space, p1, p2, seed, rnd, 11, m, op=op, **kw)
    for j in range(m):
        d = rp.CounterDraws(seed, 11 + j, rnd, op)
        cfg, invalid = rp.ga_scalar(space, None if p1 is None else _row(space, best, 0), d,
                                    best2=None if p2 is None else _row(space, best, 1), **kw)
        np.testing.assert_array_equal(_soa_col(space, cfg), want[:, j])
        assert invalid == bool(winv[j]), j


def test_ga_retries_compound_and_exhaust():
    """a one-param Bool space under normal mutation (op1_flip): the forced
    mutation of the first retry always leaves the parent, so no candidate is
    invalid, with one retry or two (the batch form agrees)"""
    from oracle.space import BOOL, Param
    space = [Param("b", BOOL)]
    for g in range(20):
        d = rp.CounterDraws(1, g, 0, ph.OP_GA)
        cfg, inv = rp.ga_scalar(space, [True], d, normal=True, max_retries=1)
        assert (cfg, inv) == ([False], False)
        cfg, inv = rp.ga_scalar(space, [True], rp.CounterDraws(1, g, 0, ph.OP_GA), normal=True, max_retries=2)
        assert (cfg, inv) == ([False], False)
    want, winv = oga.propose_ga_vec(space, np.array([1.0]), None, 1, 0, 0, 20, normal=True, max_retries=1)
    assert np.all(want == 0.0) and not winv.any()


def test_mt_replay_consumes_reference_order():
    """MTDraws: the restatement runs on CPython's MT19937 stream in the
    reference's call order -- a Float particle moves with r1, r2 = the first
    two random() of the stream (FloatParameter.op3_swarm, manipulator.py:735-741)"""
    from oracle.space import FLOAT, INT, Param
    space = [Param("x", FLOAT, -10.0, 10.0)]
    r = random.Random(123)
    r1, r2 = r.random(), r.random()
    x, v = rp.pso_move_scalar(space, [1.0], [0.5], [2.0], [4.0], rp.MTDraws(random.Random(123)))
    want_v = 0.5 * 0.5 + (4.0 - 1.0) * 0.5 * r1 + (2.0 - 1.0) * 0.5 * r2
    assert v == [want_v] and x == [min(10.0, max(1.0 + want_v, -10.0))]
    # Integer: r1, r2, then gauss(s, sigma k) (:685-699)
    space = [Param("n", INT, 0, 100)]
    r = random.Random(5)
    r1, r2 = r.random(), r.random()
    vv = 0.0 * 0.5 + (60 - 10) * 0.5 * r1 + (10 - 10) * 0.5 * r2
    s = 100 / (1 + np.exp(-vv)) + 0
    p = r.gauss(s, 0.2 * 100)
    x, v = rp.pso_move_scalar(space, [10], [0.0], [10], [60], rp.MTDraws(random.Random(5)))
    assert v == [vv] and x == [int(min(100, max(round(p), 0)))]
    # GA: selection's random() first, then shuffle(params), then a coin per other param
    sp = _spaces()["hpl64"]
    parent = rp._manip_random(sp, rp.MTDraws(random.Random(1)), 2)    # manipulator.random() on MT
    a = rp.ga_scalar(sp, parent, rp.MTDraws(random.Random(9)), mutation_rate=0.2, crossover_rate=0.0)
    b = rp.ga_scalar(sp, parent, rp.MTDraws(random.Random(9)), mutation_rate=0.2, crossover_rate=0.0)
    assert a == b and a[1] is False and a[0] != parent


class _Trace(random.Random):
    """CPython's MT19937 with a log of the top-level calls the restatement
    makes (nested calls inside random.py are not logged)"""

    def __init__(self, seed):
        super().__init__(seed)
        self.log, self._depth = [], 0

    def _wrap(name):
        def f(self, *a, **k):
            if self._depth == 0:
                self.log.append(name)
            self._depth += 1
            try:
                return getattr(random.Random, name)(self, *a, **k)
            finally:
                self._depth -= 1
        return f

    def getrandbits(self, k):   # defined here so that random.Random keeps its getrandbits-based _randbelow
        return random.Random.getrandbits(self, k)

    random = _wrap("random")
    randint = _wrap("randint")
    uniform = _wrap("uniform")
    shuffle = _wrap("shuffle")
    choice = _wrap("choice")
    gauss = _wrap("gauss")
    normalvariate = _wrap("normalvariate")


def _word_for(v, a, b):
    """a 32-bit word that randint(word, a, b) maps to v: ceil((v - a) 2^32 / n)"""
    n = b - a + 1
    return -((-(v - a) << 32) // n)


@pytest.mark.parametrize("xop", [pm.X_OX1, pm.X_OX3, pm.X_PX, pm.X_CX, pm.X_PMX])
@pytest.mark.parametrize("S", [7, 10, 23])
def test_mt_cross_consumes_reference_randints(xop, S):
    """op3_cross_* on the MT stream (MTDraws.cross): the operator draws exactly
    the reference's random.randint calls, in its order (manipulator.py:1179-1353:
    PX randint(2, len); PMX / OX1 randint(0, len - d); CX randint(0, len - 1);
    OX3 r1 then r2 over (0, len - d)), and nothing else -- the same values fed
    to the counter form as words give the same child, and the stream is left
    where the reference leaves it"""
    ranges = {pm.X_OX1: ["s"], pm.X_PMX: ["s"], pm.X_OX3: ["s", "s"], pm.X_PX: ["px"], pm.X_CX: ["cx"]}[xop]
    for seed in range(25):
        g = random.Random(1000 + seed)
        p1, p2 = list(range(S)), list(range(S))
        g.shuffle(p1)
        g.shuffle(p2)
        d = S // 3
        t = _Trace(seed)
        child = rp.MTDraws(t).cross(xop, p1, p2, d)
        assert t.log == ["randint"] * len(ranges)
        assert sorted(child) == list(range(S))
        # the reference's calls on a fresh stream of the same seed
        r = random.Random(seed)
        bounds = {"s": (0, S - d), "px": (2, S), "cx": (0, S - 1)}
        vals = [(r.randint(*bounds[k]), bounds[k]) for k in ranges]
        words = [_word_for(v, a, b) for v, (a, b) in vals]
        assert [pm.randint(w, a, b) for w, (_, (a, b)) in zip(words, vals)] == [v for v, _ in vals]
        assert pm.cross(xop, p1, p2, d, words) == child
        assert t.random() == r.random()                     # the stream position agrees


def test_mt_pso_perm_swarm_order():
    """PermutationParameter.op3_swarm on MT (manipulator.py:1115-1140): uniform()
    > c decides a crossover, a second uniform() < c1 picks the global best
    (else the particle best), then op3_cross's randint calls -- and a particle
    that does not cross consumes one uniform() only"""
    from oracle.space import Param
    sp = [Param("p", PERM, options=list(range(9)))]
    seen = set()
    for seed in range(40):
        t = _Trace(seed)
        r = random.Random(seed)
        u1 = r.uniform(0, 1)
        x, _ = rp.pso_move_scalar(sp, [list(range(9))], [0.0], [[8, 7, 6, 5, 4, 3, 2, 1, 0]],
                                  [[1, 0, 3, 2, 5, 4, 7, 6, 8]], rp.MTDraws(t), xchoice=pm.X_OX3)
        if u1 > 0.5:
            assert t.log == ["uniform", "uniform", "randint", "randint"]
            u2 = r.uniform(0, 1)
            other = [1, 0, 3, 2, 5, 4, 7, 6, 8] if u2 < 0.5 else [8, 7, 6, 5, 4, 3, 2, 1, 0]
            assert x[0] == pm.cross(pm.X_OX3, list(range(9)), other, pm.swarm_d(9), r)
            seen.add(u2 < 0.5)
        else:
            assert t.log == ["uniform"] and x[0] == list(range(9))
    assert seen == {True, False}


def test_mt_ga_crossover_mixin_order():
    """GA(crossover=...) on MT (evolutionarytechniques.py:29-49, :72-78,
    :123-134): selection's random(), then op3_cross_<op> of every permutation
    param of size > 6 in the shared list's order (d = size // 3), then the
    first retry's shuffle(params)"""
    from uptune_amd import spaces
    sp = oracle_space(spaces.perm_mixed())
    big = [i for i, p in enumerate(sp) if p.kind == PERM and len(p.options) > 6]
    assert big
    from oracle import de as ode
    b = ode.population_init(sp, 2, 3)
    p1, p2 = _row(sp, b, 0), _row(sp, b, 1)
    for xop, per in ((pm.X_OX3, 2), (pm.X_PMX, 1), (pm.X_CX, 1), (pm.X_PX, 1), (pm.X_OX1, 1)):
        t = _Trace(7)
        cfg, inv = rp.ga_scalar(sp, p1, rp.MTDraws(t), best2=p2, mutation_rate=0.1, crossover_rate=1.0,
                                crossover=xop)
        assert t.log[0] == "random"
        assert t.log[1:1 + per * len(big)] == ["randint"] * (per * len(big))
        assert t.log[1 + per * len(big)] == "shuffle"


def test_mt_shared_params_list_carries_the_shuffle():
    """GA's random.shuffle(params) permutes the manipulator's ONE
    params list in place, so the next call shuffles the order the last one
    left.  MTDraws models the shared list: a second call on the same draw
    source equals a fresh draw source given the stream state AND the list order
    the first call left, and differs (for some seeds) from one that starts from
    the declaration order again"""
    sp = _spaces()["hpl64"]
    parent = rp._manip_random(sp, rp.MTDraws(random.Random(1)), 2)
    differs = 0
    for seed in range(6):
        a = rp.MTDraws(random.Random(seed))
        rp.ga_scalar(sp, parent, a, mutation_rate=0.2)
        order = list(a.params(len(sp)))
        assert order != list(range(len(sp))) and sorted(order) == list(range(len(sp)))
        state = a.rng.getstate()
        second = rp.ga_scalar(sp, parent, a, mutation_rate=0.2)
        b = rp.MTDraws(random.Random())
        b.rng.setstate(state)
        b._params[len(sp)] = order
        assert rp.ga_scalar(sp, parent, b, mutation_rate=0.2) == second
        c = rp.MTDraws(random.Random())
        c.rng.setstate(state)
        differs += rp.ga_scalar(sp, parent, c, mutation_rate=0.2) != second
    assert differs > 0
