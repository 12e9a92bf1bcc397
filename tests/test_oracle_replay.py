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
    for xop in (pm.X_OX1, pm.X_PMX, pm.X_CX):
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
