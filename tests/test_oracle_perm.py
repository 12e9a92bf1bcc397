"""PermutationParameter oracle (oracle/perm.py): hand-traced known answers of
the reference operators (manipulator.py:1057-1353) at chosen draws, operator
invariants, and the batched DE / PSO / GA / hash restatements on a space with
permutations.  CPU only."""
import hashlib

import numpy as np
import pytest

from oracle import de as ode
from oracle import ga as oga
from oracle import hashing as oh
from oracle import perm as pm
from oracle import pso as opso
from oracle.space import PERM, Param, columns, features, row_values, soa_from_rows


class Fixed:
    """words chosen so that randint(a, b) returns the wanted value"""

    def __init__(self, picks):
        self.w = [((off << 32) + n - 1) // n for off, n in picks]

    def __getitem__(self, k):
        return self.w[k]


def test_randint_words():
    for n in (1, 2, 3, 7, 41, 1000):
        for off in range(min(n, 50)):
            assert pm.randbelow(Fixed([(off, n)])[0], n) == off


def test_ox1_known_answer():
    p1, p2 = list(range(10)), list(range(9, -1, -1))
    # r = randint(0, 10 - 3) = 2: c1 = p1 - [7, 6, 5]; c1[:2] + [7, 6, 5] + c1[2:]
    assert pm.cross_OX1(p1, p2, 3, Fixed([(2, 8)])) == [0, 1, 7, 6, 5, 2, 3, 4, 8, 9]


def test_ox3_known_answer():
    p1, p2 = list(range(10)), list(range(9, -1, -1))
    # r1 = 1, r2 = 4: segment p2[4:7] = [5, 4, 3]
    assert pm.cross_OX3(p1, p2, 3, Fixed([(1, 8), (4, 8)])) == [0, 5, 4, 3, 1, 2, 6, 7, 8, 9]


def test_px_known_answer():
    p1, p2 = list(range(10)), list(range(9, -1, -1))
    # c1 = randint(2, 10) = 4: sorted(p1[:4], key=p2.index) + p1[4:]
    assert pm.cross_PX(p1, p2, 0, Fixed([(2, 9)])) == [3, 2, 1, 0, 4, 5, 6, 7, 8, 9]


def test_cx_known_answer():
    # s = 0: cycle 0 -> p2.index(0) = 2 -> p2.index(2) = 1 -> p2.index(1) = 0
    assert pm.cross_CX([0, 1, 2, 3, 4], [1, 2, 0, 4, 3], 0, Fixed([(0, 5)])) == [1, 2, 0, 3, 4]


def test_pmx_known_answers():
    # displaced values go to the first candidate position holding the intruder
    assert pm.cross_PMX([0, 1, 2, 3, 4, 5], [3, 4, 5, 0, 1, 2], 2, Fixed([(1, 5)])) == [0, 4, 5, 3, 1, 2]
    # the link-chasing loop (c2[0] in c1) resolves inside the crossed section
    assert pm.cross_PMX([0, 1, 2, 3, 4], [1, 2, 0, 3, 4], 3, Fixed([(0, 3)])) == [1, 2, 0, 3, 4]


def test_shuffle_is_fisher_yates():
    # random.shuffle: i = 3, 2, 1 with j = randbelow(i + 1)
    x = [0, 1, 2, 3]
    pm.shuffle(x, Fixed([(0, 4), (2, 3), (0, 2)]))
    # i=3,j=0: [3,1,2,0]; i=2,j=2: same; i=1,j=0: [1,3,2,0]
    assert x == [1, 3, 2, 0]


def test_small_random_change():
    x = [0, 1, 2, 3]
    w = [0, 2 ** 31, 0]          # swap(0,1) (u = 0 < .25), keep, swap(2,3)
    pm.small_random_change(x, w)
    assert x == [1, 0, 3, 2]


@pytest.mark.parametrize("xop", [pm.X_OX1, pm.X_OX3, pm.X_PX, pm.X_CX, pm.X_PMX])
def test_crossovers_return_permutations(xop):
    for S in (1, 2, 3, 7, 10, 23):
        for g in range(40):
            p1 = pm.randomized(pm.identity(S), pm.Words(1, g, 0, 0, 1))
            p2 = pm.randomized(pm.identity(S), pm.Words(2, g, 0, 0, 1))
            for d in (0, S // 3, pm.swarm_d(S)):
                r = pm.cross(xop, p1, p2, d, pm.Words(3, g, 7, 1, 4))
                assert sorted(r) == list(range(S))
                if xop in (pm.X_OX1, pm.X_PMX) and S > 1:
                    dd = d if d else max(1, int(round(S * 0.3)))
                    rr = pm.randint(pm.Words(3, g, 7, 1, 4)[0], 0, S - dd)
                    assert r[rr:rr + dd] == p2[rr:rr + dd]     # the crossed section is p2's


def perm_space():
    from _spaces import oracle_space
    from uptune_amd import spaces
    return oracle_space(spaces.perm_mixed())


def test_columns_and_features():
    space = perm_space()
    starts, nc = columns(space)
    assert nc == 8 - 3 + 3 + 10 + 40
    pop = ode.population_init(space, 50, seed=4)
    assert pop.shape == (nc, 50)
    for p, c in zip(space, starts):
        if p.kind == PERM:
            S = len(p.options)
            assert (np.sort(pop[c:c + S], axis=0) == np.arange(S)[:, None]).all()
    rows = [row_values(space, pop, j) for j in range(50)]
    np.testing.assert_array_equal(soa_from_rows(space, rows), pop)
    f = features(space, pop)
    sched = [i for i, p in enumerate(space) if p.name == "schedule"][0]
    k = starts[sched]
    # feature of item t = its position / 9
    col = pop[k:k + 10, 0].astype(int)
    pos = {t: q / 9 for q, t in enumerate(col)}
    feat_col = 1 + 3 + 1  # alpha, loop_order(3), unroll
    assert [f[feat_col + t, 0] for t in range(10)] == [pos[t] for t in range(10)]


def test_de_scalar_equals_vec_with_permutations():
    space = perm_space()
    pop = ode.population_init(space, 16, seed=11)
    trial = ode.propose_de_vec(space, pop, 11, 2, 0, 16, 0.5, 2)
    cfgs = [row_values(space, pop, j) for j in range(16)]
    for g in range(16):
        want = ode.propose_de_scalar(space, cfgs, 11, 2, g, 0.5, 2)
        assert row_values(space, trial, g) == want


def test_hash_of_permutation_is_repr_of_list():
    space = [Param("order", PERM, options=["a", "b", 3])]
    inner = hashlib.sha256(repr([3, "a", "b"]).encode()).hexdigest()
    want = hashlib.sha256(("order" + inner + "0|").encode()).hexdigest()
    assert oh.hash_config(space, [[3, "a", "b"]]) == want


def test_pso_and_ga_keep_permutations_valid():
    space = perm_space()
    starts, nc = columns(space)
    pop = ode.population_init(space, 30, seed=5)
    gbest = pop[:, 3].copy()
    for xop in (pm.X_OX1, pm.X_OX3, pm.X_PX, pm.X_CX, pm.X_PMX):
        x, v = opso.propose_pso_vec(space, pop, np.zeros_like(pop), pop[:, ::-1].copy(), gbest, 5, 1, 0, 30,
                                    crossover=xop)
        y, inv = oga.propose_ga_vec(space, None, None, 5, 1, 0, 30, mutation_rate=0.3, crossover_rate=0.8,
                                    crossover=xop, normal=True)
        for out in (x, y):
            for p, c in zip(space, starts):
                if p.kind == PERM:
                    S = len(p.options)
                    assert (np.sort(out[c:c + S], axis=0) == np.arange(S)[:, None]).all()
