"""Reference-ordered restatements of PSO's particle move and the GA / GGA
proposal loop (TEST INFRASTRUCTURE: imported only by tests/).

Written like the reference, one configuration at a time, calling a draw
source exactly where the reference calls `random`:

  HybridParticle.move -> op3_swarm per kind     opentuner/search/pso.py:70-77;
      Float / LogInteger manipulator.py:709-744, Integer / PowerOfTwo :660-700,
      Boolean :962-996, Enum (opn_stochastic_mix) :409-443, Permutation :1115-1140
  EvolutionaryTechnique.desired_configuration   evolutionarytechniques.py:29-49
      selection :72-78, GreedySelectionMixin.select :85-96 (manipulator.random,
      manipulator.py:171-176), mutation :51-61, mutate_param :63-67,
      NormalMutationMixin :98-114 (op1_normal_mutation manipulator.py:505-521),
      CrossoverMixin :117-134
  GlobalEvolutionaryTechnique (GGA)              globalGA.py:28-85

Two draw sources feed the same code:

  MTDraws(random.Random(s))  the reference's own MT19937 stream, consumed call
                             for call in the reference's order (replay mode);
  CounterDraws(seed, g, round_, op)
                             the build's counter RNG: every call is answered
                             from the Philox site the batch form assigns to
                             it (oracle/pso.py, oracle/ga.py docstrings).

tests/test_oracle_replay.py shows that this scalar code fed CounterDraws
reproduces the batch oracle (oracle/pso.py, oracle/ga.py) exactly, candidate
for candidate: the batch form follows the reference's control flow (which
draw decides what, retry and acceptance order, compounding mutations across
retries), and differs only in where its random numbers come from.  (DE has
the same pair: oracle/de.py propose_de_scalar.)  The reference itself cannot
be imported here; MT replay runs this restatement on the
reference's RNG, it is not compared with the reference's own output.

The PSO sigmoid's numpy.exp is part of the draw source: MTDraws uses
numpy.exp (the reference), CounterDraws the build's ut_exp (oracle/mathx.py,
= the device's), the one non-random substitution.

MT mode covers every random call of the path: the permutation crossovers
op3_cross_{OX1,OX3,PX,CX,PMX} (manipulator.py:1179-1353; PSO's permutation
op3_swarm :1115-1140 and CrossoverMixin :123-134) draw their random.randint
calls from the stream in the reference's order (oracle/perm.py `ints`), and
MTDraws.params keeps the manipulator's ONE shared params list that GA / GGA
shuffle in place: seed_config, random(), the next mutation,
CrossoverMixin and HybridParticle.move iterate the order the last shuffle
left, across calls.  (The counter form keys each draw by param index, so the
order does not change its output.)
"""
import random

import numpy as np

from . import hashing as oh
from . import perm as pm
from . import philox as ph
from .mathx import normal_draw, ut_exp
from .space import (BOOL, ENUM, FLOAT, INT, LOGINT, PERM, POW2, get_unit_value, randomize, scale, set_unit_value,
                    unscale)


# ---------------------------------------------------------------------------
# draw sources
# ---------------------------------------------------------------------------
class MTDraws:
    """CPython's random.Random, one stream for every site (the reference's)."""

    def __init__(self, rng: random.Random):
        self.rng = rng
        self._params = {}

    exp = staticmethod(np.exp)

    def site(self, *key):
        return self

    def params(self, P):
        """manipulator.parameters(cfg) / manipulator.params: ONE shared list
        (manipulator.py:178-185) that GA / GGA shuffle in place
        (evolutionarytechniques.py:55-56, globalGA.py:54-56,71-72):
        every later iteration -- seed_config, random(), the next mutation's
        shuffle, CrossoverMixin, HybridParticle.move -- sees the order the last
        shuffle left.  Persistent across calls on this draw source."""
        if P not in self._params:
            self._params[P] = list(range(P))
        return self._params[P]

    def random(self):
        return self.rng.random()

    def uniform(self, a, b):
        return self.rng.uniform(a, b)

    def gauss(self, mu, sigma):
        return self.rng.gauss(mu, sigma)

    def normalvariate(self, mu, sigma):
        return self.rng.normalvariate(mu, sigma)

    def shuffle(self, x):
        self.rng.shuffle(x)

    def choice(self, seq):
        return self.rng.choice(seq)

    def seed_value(self, prm):
        """Parameter.seed_value (manipulator.py:581-583, 948-949, 1041-1042, 1081-1082)"""
        if prm.kind == BOOL:
            return self.rng.choice((True, False))
        if prm.kind == ENUM:
            return self.rng.choice(prm.options)
        if prm.kind == PERM:
            return list(range(len(prm.options)))
        return prm.lo

    def op1_randomize(self, prm, cur):
        """op1_randomize (manipulator.py:596-606, 940-949, 1033-1039, 1057-1064)"""
        if prm.kind == PERM:
            v = list(cur)
            self.rng.shuffle(v)
            return v
        if prm.kind == BOOL:
            return self.rng.choice((True, False))
        if prm.kind == ENUM:
            return self.rng.choice(prm.options)
        lo, hi = prm.legal_range()
        if prm.is_integer_type():
            return unscale(prm, self.rng.randint(lo, hi))
        return unscale(prm, self.rng.uniform(lo, hi))

    def small_random_change(self, cur, p=0.25):
        """op1_small_random_change (manipulator.py:1066-1079)"""
        v = list(cur)
        for i in range(1, len(v)):
            if self.rng.random() < p:
                v[i - 1], v[i] = v[i], v[i - 1]
        return v

    def cross(self, xop, p1, p2, d):
        """op3_cross_<xop> (manipulator.py:1179-1353) on the MT stream: each
        operator's random.randint calls, in the reference's order (PX: the cut
        point; PMX, OX1: the section start; CX: the start index; OX3: r1 then
        r2), through the same list code as the counter form (oracle/perm.py)"""
        return pm.cross(xop, list(p1), list(p2), d, self.rng)


class _Queue:
    """answers random() / uniform(0, 1) / gauss calls from a fixed list of
    counter draws, in call order"""

    def __init__(self, uniforms=(), normals=(), words=None, exp=ut_exp):
        self.u, self.z, self.words = list(uniforms), list(normals), words
        self.exp = exp

    def random(self):
        return float(self.u.pop(0))

    def uniform(self, a, b):
        u = self.random()
        return a + (b - a) * u

    def gauss(self, mu, sigma):
        return mu + float(self.z.pop(0)) * sigma

    normalvariate = gauss


class CounterDraws:
    """The build's counter RNG for candidate g of a round: each reference call
    site is answered from its Philox site (the batch oracles' site map)."""

    def __init__(self, seed, g, round_, op):
        self.seed, self.g, self.round_, self.op = int(seed), int(g), int(round_), int(op)
        self.ga = np.array([self.g], dtype=np.uint64)

    exp = staticmethod(ut_exp)

    @staticmethod
    def params(P):
        """the batch form keys every draw by parameter index, so the order of
        the manipulator's shared list does not matter: a fresh list"""
        return list(range(P))

    def _blk(self, stream):
        return [int(v[0]) for v in ph.draw(self.seed, self.ga, stream & 0xFFFFFFFF, self.round_, self.op)]

    def _u(self, stream, hi=False):
        x, y, z, w = self._blk(stream)
        return float(ph.u01(np.uint32(z), np.uint32(w))) if hi else float(ph.u01(np.uint32(x), np.uint32(y)))

    def _words(self, stream):
        return pm.Words(self.seed, self.g, stream, self.round_, self.op)

    def site(self, kind, *key):
        S = ph.STREAM_SUB_SHIFT
        if kind == "pso":      # (p, param kind): op3_swarm's random() / uniform / gauss calls
            p, pk = key
            x, y, z, w = self._blk(p)
            r1, r2 = float(ph.u01(np.uint32(x), np.uint32(y))), float(ph.u01(np.uint32(z), np.uint32(w)))
            if pk == ENUM:     # opn_stochastic_mix's r
                return _Queue([self._u(p | (1 << S))])
            if pk == BOOL:     # r1, r2, then the position coin
                return _Queue([r1, r2, self._u(p | (1 << S))])
            if pk == PERM:     # the two uniform(0, 1), then the crossover's words
                return _CounterSite(self, _Queue([r1, r2]), cross_stream=p | (1 << S))
            normals = [float(normal_draw(self.seed, self.ga, p | (2 << S), self.round_, self.op)[0])] \
                if pk in (INT, POW2) else []
            return _Queue([r1, r2], normals)
        if kind == "select":   # selection's random() < crossover_rate
            return _Queue([self._u(ph.STREAM_CAND | 0)])
        if kind == "parent":   # manipulator.random() of parent `which` (2 or 3), param p
            which, p = key
            return _CounterSite(self, _Queue(), rand_stream=p | (which << 28))
        if kind == "gga":      # GGA crossover: shuffle(params), first d taken
            d, P = key
            u = np.array([[self._u(p | (4 << 28))] for p in range(P)])
            return _SubsetShuffle(_subset(u, d))
        if kind == "xmix":     # CrossoverMixin's op3_cross_<op> on param p
            p, = key
            return _CounterSite(self, _Queue(), cross_stream=p | (5 << 28))
        if kind == "mutation":  # retry r: shuffle(params), must-mutate first, coins for the rest
            r, mmc, P = key
            blks = [self._blk(p | (r << 20)) for p in range(P)]
            u = np.array([[float(ph.u01(np.uint32(b[0]), np.uint32(b[1])))] for b in blks])
            coins = {p: float(ph.u01(np.uint32(b[2]), np.uint32(b[3]))) for p, b in enumerate(blks)}
            return _SubsetShuffle(_subset(u, mmc), coins)
        if kind == "mutate":   # mutate_param of param p in retry r
            r, p = key
            sp = p | (r << 20) | (1 << 28)
            normals = [float(normal_draw(self.seed, self.ga, p | (r << 20) | (2 << 28), self.round_, self.op)[0])]
            _, _, qz, qw = self._blk(sp)
            return _CounterSite(self, _Queue([], normals), rand_stream=sp,
                                choice2=int(ph.below64(ph.u64(np.uint32(qz), np.uint32(qw)), 2)))
        raise KeyError(kind)


def _subset(u, d):
    """Algorithm S over params in order (oracle/ga.py select_subset), one candidate"""
    P = u.shape[0]
    chosen, out = 0.0, []
    for p in range(P):
        if float(P - p) * float(u[p, 0]) < float(d) - chosen:
            out.append(p)
            chosen += 1.0
    return out


class _SubsetShuffle:
    """random.shuffle(params) whose first d entries are the Algorithm S subset
    (a uniformly random d-subset, as the first d of a uniform shuffle are);
    random() then answers the coin of the next param in the shuffled order"""

    def __init__(self, chosen, coins=None):
        self.chosen, self.coins, self.order = chosen, coins or {}, []

    def shuffle(self, params):
        head = [p for p in params if p in self.chosen]
        params[:] = head + [p for p in params if p not in self.chosen]
        self.order = params[len(head):]

    def random(self):
        return self.coins[self.order.pop(0)]


class _CounterSite:
    def __init__(self, d, queue, rand_stream=None, cross_stream=None, choice2=0):
        self.d, self.q, self.rand_stream, self.cross_stream, self.choice2 = d, queue, rand_stream, cross_stream, choice2

    def random(self):
        return self.q.random()

    def uniform(self, a, b):
        return self.q.uniform(a, b)

    def normalvariate(self, mu, sigma):
        return self.q.normalvariate(mu, sigma)

    def seed_value(self, prm):
        return list(range(len(prm.options))) if prm.kind == PERM else None

    def op1_randomize(self, prm, cur):
        if prm.kind == PERM:
            v = list(cur)
            pm.shuffle(v, self.d._words(self.rand_stream))
            return v
        x, y, z, w = self.d._blk(self.rand_stream)
        return randomize(prm, x, y, z, w)

    def small_random_change(self, cur, p=0.25):
        v = list(cur)
        pm.small_random_change(v, self.d._words(self.rand_stream), p)
        return v

    def choice(self, seq):
        return seq[self.choice2 if len(seq) == 2 else 0]

    def cross(self, xop, p1, p2, d):
        return pm.cross(xop, p1, p2, d, self.d._words(self.cross_stream))


# ---------------------------------------------------------------------------
# PSO: HybridParticle.move
# ---------------------------------------------------------------------------
def op3_swarm(prm, draws, x, gb, lb, c, c1, c2, velocity, sigma=0.2, xchoice=pm.X_OX1):
    """one param's op3_swarm (cfg = x, cfg1 = global best, cfg2 = particle best,
    stored values); -> (new stored value, returned velocity)"""
    if prm.kind in (FLOAT, LOGINT):           # FloatParameter.op3_swarm :709-744 (LogInteger inherits)
        vmin, vmax = prm.legal_range()
        v = velocity * c + (scale(prm, gb) - scale(prm, x)) * c1 * draws.random() + \
            (scale(prm, lb) - scale(prm, x)) * c2 * draws.random()
        p = scale(prm, x) + v
        p = min(vmax, max(p, vmin))
        return unscale(prm, p), v
    if prm.kind in (INT, POW2):               # IntegerParameter.op3_swarm :660-700 (PowerOfTwo inherits)
        vmin, vmax = prm.legal_range()
        k = vmax - vmin
        v = velocity * c + (scale(prm, gb) - scale(prm, x)) * c1 * draws.random() + \
            (scale(prm, lb) - scale(prm, x)) * c2 * draws.random()
        s = k / (1 + float(draws.exp(-v))) + vmin
        p = draws.gauss(s, sigma * k)
        p = int(min(vmax, max(round(p), vmin)))
        return unscale(prm, p), v
    if prm.kind == BOOL:                      # BooleanParameter.op3_swarm :962-996
        v = velocity * c + (int(gb) - int(x)) * c1 * draws.random() + (int(lb) - int(x)) * c2 * draws.random()
        s = 1 / (1 + float(draws.exp(-v)))
        p = (s - draws.random()) > 0
        return bool(p), v
    if prm.kind == ENUM:                      # opn_stochastic_mix :424-443: copy_value(cfg, cfgs[i])
        r = draws.random()                    # copies FROM the particle: x is kept
        del r
        return x, None
    if prm.kind == PERM:                      # PermutationParameter.op3_swarm :1115-1140
        if draws.uniform(0, 1) > c:
            other = gb if draws.uniform(0, 1) < c1 else lb
            x = draws.cross(xchoice, list(x), list(other), pm.swarm_d(len(x)))
        return list(x), None
    raise NotImplementedError(prm.kind)


def pso_move_scalar(space, position, velocity, best, global_best, draws, omega=0.5, phi_l=0.5, phi_g=0.5,
                    sigma=0.2, xchoice=pm.X_OX1):
    """HybridParticle.move(global_best) (pso.py:70-77): for p in params,
    velocity[p] = p.op3_swarm(position, global_best, self.best, c=omega,
    c1=phi_g, c2=phi_l, xchoice, velocity=velocity[p]).  Stored-value rows
    (PERM: item-index lists).  -> (new position, new velocity)"""
    pos, vel = list(position), list(velocity)
    for i in draws.params(len(space)):                  # for p in m.params (the shared list's order)
        prm = space[i]
        d = draws.site("pso", i, prm.kind)
        pos[i], nv = op3_swarm(prm, d, pos[i], global_best[i], best[i], omega, phi_g, phi_l, vel[i], sigma,
                               xchoice)
        vel[i] = vel[i] if nv is None else nv   # Enum / Permutation return no velocity
    return pos, vel


# ---------------------------------------------------------------------------
# GA / GGA: desired_configuration
# ---------------------------------------------------------------------------
def _manip_random(space, draws, which):
    """manipulator.random() (manipulator.py:171-176): seed_config, then
    op1_randomize of every param"""
    order = list(draws.params(len(space)))              # seed_config / random() iterate self.params
    cfg = [None] * len(space)
    for i in order:
        cfg[i] = draws.site("parent", which, i).seed_value(space[i])
    for i in order:
        cfg[i] = draws.site("parent", which, i).op1_randomize(space[i], cfg[i])
    return cfg


def _key(space, cfg):
    return oh.hash_config(space, [list(v) if p.kind == PERM else v for p, v in zip(space, cfg)])


def ga_scalar(space, best, draws, mutation_rate=0.1, must_mutate_count=1, normal=False, sigma=0.1,
              crossover_rate=0.0, crossover_strength=0.0, max_retries=10, crossover=pm.X_NONE, best2=None):
    """EvolutionaryTechnique.desired_configuration (evolutionarytechniques.py:29-49)
    with GreedySelectionMixin.select (best is the driver's best config, None
    before any result -> manipulator.random()); crossover_strength > 0 is the
    GGA crossover (globalGA.py:68-76), crossover != X_NONE CrossoverMixin's
    (:117-134).  best2: the second select()'s config (the batch form's
    parent2; the greedy mixin returns `best` again).
    -> (cfg, invalid): invalid = every retry reproduced a parent (returns None)"""
    P = len(space)
    # selection (:72-78)
    if draws.site("select").random() < crossover_rate:
        parents = [_select(space, draws, best, 2), _select(space, draws, best2 if best2 is not None else best, 3)]
    else:
        parents = [_select(space, draws, best, 2)]
    parents = [list(c) for c in parents]                       # map(copy.deepcopy, parents)
    parent_hashes = [_key(space, c) for c in parents]
    if len(parents) > 1:
        cfg = _crossover(space, draws, parents, crossover_strength, crossover)
    else:
        cfg = parents[0]
    for z in range(max_retries):                                  # retries (:45-49)
        _mutation(space, draws, cfg, z, mutation_rate, must_mutate_count, normal, sigma, P)
        if _key(space, cfg) in parent_hashes:
            continue
        return cfg, False
    return cfg, True


def _select(space, draws, cfg, which):
    return list(cfg) if cfg is not None else _manip_random(space, draws, which)


def _crossover(space, draws, parents, crossover_strength, crossover):
    cfg1, cfg2 = parents
    new = list(cfg1)                                              # manipulator.copy(cfg1)
    if crossover_strength > 0:                                    # GlobalEvolutionaryTechnique.crossover
        params = draws.params(len(space))                         # the shared list, shuffled in place
        d = int(crossover_strength * len(params))
        draws.site("gga", d, len(space)).shuffle(params)
        for i in params[:d]:
            new[i] = cfg2[i]                                      # set_value(new, get_value(cfg2))
        return new
    for i in list(draws.params(len(space))):                      # CrossoverMixin.crossover
        prm = space[i]
        if crossover != pm.X_NONE and prm.kind == PERM and len(prm.options) > 6:
            new[i] = draws.site("xmix", i).cross(crossover, list(cfg1[i]), list(cfg2[i]), len(prm.options) // 3)
    return new


def _mutation(space, draws, cfg, z, mutation_rate, must_mutate_count, normal, sigma, P):
    """EvolutionaryTechnique.mutation (:51-61), in place"""
    params = draws.params(P)                                      # the shared list, shuffled in place
    site = draws.site("mutation", z, must_mutate_count, P)
    site.shuffle(params)
    for i in list(params[:must_mutate_count]):
        _mutate_param(space[i], draws.site("mutate", z, i), cfg, i, normal, sigma)
    for i in list(params[must_mutate_count:]):
        if site.random() < mutation_rate:
            _mutate_param(space[i], draws.site("mutate", z, i), cfg, i, normal, sigma)


def _mutate_param(prm, d, cfg, i, normal, sigma):
    if not normal:                                                # mutate_param: op1_randomize (:63-67)
        cfg[i] = d.op1_randomize(prm, cfg[i])
        return
    if prm.is_primitive():                                        # op1_normal_mutation (manipulator.py:505-521)
        v = get_unit_value(prm, cfg[i])
        v += d.normalvariate(0.0, sigma)
        if v < 0.0:
            v *= -1.0
        if v > 1.0:
            v = 1.0 - (v % 1)
        cfg[i] = set_unit_value(prm, v, cfg[i])
        return
    # random.choice(param.manipulators(cfg))(cfg)   (NormalMutationMixin :113-120)
    if prm.kind == BOOL:                                          # [op1_flip]
        d.choice([None])
        cfg[i] = not cfg[i]
    elif prm.kind == PERM:                                        # [op1_randomize, op1_small_random_change]
        op = d.choice(["randomize", "small"])
        cfg[i] = d.op1_randomize(prm, cfg[i]) if op == "randomize" else d.small_random_change(cfg[i])
    else:                                                         # [op1_randomize]
        d.choice([None])
        cfg[i] = d.op1_randomize(prm, cfg[i])
