"""Batched GA-family proposal restated from
python/uptune/opentuner/search/evolutionarytechniques.py:29-134 and
globalGA.py:28-76.

Per candidate (one `desired_configuration` call):
  parents   = [select(), select()] if random() < crossover_rate else [select()]   (:72-78)
              select() = the global best config (GreedySelectionMixin, :90-96),
              or manipulator.random() when there is none (parent1 is None)
  crossover = GGA (crossover_strength > 0): copy the first
              int(crossover_strength * P) params of a shuffle from parent 2
              (globalGA.py:68-76); GA(crossover=op) (CrossoverMixin, :123-134):
              op3_cross_<op>(new, parent1, parent2, d=size // 3) on every
              permutation of size > 6 when two parents were selected (perm draw
              site p|5<<28)
  retry <= max_retries (:45-49):
      mutation: shuffle(params); mutate the first must_mutate_count; each other
                param with probability mutation_rate (:51-61)
        uniform: op1_randomize                                    (:63-67)
        normal (NormalMutationMixin, :107-114): primitive ->
                op1_normal_mutation(sigma) (manipulator.py:505-521); Bool -> op1_flip,
                Enum -> op1_randomize, Permutation -> op1_randomize or
                op1_small_random_change (random.choice(manipulators), :1084-1085;
                the choice from the (z, w) words of draw p|r<<20|1<<28)
      accept when hash_config(cfg) is not a parent hash  == the values differ
      bitwise from every parent
  after max_retries failures the technique returns None (candidate invalid).
"The first d params of a shuffle" is a uniformly random d-subset; the batch
form draws it with Knuth's selection sampling (Algorithm S: param p joins
with probability (d - chosen) / (P - p), exactly d chosen), one uniform per
param.
Draws (op = OP_GA or OP_GGA): CAND|0 -> parents; p|2<<28 / p|3<<28 random
parent values; p|4<<28 crossover subset; p|r<<20: (x,y) must-mutate subset,
(z,w) mutation coin; p|r<<20|1<<28 randomize values; p|r<<20|2<<28 normal
draws.
"""
import numpy as np

from . import perm as pm
from . import philox as ph
from .mathx import normal_draw
from .space import BOOL, ENUM, PERM, columns, get_unit_value_vec, randomize, set_unit_value_vec, to_f64, width


def _rand_col(prm, seed, g, stream, round_, op):
    x, y, z, w = ph.draw(seed, g, stream, round_, op)
    return np.array([to_f64(prm, randomize(prm, int(a), int(b), int(c), int(d))) for a, b, c, d in zip(x, y, z, w)])


def select_subset(u, d):
    """Algorithm S over params in order: u [P][m] uniforms -> bool [P][m] with
    exactly d True per column"""
    P, m = u.shape
    chosen = np.zeros(m, dtype=np.float64)
    out = np.zeros((P, m), dtype=bool)
    for p in range(P):
        take = (float(P - p) * u[p]) < (float(d) - chosen)
        out[p] = take
        chosen = chosen + take
    return out


def _uniforms(seed, g, P, stream_of, round_, op, hi=False):
    rows = []
    for p in range(P):
        x, y, z, w = ph.draw(seed, g, stream_of(p), round_, op)
        rows.append(ph.u01(z, w) if hi else ph.u01(x, y))
    return np.stack(rows)


def _perm_rand(S, seed, g, stream, round_, op):
    return pm.randomized(pm.identity(S), pm.Words(seed, g, stream, round_, op))


def propose_ga_vec(space, parent1, parent2, seed, round_, cand_base, m, mutation_rate=0.1, must_mutate_count=1,
                   normal=False, sigma=0.1, crossover_rate=0.0, crossover_strength=0.0, max_retries=10,
                   op=ph.OP_GA, crossover=pm.X_NONE, g=None):
    """g: explicit global candidate indices (then cand_base / m are ignored)"""
    P = len(space)
    starts, nc = columns(space)
    g = np.arange(cand_base, cand_base + m, dtype=np.uint64) if g is None else np.asarray(g, dtype=np.uint64)
    m = g.size
    x, y, _, _ = ph.draw(seed, g, ph.STREAM_CAND | 0, round_, op)
    two = ph.u01(x, y) < crossover_rate
    P1 = np.empty((nc, m))
    P2 = np.empty((nc, m))
    for p, prm in enumerate(space):
        c0 = starts[p]
        if prm.kind == PERM:
            S = width(prm)
            for j in range(m):
                a = parent1[c0:c0 + S] if parent1 is not None else \
                    _perm_rand(S, seed, g[j], p | (2 << 28), round_, op)
                if parent2 is not None:
                    b = parent2[c0:c0 + S]
                elif parent1 is not None:
                    b = parent1[c0:c0 + S]
                else:
                    b = _perm_rand(S, seed, g[j], p | (3 << 28), round_, op)
                P1[c0:c0 + S, j] = a
                P2[c0:c0 + S, j] = b
            continue
        P1[c0] = parent1[c0] if parent1 is not None else _rand_col(prm, seed, g, p | (2 << 28), round_, op)
        if parent2 is not None:
            P2[c0] = parent2[c0]
        elif parent1 is not None:
            P2[c0] = parent1[c0]
        else:
            P2[c0] = _rand_col(prm, seed, g, p | (3 << 28), round_, op)
    cfg = P1.copy()
    sel = np.zeros((P, m), dtype=bool)
    if crossover_strength > 0:
        d = int(crossover_strength * P)
        sel = select_subset(_uniforms(seed, g, P, lambda p: p | (4 << 28), round_, op), d) & two[None, :]
    for p, prm in enumerate(space):
        c0, w = starts[p], width(prm)
        cfg[c0:c0 + w] = np.where(sel[p][None, :], P2[c0:c0 + w], cfg[c0:c0 + w])
        # CrossoverMixin.crossover: permutation params of size > 6, d = size // 3
        if prm.kind == PERM and crossover != pm.X_NONE and w > 6:
            for j in range(m):
                if two[j] and not sel[p, j]:
                    W = pm.Words(seed, g[j], p | (5 << 28), round_, op)
                    cfg[c0:c0 + w, j] = pm.cross(crossover, [int(a) for a in P1[c0:c0 + w, j]],
                                                 [int(a) for a in P2[c0:c0 + w, j]], w // 3, W)
    accepted = np.zeros(m, dtype=bool)
    for r in range(max_retries):
        active = ~accepted
        forced = select_subset(_uniforms(seed, g, P, lambda p: p | (r << 20), round_, op), must_mutate_count)
        for p, prm in enumerate(space):
            c0 = starts[p]
            _, _, zz, ww = ph.draw(seed, g, p | (r << 20), round_, op)
            mut = active & (forced[p] | (ph.u01(zz, ww) < mutation_rate))
            if not mut.any():
                continue
            if prm.kind == PERM:
                S = width(prm)
                sp = p | (r << 20) | (1 << 28)
                _, _, qz, qw = ph.draw(seed, g, sp, round_, op)
                for j in np.nonzero(mut)[0]:
                    cur = [int(a) for a in cfg[c0:c0 + S, j]]
                    W = pm.Words(seed, g[j], sp, round_, op)
                    # uniform: op1_randomize; normal: random.choice(manipulators)
                    if normal and int(ph.below64(ph.u64(qz[j], qw[j]), 2)) == 1:
                        pm.small_random_change(cur, W)
                    else:
                        pm.shuffle(cur, W)
                    cfg[c0:c0 + S, j] = cur
                continue
            gi = g[mut]
            cur = cfg[c0, mut]
            if normal and prm.is_primitive():
                v = get_unit_value_vec(prm, cur)
                z = normal_draw(seed, gi, p | (r << 20) | (2 << 28), round_, op)
                v = v + (0.0 + z * sigma)
                v = np.where(v < 0.0, v * -1.0, v)
                v = np.where(v > 1.0, 1.0 - np.fmod(v, 1.0), v)
                new = set_unit_value_vec(prm, v, cur)
            elif normal and prm.kind == BOOL:
                new = 1.0 - cur
            else:
                new = _rand_col(prm, seed, gi, p | (r << 20) | (1 << 28), round_, op)
            cfg[c0, mut] = new
        b = cfg.view(np.uint64)
        diff1 = np.any(b != P1.view(np.uint64), axis=0)
        diff2 = np.any(b != P2.view(np.uint64), axis=0)
        accepted |= active & diff1 & (~two | diff2)
    return cfg, ~accepted
