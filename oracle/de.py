"""Batched DE/rand/1/bin restated from
python/uptune/opentuner/search/differentialevolution.py:105-129.

Batch semantics (the build's): candidate g (global index)
targets population member g % npop and produces one trial.  The reference's
random draws are replaced by Philox draws keyed by (seed, g, stream, round):

  donors  x1,x2,x3 : the first 3 of shuffle(list(set(pop) - {target})
                     + [best] * information_sharing)     (:109-118)
                     = 3 distinct positions of that pool; a position past the
                     npop - 1 other members is a copy of the best config
  use_f   = random()/2.0 + 0.5                          (:120)
  forced  = first n_cross names of a shuffled name list (:122-125)
            == a uniform n_cross-subset, drawn by skip-rank (forced_mask)
  cross   = forced or random() < cr                     (:125; cr_tests:
            32-bit uniforms, four params per Philox block)
  primitive: op4_set_linear(x1, x2, x3, 1.0, F, -F)     (manipulator.py:523-542)
  complex:   copy x1; randomize iff x2 != x3            (manipulator.py:866-914)
             (PERM: randomize = shuffle of the x1 copy, oracle/perm.py)
  otherwise the target's value is kept (cfg = copy(parent))  (:106)
"""
import numpy as np

from . import perm as pm
from . import philox as ph
from .space import (PERM, columns, get_unit_value_vec, op4_set_linear_primitive, randomize, set_unit_value_vec,
                    width)


def donors(g, npop, seed, round_, share=0):
    """(t, d1, d2, d3) for t = g % npop (vectorised).  The donor pool is the
    npop - 1 members other than t followed by `share` copies of the best
    config (differentialevolution.py:110-116); three distinct positions a, b, c
    of it are drawn (shuffle()[0:3]); a member position q maps to member
    q + (q >= t), a best-copy position to -1."""
    g = np.asarray(g, dtype=np.uint64)
    t = (g % np.uint64(npop)).astype(np.int64)
    Q = npop - 1 + share
    x, y, z, _ = ph.draw(seed, g, ph.STREAM_CAND | 0, round_, ph.OP_DE)
    a = ph.umulhi32(x, Q).astype(np.int64)
    b = ph.umulhi32(y, Q - 1).astype(np.int64)
    b = b + (b >= a)
    s0, s1 = np.minimum(a, b), np.maximum(a, b)
    c = ph.umulhi32(z, Q - 2).astype(np.int64)
    c = c + (c >= s0)
    c = c + (c >= s1)

    def member(q):
        return np.where(q < npop - 1, q + (q >= t), -1)
    return t, member(a), member(b), member(c)


def use_f(g, seed, round_):
    x, y, _, _ = ph.draw(seed, g, ph.STREAM_CAND | 1, round_, ph.OP_DE)
    return ph.u01(x, y) / 2.0 + 0.5


DE_CR_STREAM = 0x100


def forced_mask(g, P, n_cross, seed, round_):
    """bool [P][m]: the forced set, a uniform n_cross-subset of the params
    (the first n_cross names of the shuffled list, :122-125; n_cross <= 4),
    drawn by skip-rank from the words of block (STREAM_CAND | 2): element k is
    the (umulhi32(word_k, P - k))-th param not yet chosen (ut_core.h de_forced_set)"""
    g = np.asarray(g, dtype=np.uint64)
    out = np.zeros((P, g.size), dtype=bool)
    nc = min(n_cross, P)
    if nc <= 0:
        return out
    assert nc <= 4, "n_cross <= 4"
    words = ph.draw(seed, g, ph.STREAM_CAND | 2, round_, ph.OP_DE)
    chosen = []
    cols = np.arange(g.size)
    for k in range(nc):
        v = ph.umulhi32(words[k], P - k).astype(np.int64)
        if chosen:
            for c in np.sort(np.stack(chosen), axis=0):   # skip the chosen ones, ascending
                v = v + (v >= c)
        chosen.append(v)
        out[v, cols] = True
    return out


def cr_tests(g, P, cr, seed, round_):
    """bool [P][m]: `random() < cr` (:125) of param p = word p % 4 of block
    (STREAM_CAND | (DE_CR_STREAM + p // 4)), a 32-bit uniform"""
    g = np.asarray(g, dtype=np.uint64)
    out = np.empty((P, g.size), dtype=bool)
    for b in range((P + 3) // 4):
        ws = ph.draw(seed, g, ph.STREAM_CAND | (DE_CR_STREAM + b), round_, ph.OP_DE)
        for q in range(4):
            p = 4 * b + q
            if p < P:
                out[p] = ws[q].astype(np.float64) * 2.0 ** -32 < cr
    return out


def propose_de_vec(space, pop, seed, round_, cand_base, m, cr, n_cross=1, best=None, information_sharing=1):
    """pop: SoA [ncols][npop] float64 -> trial SoA [ncols][m].  best: the
    driver's best config as a value row [ncols] (None: no result yet, the pool
    is the population only)."""
    ncols, npop = pop.shape
    g = np.arange(cand_base, cand_base + m, dtype=np.uint64)
    share = information_sharing if best is not None else 0
    t, d1, d2, d3 = donors(g, npop, seed, round_, share)
    if share:   # the best config as an extra population column npop
        pop = np.concatenate([pop, np.asarray(best, dtype=np.float64).reshape(ncols, 1)], axis=1)
        d1, d2, d3 = (np.where(d < 0, npop, d) for d in (d1, d2, d3))
    return _trials(space, pop, g, t, d1, d2, d3, seed, round_, cr, n_cross)


def propose_de_at(space, g, npop, seed, round_, cr, n_cross=1):
    """The trials of explicit global candidate indices g of a round over the
    op1_randomize population of npop members (no best config yet), computing
    only the members those trials read (target + 3 donors): the bench's parity
    check of a full-size round's selections.  = propose_de_vec(...)[:, g]."""
    g = np.asarray(g, dtype=np.uint64)
    t, d1, d2, d3 = donors(g, npop, seed, round_, 0)
    members = np.unique(np.concatenate([t, d1, d2, d3]))
    pop = population_init(space, npop, seed, members=members)
    t, d1, d2, d3 = (np.searchsorted(members, d) for d in (t, d1, d2, d3))
    return _trials(space, pop, g, t, d1, d2, d3, seed, round_, cr, n_cross)


def _trials(space, pop, g, t, d1, d2, d3, seed, round_, cr, n_cross):
    """the DE trial of every candidate g: target column t, donor columns d1-d3 of pop"""
    ncols = pop.shape[0]
    m = g.size
    P = len(space)
    starts, _ = columns(space)
    F = use_f(g, seed, round_)
    forced = forced_mask(g, P, n_cross, seed, round_)
    crt = cr_tests(g, P, cr, seed, round_)
    out = np.empty((ncols, m), dtype=np.float64)
    for p, prm in enumerate(space):
        cross = forced[p] | crt[p]
        c0 = starts[p]
        if prm.kind == PERM:
            S = width(prm)
            blk = pop[c0:c0 + S]
            for j in range(m):
                if cross[j]:
                    v = [int(a) for a in blk[:, d1[j]]]                 # copy_value(x1)
                    if list(blk[:, d2[j]]) != list(blk[:, d3[j]]):     # add_difference -> op1_randomize
                        pm.shuffle(v, pm.Words(seed, g[j], p | (1 << ph.STREAM_SUB_SHIFT), round_, ph.OP_DE))
                    out[c0:c0 + S, j] = v
                else:
                    out[c0:c0 + S, j] = blk[:, t[j]]
            continue
        col = pop[c0]
        vt = col[t]
        x1, x2, x3 = col[d1], col[d2], col[d3]
        if prm.is_primitive():
            va, vb, vc = get_unit_value_vec(prm, x1), get_unit_value_vec(prm, x2), get_unit_value_vec(prm, x3)
            u = (1.0 * va + F * vb) + (-F) * vc
            u = np.where(1.0 < u, 1.0, u)
            u = np.where(u > 0.0, u, 0.0)
            nv = set_unit_value_vec(prm, u, vt)
        else:
            nv = x1.copy()
            diff = x2 != x3
            if diff.any():
                gi = g[diff]
                rx, ry, rz, rw = ph.draw(seed, gi, p | (1 << ph.STREAM_SUB_SHIFT), round_, ph.OP_DE)
                from .space import to_f64
                nv[diff] = [to_f64(prm, randomize(prm, int(a), int(b), int(c), int(d)))
                            for a, b, c, d in zip(rx, ry, rz, rw)]
        out[c0] = np.where(cross, nv, vt)
    return out


def propose_de_scalar(space, pop_cfgs, seed, round_, g, cr, n_cross=1, best_cfg=None, information_sharing=1):
    """One trial, written like create_new_configuration (:105-129) over
    Python values.  pop_cfgs: list of configs (lists of stored values)."""
    npop = len(pop_cfgs)
    share = information_sharing if best_cfg is not None else 0
    t, d1, d2, d3 = (int(v[0]) for v in donors(np.array([g]), npop, seed, round_, share))
    cfg = list(pop_cfgs[t])                         # manipulator.copy(parent.config.data)
    # shuffled_pop += [PopulationMember(best)] * information_sharing (:113-116)
    x1, x2, x3 = (best_cfg if d < 0 else pop_cfgs[d] for d in (d1, d2, d3))
    F = float(use_f(np.array([g]), seed, round_)[0])
    forced = forced_mask(np.array([g]), len(space), n_cross, seed, round_)[:, 0]
    crt = cr_tests(np.array([g]), len(space), cr, seed, round_)[:, 0]
    for p, prm in enumerate(space):
        if forced[p] or crt[p]:
            if prm.is_primitive():
                cfg[p] = op4_set_linear_primitive(prm, x1[p], x2[p], x3[p], 1.0, F, -F, cfg[p])
            elif prm.kind == PERM:
                cfg[p] = list(x1[p])                # copy_value: deepcopy of the list
                if x2[p] != x3[p]:                  # add_difference -> op1_randomize = shuffle
                    pm.shuffle(cfg[p], pm.Words(seed, g, p | (1 << ph.STREAM_SUB_SHIFT), round_, ph.OP_DE))
            else:
                cfg[p] = x1[p]                      # copy_value(cfg_a, cfg)
                if x2[p] != x3[p]:                  # add_difference: not same_value -> randomize
                    rx, ry, rz, rw = ph.draw(seed, np.array([g]), p | (1 << ph.STREAM_SUB_SHIFT), round_, ph.OP_DE)
                    cfg[p] = randomize(prm, int(rx[0]), int(ry[0]), int(rz[0]), int(rw[0]))
    return cfg


def population_init(space, npop, seed, round_=0, members=None):
    """op1_randomize every member (manipulator.py:171-176) -> SoA [ncols][npop]
    (members: only those member indices, in that order -> [ncols][len(members)])"""
    from .space import to_f64
    g = np.arange(npop, dtype=np.uint64) if members is None else np.asarray(members, dtype=np.uint64)
    npop = g.size
    starts, nc = columns(space)
    out = np.empty((nc, npop), dtype=np.float64)
    for p, prm in enumerate(space):
        c0 = starts[p]
        if prm.kind == PERM:   # seed_value() = list(items), then shuffle
            S = width(prm)
            for j in range(npop):
                out[c0:c0 + S, j] = pm.randomized(pm.identity(S), pm.Words(seed, int(g[j]), p, round_, ph.OP_INIT))
            continue
        x, y, z, w = ph.draw(seed, g, p, round_, ph.OP_INIT)
        if prm.kind == 0:  # FLOAT, vectorised: lo + (hi - lo) * u
            out[c0] = prm.lo + (prm.hi - prm.lo) * ph.u01(x, y)
        else:
            out[c0] = [to_f64(prm, randomize(prm, int(a), int(b), int(c), int(d))) for a, b, c, d in zip(x, y, z, w)]
    return out
