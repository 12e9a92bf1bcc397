"""Batched PSO move restated from python/uptune/opentuner/search/pso.py:23-77
and the per-kind op3_swarm (manipulator.py:660-700 Int, :709-744 Float,
:962-996 Bool, :409-443 default/Enum).

HybridParticle.move calls, for every param,
    op3_swarm(position, global_best, self.best, c=omega, c1=phi_g, c2=phi_l, velocity=v)
so with cfg = x, cfg1 = g, cfg2 = l:
    v' = v*c + (g - x)*c1*r1 + (l - x)*c2*r2            (draw order r1, r2)
  Float:  x' = min(vmax, max(x + v', vmin))          (LogInt: on log values, then _unscale)
  Int:    s = k / (1 + exp(-v')) + vmin,  p ~ N(s, (sigma k)^2),  x' = int(min(vmax, max(round(p), vmin)))
          (PowerOfTwo: on exponents, then 2 ** x')
  Bool:   s = 1 / (1 + exp(-v')),  x' = (s - U) > 0
  Enum:   opn_stochastic_mix(cfg, [cfg, g, l], [c, c1, c2]) copies FROM the particle
          INTO the drawn parent (manipulator.py:442) -> the particle's
          value never changes (enum_mode=0, reference); enum_mode=1 copies from
          the drawn parent instead (corrected).
Reference quirk kept by default: `self.best = self.position` aliases the same
dict (pso.py:60, :46), so l == x and the local term is 0 -- pass
pbest = pos to reproduce it.

  Permutation (:1115-1140): if uniform(0,1) > c: op3_cross(cfg, cfg, g if
          uniform(0,1) < c1 else l, xchoice, strength=0.3); velocity None (0 here).
Draws: Philox (seed, g, p, round, OP_PSO): (x,y)->r1, (z,w)->r2 (PERM: the two
uniforms); perm draw site p|1<<28 for the crossover (oracle/perm.py); block
p|1<<28: (x,y) -> U (Bool) / r (Enum); normal draws (Int) from
mathx.normal_draw(stream p|2<<28); exp is mathx.ut_exp.
"""
import numpy as np

from . import perm as pm
from . import philox as ph
from .mathx import normal_draw, ut_exp
from .space import BOOL, ENUM, FLOAT, INT, LOGINT, PERM, POW2, columns, scale_vec, unscale_vec, width


def propose_pso_vec(space, pos, vel, pbest, gbest, seed, round_, cand_base, m, omega=0.5, phi_l=0.5, phi_g=0.5,
                    sigma=0.2, enum_mode=0, crossover=pm.X_OX1):
    ncols, npop = pos.shape
    starts, _ = columns(space)
    g = np.arange(cand_base, cand_base + m, dtype=np.uint64)
    t = (g % np.uint64(npop)).astype(np.int64)
    out_x = np.empty((ncols, m))
    out_v = np.empty((ncols, m))
    c, c1, c2 = omega, phi_g, phi_l
    gbest = np.asarray(gbest, dtype=np.float64)
    for p, prm in enumerate(space):
        c0 = starts[p]
        if prm.kind == PERM:
            S = width(prm)
            r = ph.draw(seed, g, p, round_, ph.OP_PSO)
            u1, u2 = ph.u01(r[0], r[1]), ph.u01(r[2], r[3])
            for j in range(m):
                x = [int(a) for a in pos[c0:c0 + S, t[j]]]
                if u1[j] > c:
                    other = gbest[c0:c0 + S] if u2[j] < c1 else pbest[c0:c0 + S, t[j]]
                    W = pm.Words(seed, g[j], p | (1 << ph.STREAM_SUB_SHIFT), round_, ph.OP_PSO)
                    x = pm.cross(crossover, x, [int(a) for a in other], pm.swarm_d(S), W)
                out_x[c0:c0 + S, j] = x
            out_v[c0:c0 + S] = 0.0
            continue
        p_ = c0
        # scaled kinds move in their search scale (get_value/set_value):
        # LOGINT by the Float rule on log values, POW2 by the Int rule on exponents
        x = scale_vec(prm, pos[p_, t])
        v = vel[p_, t]
        lb = scale_vec(prm, pbest[p_, t])
        gb = float(scale_vec(prm, np.array([gbest[p_]]))[0])
        vmin, vmax = (float(b) for b in prm.legal_range()) if prm.is_primitive() else (0.0, 0.0)
        r = ph.draw(seed, g, p, round_, ph.OP_PSO)
        r1, r2 = ph.u01(r[0], r[1]), ph.u01(r[2], r[3])
        if prm.kind == ENUM:
            nv = v
            if enum_mode == 1:
                q = ph.draw(seed, g, p | (1 << ph.STREAM_SUB_SHIFT), round_, ph.OP_PSO)
                rr = ph.u01(q[0], q[1])
                tot = c + c1 + c2
                w0, w1 = c / tot, c1 / tot
                nx = np.where(rr < w0, x, np.where(rr < w0 + w1, gb, lb))
            else:
                nx = x
        else:
            nv = ((v * c) + (((gb - x) * c1) * r1)) + (((lb - x) * c2) * r2)
            if prm.kind in (FLOAT, LOGINT):
                y = x + nv
                y = np.where(vmin > y, vmin, y)           # max(p, vmin)
                nx = unscale_vec(prm, np.where(y < vmax, y, vmax))   # min(vmax, .); set_value
            elif prm.kind in (INT, POW2):
                k = vmax - vmin
                s = k / (1.0 + ut_exp(-nv)) + vmin
                z = normal_draw(seed, g, p | (2 << ph.STREAM_SUB_SHIFT), round_, ph.OP_PSO)
                pp = np.rint(s + z * (sigma * k))
                pp = np.where(vmin > pp, vmin, pp)
                nx = unscale_vec(prm, np.where(pp < vmax, pp, vmax))
            elif prm.kind == BOOL:
                s = 1.0 / (1.0 + ut_exp(-nv))
                q = ph.draw(seed, g, p | (1 << ph.STREAM_SUB_SHIFT), round_, ph.OP_PSO)
                nx = ((s - ph.u01(q[0], q[1])) > 0).astype(np.float64)
            else:
                raise NotImplementedError(prm.kind)
        out_x[p_] = nx
        out_v[p_] = nv
    return out_x, out_v
