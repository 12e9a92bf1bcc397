import sys, numpy as np, torch
sys.path.insert(0, "."); sys.path.insert(0, "tests")
from oracle import de as ode, pso as opso, perm as opm, philox as ph
from oracle.space import columns
from _spaces import oracle_space, to_manip
from uptune_amd import spaces
from uptune_amd.engine import BatchEngine
space = oracle_space(spaces.perm_mixed())
e = BatchEngine(to_manip(space), device=0, seed=29)
pop = ode.population_init(space, 600, seed=8)
e.population_set(torch.from_numpy(pop).cuda()); e.pso_reset()
gbest = pop[:, 7].copy()
x, v = e.propose_pso(gbest, 600, round_=2, alias_pbest=True, crossover="op3_cross_OX1")
wx, wv = opso.propose_pso_vec(space, pop, np.zeros_like(pop), pop, gbest, 29, 2, 0, 600, crossover=1)
x = x.cpu().numpy()
bad = np.argwhere(x != wx)
print("bad rows", sorted(set(bad[:, 0].tolist()))[:80])
cands = sorted(set(bad[:, 1].tolist()))
print("n bad cands", len(cands), cands[:20])
starts, nc = columns(space)
print("starts", starts)
j = cands[0]
g = np.array([j], dtype=np.uint64)
for p, prm in enumerate(space):
    c0 = starts[p]
    if prm.kind == 6:
        S = len(prm.options)
        r = ph.draw(29, g, p, 2, ph.OP_PSO)
        print(p, prm.name, "u1", ph.u01(r[0], r[1]), "u2", ph.u01(r[2], r[3]))
        print(" pos ", pop[c0:c0+S, j].astype(int).tolist())
        print(" gb  ", gbest[c0:c0+S].astype(int).tolist())
        print(" dev ", x[c0:c0+S, j].astype(int).tolist())
        print(" orc ", wx[c0:c0+S, j].astype(int).tolist())
        W = opm.Words(29, j, p | (1 << 28), 2, 3)
        print(" w0", W[0], W[1])
