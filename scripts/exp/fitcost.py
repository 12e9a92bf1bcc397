import sys, time, os
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
import numpy as np, torch
import bench
from uptune_amd.engine import BatchEngine
from uptune_amd.manipulator import ConfigurationManipulator, FloatParameter
m, n, d, k = 1 << 20, 1024, 64, 256
eng = BatchEngine(ConfigurationManipulator([FloatParameter(i, -1000.0, 1000.0) for i in range(d)]), seed=1)
eng.population_init(m); eng.history_reset(0)
X, y = bench.training_set(n, d, 101)
acq = eng.acq("ei", xi=0.0)
def run(fit_each, steps=10):
    for r in range(3):
        eng.gp_fit(X, y, lengthscale=0.2, sigma_f2=1.0, sigma_n2=1e-6, wait=False)
        eng.score_round_de(m, k, round_=r, acq=acq, want_values=False)
    torch.cuda.synchronize(); t0 = time.perf_counter()
    for r in range(steps):
        if fit_each:
            eng.gp_fit(X, y, lengthscale=0.2, sigma_f2=1.0, sigma_n2=1e-6, wait=False)
        eng.score_round_de(m, k, round_=r + 3, acq=acq, want_values=False)
    torch.cuda.synchronize(); return (time.perf_counter() - t0) / steps * 1e3
print("fit each round: %.2f ms" % run(True))
print("no refit:       %.2f ms" % run(False))
print("fit each round: %.2f ms" % run(True))
