"""The GP fit alone (refit, waited on), n = 1024 / 4096 / 4480, d = 64: host
wall time per ut_gp_fit including its device work.  Env knobs of the library
(UT_CHOL_FUSE) select the variant."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from uptune_amd.engine import BatchEngine  # noqa: E402
from uptune_amd.manipulator import ConfigurationManipulator, FloatParameter  # noqa: E402

d = 64
eng = BatchEngine(ConfigurationManipulator([FloatParameter(i, 0.0, 1.0) for i in range(d)]), seed=1)
eng.gp_set_fit_append(False)
rng = np.random.default_rng(0)
for n in (1024, 4096, 4480):
    X = rng.uniform(size=(n, d))
    y = np.sum((X - 0.4) ** 2, axis=1)
    eng.gp_fit(X, y, lengthscale=1.0, sigma_f2=1.0, sigma_n2=1e-6, jitter=1e-8)
    t = []
    for _ in range(5):
        t0 = time.perf_counter()
        eng.gp_fit(X, y, lengthscale=1.0, sigma_f2=1.0, sigma_n2=1e-6, jitter=1e-8)
        t.append(time.perf_counter() - t0)
    print(f"n={n}: fit {min(t) * 1e3:.2f} ms  stats {eng.gp_stats()}", flush=True)
