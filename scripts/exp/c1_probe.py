"""C1 probe: AUCBanditMetaTechniqueA's device counterpart (technique.bandit_a) on
2-D Rosenbrock over [-1000, 1000]^2, test-limit 5000, under model variants:
the GP on raw times, on rank normal scores, or no model (the reference's
techniques have none: selections in proposal order).  Prints best and wall."""
import sys
import time

import numpy as np

sys.path.insert(0, ".")
from uptune_amd import technique as T  # noqa: E402
from uptune_amd.driver import SearchDriver  # noqa: E402
from uptune_amd.manipulator import ConfigurationManipulator, FloatParameter  # noqa: E402


def rosen(cfg):
    x0, x1 = cfg[0], cfg[1]
    return 100.0 * (x1 - x0 * x0) ** 2 + (x0 - 1.0) ** 2


VARIANTS = {
    "gp_raw_l0.3": dict(lengthscale=0.3),
    "no_model": dict(min_train=10 ** 9),
    "gp_rank_l0.3": dict(lengthscale=0.3, y_transform="rank"),
    "gp_rank_l0.1": dict(lengthscale=0.1, y_transform="rank"),
    "gp_rank_l0.03": dict(lengthscale=0.03, y_transform="rank"),
    "p30_no_model": dict(min_train=10 ** 9, population=30),
    "p30_gp_raw": dict(lengthscale=0.3, population=30),
    "p30_gp_rank_l0.3": dict(lengthscale=0.3, y_transform="rank", population=30),
    "p30_gp_rank_l0.1": dict(lengthscale=0.1, y_transform="rank", population=30),
    "p30_pool256_rank": dict(lengthscale=0.1, y_transform="rank", population=30, pool=256),
    "p30_pool256_none": dict(min_train=10 ** 9, population=30, pool=256),
}

for name in (sys.argv[1:] or VARIANTS):
    for seed in (11, 12, 13):
        m = ConfigurationManipulator([FloatParameter(0, -1000.0, 1000.0), FloatParameter(1, -1000.0, 1000.0)])
        kw = dict(pool=4096, batch=8, population=256)
        kw.update(VARIANTS[name])
        meta = T.bandit_a(bandit_seed=5, seed=seed, **kw)
        d = SearchDriver(m, meta, parallelism=4)
        t0 = time.time()
        best = d.main(rosen, test_limit=5000)
        dt = time.time() - t0
        b = d.root_technique.bandit
        print("%-14s seed %d best %.6g tests %d wall %.1fs uses %s" % (name, seed, best.time, d.test_count, dt,
                                                                      dict(b.use_counts)), flush=True)
