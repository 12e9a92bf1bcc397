"""k_gp_kstar alone (HIP-event stage times on the library stream, nothing
beside it): C2 shape fp64 (ut_gp_score: plain K*), C2 fp32 (K* with the mean
partial), C2 precision 8 (the mean partial and six int8 digit planes), and the C3 shape (n = 4096, d = 119) through ut_gp_topk_pruned (K*
with the mean and |k*|^2 partials, bound rows stored).  UTHOT_LIB picks the
library build to time."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from uptune_amd.engine import BatchEngine  # noqa: E402
from uptune_amd.manipulator import ConfigurationManipulator, FloatParameter  # noqa: E402


def run(d, n, m, ell, mode, reps=5):
    eng = BatchEngine(ConfigurationManipulator([FloatParameter(i, 0.0, 1.0) for i in range(d)]), seed=1)
    rng = np.random.default_rng(0)
    X = rng.uniform(size=(n, d))
    y = np.sum((X - 0.4) ** 2, axis=1)
    feat = torch.rand(d, m, dtype=torch.float64, device="cuda")
    eng.gp_set_precision({"f32": 32, "i8": 8}.get(mode, 64))
    eng.gp_fit(X, y, lengthscale=ell, sigma_f2=1.0, sigma_n2=1e-6)
    call = (lambda: eng.gp_topk_pruned(feat, 256, bound_rows=128)) if mode == "pruned" else (lambda: eng.gp_score(feat))
    call()
    torch.cuda.synchronize()
    eng.set_timing(True)
    for _ in range(reps):
        call()
    torch.cuda.synchronize()
    t = eng.stage_time("kstar")
    eng.set_timing(False)
    eng.close()
    return t


CASES = {"c2_f64": (64, 1024, 1 << 20, 0.2, "f64"), "c2_f32_mu": (64, 1024, 1 << 20, 0.2, "f32"),
         "c2_i8_mu": (64, 1024, 1 << 20, 0.2, "i8"), "c3_pruned_mu": (119, 4096, 1 << 21, 1.0, "pruned")}
if len(sys.argv) > 1:   # a subset (profiling runs)
    res = {k: run(*CASES[k]) for k in sys.argv[1:]}
    print(os.environ.get("UTHOT_LIB", "default"), json.dumps({k: round(v, 3) for k, v in res.items()}), flush=True)
    sys.exit(0)
res = {"c2_f64": run(64, 1024, 1 << 20, 0.2, "f64"),
       "c2_f32_mu": run(64, 1024, 1 << 20, 0.2, "f32"),
       "c2_i8_mu": run(64, 1024, 1 << 20, 0.2, "i8"),
       "c3_pruned_mu": run(119, 4096, 1 << 21, 1.0, "pruned")}
print(os.environ.get("UTHOT_LIB", "default"), json.dumps({k: round(v, 3) for k, v in res.items()}), flush=True)
