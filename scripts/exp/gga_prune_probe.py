"""Why the C5 loop's GGA round falls back to the dense variance when pruned,
and whether a bound from the LAST training rows would prune it: capture the
GGA round's candidates and the shared model's training set, then run
ut_gp_topk_pruned on them with the training set in its own order (the prefix
bound = the first rows, as shipped) and reversed (the prefix bound = the most
recent rows), and with the best-y rows first.  Prints survivors / dense."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from scripts.c5_bandit import rosenbrock64  # noqa: E402
from uptune_amd import spaces  # noqa: E402
from uptune_amd import technique as T  # noqa: E402
from uptune_amd.tuner import tune_bandit  # noqa: E402

cap = {}


def make_spy(cls, key, at_round):
    orig = cls._local_round

    def spy(self):
        out = orig(self)
        if key not in cap and self.round >= at_round:
            cap[key] = dict(vals=out[0].clone(), X=self.model._Xa[:self.model._n].copy(), y=self.model._ya[:self.model._n].copy(),
                            eng=self.engine, round=self.round)
        return out
    cls._local_round = spy


make_spy(T.GpuGGA, "gga", 0)
make_spy(T.GpuGA, "ga", 20)
torch.cuda.set_device(0)
tune_bandit(spaces.r64(), rosenbrock64, generations=100, parallelism=4, n_init=4096, pool=1 << 18, batch=8,
            population=4096, seed=1, lengthscale=0.3, prune_rows=256)
import time  # noqa: E402
for key in ("gga", "ga"):
    if key not in cap:
        continue
    c = cap[key]
    eng = c["eng"]
    X, y, vals = c["X"], c["y"], c["vals"]
    print(key, "round", c["round"], "training", X.shape, "best row", int(np.argmin(y)), "of", len(y))
    feat = eng.encode(vals)
    acq = eng.acq("ei")
    for name, order in (("as fitted", np.arange(len(y))), ("reversed", np.arange(len(y))[::-1]),
                        ("best-y first", np.argsort(y, kind="stable"))):
        eng.gp_fit(X[order], y[order], lengthscale=0.3, sigma_f2=1.0, sigma_n2=1e-6, jitter=1e-8)
        for rows in (256, 512):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            idx, top, st = eng.gp_topk_pruned(feat, 8, acq=acq, bound_rows=rows)
            torch.cuda.synchronize()
            ms = (time.perf_counter() - t0) * 1e3
            print(f"  {name:14s} bound_rows {rows:5d}: survivors {st['survivors']:7d} of {st['m']} dense {st['dense']} "
                  f"{ms:7.2f} ms top {idx.cpu().numpy().tolist()}")
