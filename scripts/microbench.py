"""Per-kernel microbenchmarks on synthetic inputs (one process, HIP events on
the library stream).  Usage: python scripts/microbench.py [hash|fit|score|forest|all]"""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from uptune_amd.engine import BatchEngine  # noqa: E402
from uptune_amd.manipulator import (ConfigurationManipulator, EnumParameter, FloatParameter,  # noqa: E402
                                    IntegerParameter)


def timeit(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for a, b in ev:
        a.record()
        fn()
        b.record()
    torch.cuda.synchronize()
    return float(np.median([a.elapsed_time(b) for a, b in ev]))


def bench_hash(m=1 << 20):
    out = {}
    spaces = {
        "r64_float": [FloatParameter(i, -1000.0, 1000.0) for i in range(64)],
        "int64_lut": [IntegerParameter(i, 0, 1000) for i in range(64)],
        "int64_repr": [IntegerParameter(i, 0, 10**9) for i in range(64)],
        "enum64": [EnumParameter(i, ["on", "off", "default"]) for i in range(64)],
    }
    for name, params in spaces.items():
        eng = BatchEngine(ConfigurationManipulator(params), seed=1)
        eng.population_init(m)
        vals = eng.population_get()
        ms = timeit(lambda: eng.hash(vals))
        L, nb, _ = eng.space_info()
        out[name] = {"ms": ms, "outer_blocks": nb, "ns_per_cand": ms * 1e6 / m}
        if name == "r64_float":   # the bench's input: DE-Alt trials of that population
            trial = eng.propose_de(m, round_=1, cr=0.2)
            ms = timeit(lambda: eng.hash(trial))
            out["r64_de_trials"] = {"ms": ms, "outer_blocks": nb, "ns_per_cand": ms * 1e6 / m}
            # the same trials through ut_hash_de (target inner digests reused; the
            # population cache is built by the warm-up call)
            ms = timeit(lambda: eng.hash_de(trial, 0))
            out["r64_de_trials_reuse"] = {"ms": ms, "outer_blocks": nb, "ns_per_cand": ms * 1e6 / m}
            # the outer message alone (every inner digest reused: trial == population)
            ms = timeit(lambda: eng.hash_de(vals, 0))
            out["r64_outer_only"] = {"ms": ms, "outer_blocks": nb, "ns_per_cand": ms * 1e6 / m}
        del eng
    return out


def synthetic_forest(n_trees=300, depth=10, d=64, seed=0):
    """complete binary trees of the reference's XGB size (plugins/xgbregressor.py:
    n_estimators=300, max_depth=10) with random splits"""
    from uptune_amd import _lib as L
    from uptune_amd.forest import NODE_DTYPE, Forest
    rng = np.random.default_rng(seed)
    per = (1 << (depth + 1)) - 1
    nodes = np.zeros(n_trees * per, dtype=NODE_DTYPE)
    for t in range(n_trees):
        o = t * per
        k = np.arange(per)
        inner = k < (1 << depth) - 1
        nodes["feature"][o:o + per] = np.where(inner, rng.integers(0, d, per), -1)
        nodes["left"][o:o + per] = np.where(inner, o + 2 * k + 1, 0)
        nodes["right"][o:o + per] = np.where(inner, o + 2 * k + 2, 0)
        nodes["threshold"][o:o + per] = rng.uniform(size=per)
        nodes["value"][o:o + per] = np.where(inner, 0.0, rng.normal(size=per) * 0.01)
    return Forest(nodes, np.arange(n_trees, dtype=np.int32) * per, L.UT_SPLIT_LT, 0.5, 1.0, 1.0)


def bench_forest(m=1 << 20, d=64):
    eng = BatchEngine(ConfigurationManipulator([FloatParameter(i, 0.0, 1.0) for i in range(d)]), seed=1)
    out = {}
    for n_trees, depth in ((300, 10), (100, 6)):
        f = synthetic_forest(n_trees, depth, d)
        eng.forest_set(f)
        feat = torch.rand(d, m, dtype=torch.float64, device="cuda")
        ms = timeit(lambda: eng.forest_predict(feat))
        visits = n_trees * (depth + 1)
        out[f"{n_trees}x{depth}"] = {"ms": ms, "cands_per_s": m / ms * 1e3, "node_visits_per_cand": visits,
                                     "node_bytes_GBps": m * visits * 32 / ms / 1e6}
    return out


def bench_fit(d=64):
    """ut_gp_fit latency (Cholesky, L^-1, alpha on the device) by training-set size"""
    out = {}
    eng = BatchEngine(ConfigurationManipulator([FloatParameter(i, 0.0, 1.0) for i in range(d)]), seed=1)
    rng = np.random.default_rng(0)
    for n in (256, 1024, 2048, 4096):
        X = rng.uniform(size=(n, d))
        y = np.sum((X - 0.4) ** 2, axis=1)
        eng.gp_fit(X, y, lengthscale=0.5, sigma_f2=1.0, sigma_n2=1e-6, jitter=1e-8)
        torch.cuda.synchronize()
        ts = []
        for _ in range(5):
            t0 = time.perf_counter()
            eng.gp_fit(X, y, lengthscale=0.5, sigma_f2=1.0, sigma_n2=1e-6, jitter=1e-8)
            ts.append((time.perf_counter() - t0) * 1e3)
        out[n] = {"ms": float(np.median(ts))}
    return out


def bench_score(m=1 << 20, d=64):
    """standalone ut_gp_score stages (K*, variance) at C2 shapes, fp64 and fp32,
    with nothing running beside them"""
    out = {}
    eng = BatchEngine(ConfigurationManipulator([FloatParameter(i, 0.0, 1.0) for i in range(d)]), seed=1)
    rng = np.random.default_rng(0)
    X = rng.uniform(size=(1024, d))
    y = np.sum((X - 0.4) ** 2, axis=1)
    feat = torch.rand(d, m, dtype=torch.float64, device="cuda")
    for prec in (64, 32):
        eng.gp_set_precision(prec)
        eng.gp_fit(X, y, lengthscale=0.2, sigma_f2=1.0, sigma_n2=1e-6)
        eng.gp_score(feat)
        torch.cuda.synchronize()
        eng.set_timing(True)            # stage times are averaged over the calls from here
        for _ in range(5):
            eng.gp_score(feat)
        torch.cuda.synchronize()
        out[f"fp{prec}"] = {st: eng.stage_time(st) for st in ("kstar", "var")}
        eng.set_timing(False)
    eng.gp_set_precision(64)
    return out


if __name__ == "__main__":
    which = sys.argv[1] if len(sys.argv) > 1 else "all"
    res = {}
    if which in ("hash", "all"):
        res["hash"] = bench_hash()
    if which in ("fit", "all"):
        res["fit"] = bench_fit()
    if which in ("score", "all"):
        res["score"] = bench_score()
    if which in ("forest", "all"):
        res["forest"] = bench_forest()
    print(json.dumps(res, indent=1))
