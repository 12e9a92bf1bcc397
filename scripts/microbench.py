"""Per-kernel microbenchmarks on synthetic inputs (one process, HIP events on
the library stream).  Usage: python scripts/microbench.py [hash|gp|all]"""
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
        del eng
    return out


if __name__ == "__main__":
    which = sys.argv[1] if len(sys.argv) > 1 else "all"
    res = {}
    if which in ("hash", "all"):
        res["hash"] = bench_hash()
    print(json.dumps(res, indent=1))
