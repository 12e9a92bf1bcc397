"""k_de alone: member-major donor staging (UT_DE_AOS=1) vs column-major gathers
(UT_DE_AOS=0) on the C2 R64 space and the C3 HPL-64 space, m = 2^20 candidates
over a population of 2^20.  Prints ms per launch (median of HIP-event times)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from uptune_amd import spaces  # noqa: E402
from uptune_amd.engine import BatchEngine  # noqa: E402
from uptune_amd.manipulator import ConfigurationManipulator, FloatParameter  # noqa: E402


def timeit(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for a, b in ev:
        a.record()
        fn()
        b.record()
    torch.cuda.synchronize()
    return float(np.median([a.elapsed_time(b) for a, b in ev]))


m = int(os.environ.get("M", 1 << 20))
npop = int(os.environ.get("NPOP", m))
for name, mk in (("r64", lambda: ConfigurationManipulator([FloatParameter(i, -1000.0, 1000.0) for i in range(64)])),
                 ("hpl64", spaces.hpl64)):
    res = {}
    outs = {}
    for aos in ("1", "0"):
        os.environ["UT_DE_AOS"] = aos
        eng = BatchEngine(mk(), seed=1)
        eng.population_init(npop)
        res[aos] = timeit(lambda: eng.propose_de(m, round_=1, cr=0.2))
        outs[aos] = eng.propose_de(m, round_=2, cr=0.2).cpu().numpy()
        eng.close()
    same = np.array_equal(outs["1"].view(np.uint64), outs["0"].view(np.uint64))
    print(f"npop={npop} {name}: aos {res['1']:.3f} ms  soa {res['0']:.3f} ms  identical={same}", flush=True)
