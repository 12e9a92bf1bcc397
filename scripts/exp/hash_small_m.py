"""ut_hash at small m (PSO swarms, small pools): device time per call on the
R64 and HPL-64 spaces, m = 2^12 .. 2^17.  UTHOT_LIB picks the library build."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from uptune_amd import spaces  # noqa: E402
from uptune_amd.engine import BatchEngine  # noqa: E402

torch.cuda.set_device(0)
for name, manip in (("r64", spaces.r64()), ("hpl64", spaces.hpl64())):
    eng = BatchEngine(manip, device=0, seed=3)
    for lg in (12, 14, 15, 16, 17):
        m = 1 << lg
        eng.population_init(m)
        v = eng.population_get()
        ref = eng.hash(v)
        torch.cuda.synchronize()
        t = []
        for _ in range(5):
            t0 = time.perf_counter()
            d = eng.hash(v)
            torch.cuda.synchronize()
            t.append(time.perf_counter() - t0)
        assert torch.equal(d, ref)
        print(f"{name} m=2^{lg}: {min(t) * 1e3:.3f} ms  digest0 {d[0, 0].item() & 0xffffffff:08x}", flush=True)
    eng.close()
