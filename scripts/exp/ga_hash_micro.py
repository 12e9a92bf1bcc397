"""ut_hash vs ut_hash_parent on GA children of one parent (R64, m = 2^20,
UniformGreedyMutation 0.1): HIP-event times on the library stream."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from scripts.microbench import timeit  # noqa: E402
from uptune_amd import spaces  # noqa: E402
from uptune_amd.engine import BatchEngine  # noqa: E402

eng = BatchEngine(spaces.r64(), seed=1)
eng.population_init(4096)
p = eng.population_get()[:, 0].contiguous()
kids, _ = eng.propose_ga(1 << 20, parent1=p, mutation_rate=0.1)
print("GA children, m=2^20: hash %.3f ms, hash_parent %.3f ms" % (timeit(lambda: eng.hash(kids)),
      timeit(lambda: eng.hash_parent(kids, p))), flush=True)
