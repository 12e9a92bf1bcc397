"""Where the C5 pruned loop's wall time goes, without cProfile's per-call
overhead: wrap the loop's stages with perf_counter accumulators (inclusive
times; a stage that waits on the device includes the wait) and run the same
tune_bandit call as scripts/c5_bandit.py --prune 256."""
import collections
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from scripts.c5_bandit import rosenbrock64  # noqa: E402
from uptune_amd import driver as D  # noqa: E402
from uptune_amd import engine as E  # noqa: E402
from uptune_amd import spaces  # noqa: E402
from uptune_amd import technique as T  # noqa: E402
from uptune_amd.tuner import tune_bandit  # noqa: E402

acc = collections.defaultdict(float)
cnt = collections.Counter()


def wrap(cls, name, key=None):
    orig = getattr(cls, name)
    key = key or f"{cls.__name__}.{name}"

    def f(*a, **k):
        t = time.perf_counter()
        try:
            return orig(*a, **k)
        finally:
            acc[key] += time.perf_counter() - t
            cnt[key] += 1
    setattr(cls, name, f)


for cls, names in ((T.SharedModel, ("sync_history", "fit")),
                   (T.GpuBatchTechnique, ("_round", "_local_round", "propose", "hash_proposals", "desired_configuration")),
                   (T.GpuGA, ("propose", "hash_proposals")),
                   (T.GpuDifferentialEvolution, ("propose", "hash_proposals", "after_round", "handle_requested_result")),
                   (T.GpuPSO, ("propose",)),
                   (T.AUCBanditMetaTechnique, ("select_technique_order", "on_technique_result")),
                   (T.MetaSearchTechnique, ("desired_result",)),
                   (E.BatchEngine, ("gp_topk_pruned", "gp_fit", "features_host", "dedup", "encode", "decode",
                                    "history_add", "gp_join_fit")),
                   (D.SearchDriver, ("run_generation_techniques", "run_generation_results", "process_new_results",
                                     "report", "results_query", "configuration_from_digest"))):
    for n in names:
        if n in cls.__dict__:
            wrap(cls, n)
wrap(E, "digests_to_hex", "digests_to_hex")
T_digests = E.digests_to_hex

torch.cuda.set_device(0)
tune_bandit(spaces.r64(), rosenbrock64, generations=3, parallelism=4, n_init=512, pool=1 << 18, batch=8,
            population=4096, seed=2, lengthscale=0.3, prune_rows=256)
torch.cuda.synchronize()
for reps in range(2):
    acc.clear()
    cnt.clear()
    t0 = time.perf_counter()
    drv = tune_bandit(spaces.r64(), rosenbrock64, generations=100, parallelism=4, n_init=4096, pool=1 << 18,
                      batch=8, population=4096, seed=1, lengthscale=0.3, prune_rows=256)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    print(json.dumps({"wall_s": wall, "seed_s": drv.seed_s, "best": drv.best_result.time}))
    for k, v in sorted(acc.items(), key=lambda kv: -kv[1]):
        print(f"  {v * 1e3:8.2f} ms {cnt[k]:6d} {k}")
