"""The search loop over the GPU techniques (BASELINE.json configs[4], "C5"):
an AUC bandit over DE + PSO + GA + GGA sharing one GP surrogate, on one GPU
or SPMD over N GPUs (one process per GPU, torch.distributed).

Per generation the driver asks the bandit for `parallelism` configurations
(bandittechniques.py:150-165 -> metatechniques.py:40-57 -> the technique's
desired_configuration()).  A GPU technique whose queue is empty runs one
scoring round: propose its pool (sharded over the ranks by global candidate
index) -> hash_config -> dedup against every configuration seen -> GP-EI on
the results so far -> local top-k -> all-gather merge.  Rank 0 evaluates the
generation and broadcasts the results (DistributedSearchDriver), which is
the reference's batch dispatch + api.sync (api.py:428-482, :547-553).
"""
from __future__ import annotations

from typing import Any, Callable, Dict, Optional

from .driver import DistributedSearchDriver, SearchDriver
from .technique import pso_ga_de_bandit


def random_configs(manipulator, n: int, seed: int, device: int = 0, with_keys: bool = False):
    """n configurations drawn by op1_randomize on the device (manipulator.random());
    with_keys: also their hash_config hex digests, hashed on the device from the
    drawn values (no host re-encoding)"""
    from .engine import BatchEngine, digests_to_hex
    eng = BatchEngine(manipulator, device=device, seed=seed)
    try:
        eng.population_init(max(n, 4), round_=0)
        vals = eng.population_get()[:, :n].contiguous()
        cfgs = eng.decode(vals)
        return (cfgs, digests_to_hex(eng.hash(vals))) if with_keys else cfgs
    finally:
        eng.close()


def tune_bandit(manipulator, objective: Callable[[Dict[Any, Any]], float], generations: int = 100,
                parallelism: int = 4, n_init: int = 0, pool: int = 1 << 16, batch: int = 8, population: int = 1024,
                seed: int = 0, lengthscale: float = 0.3, device: int = 0, group=None,
                precision: int = 64, prune_rows: int = 0) -> SearchDriver:
    """Run the bandit for `generations` generations; returns the driver (results,
    best_result, bandit statistics).  With torch.distributed initialised and
    world > 1 the run is SPMD: call it on every rank with the same arguments."""
    import torch.distributed as dist
    world = dist.get_world_size(group) if dist.is_available() and dist.is_initialized() else 1
    meta = pso_ga_de_bandit(bandit_seed=seed, pool=pool, batch=batch, population=population, seed=seed,
                            device=device, lengthscale=lengthscale, group=group, precision=precision,
                            prune_rows=prune_rows)
    if world > 1:
        import torch
        drv = DistributedSearchDriver(manipulator, meta, parallelism=parallelism, group=group,
                                      device=torch.device("cuda", device) if dist.get_backend(group) != "gloo"
                                      else None)
    else:
        drv = SearchDriver(manipulator, meta, parallelism=parallelism)
    import time
    t0 = time.perf_counter()
    if n_init:
        cfgs, keys = random_configs(manipulator, n_init, seed + 7919, device, with_keys=True)
        drv.seed_results(cfgs, objective, keys=keys)
    drv.seed_s = time.perf_counter() - t0    # initial design: draw, evaluate, record (host)
    drv.main(objective, test_limit=generations * parallelism, max_generations=generations)
    return drv
