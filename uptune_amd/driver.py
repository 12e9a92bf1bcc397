"""Minimal in-memory search driver with the reference SearchDriver's semantics.

This is the caller side of the plugin boundary, kept just large enough to run
a technique tree end to end without the reference's SQL
results database:

  get_configuration (hash identity)            opentuner/search/driver.py:253-258
  register_result_callback / result_callbacks   driver.py:130-155
  run_generation_techniques (dup requests)      driver.py:160-207
  process_new_results (was_new_best, best)      driver.py:209-225
  MinimizeTime.lt                               opentuner/search/objective.py:161-183
  convergence by test_limit                     driver.py:113-128

A configuration's identity is its hash_config digest, computed on the device
by the same kernel the GPU techniques use (GPU path), or by a host callable
passed as `hash_fn` (CPU-only plumbing tests supply hashlib-based hashing).
"""
from __future__ import annotations

import copy
from typing import Any, Callable, Dict, List, Optional

import numpy as np


class Result:
    __slots__ = ("configuration", "time", "was_new_best", "requestor", "state")

    def __init__(self, configuration, time: float, requestor: str = ""):
        self.configuration = configuration
        self.time = float(time)
        self.was_new_best = None
        self.requestor = requestor
        self.state = "OK"


class DesiredResult:
    __slots__ = ("configuration", "key", "requestor", "generation", "result", "state")

    def __init__(self, configuration, key: str, requestor: str, generation: int):
        self.configuration = configuration
        self.key = key
        self.requestor = requestor
        self.generation = generation
        self.result: Optional[Result] = None
        self.state = "REQUESTED"


class MinimizeTime:
    """objective.py:161-183: compare results on .time"""

    def lt(self, a: Result, b: Result) -> bool:
        return a.time < b.time

    def lte(self, a: Result, b: Result) -> bool:
        return a.time <= b.time

    def relative(self, a: Result, b: Result) -> float:
        return a.time / b.time if b.time else float("inf")


class SearchDriver:
    def __init__(self, manipulator, root_technique, objective=None, parallelism: int = 4,
                 hash_fn: Optional[Callable[[Dict[Any, Any]], str]] = None):
        self.manipulator = manipulator
        self.objective = objective or MinimizeTime()
        self.parallelism = parallelism
        self._hash_fn = hash_fn
        # techniques are deep-copied into every driver (driver.py:75)
        self.root_technique = copy.deepcopy(root_technique)
        self.generation = 0
        self.test_count = 0
        self.best_result: Optional[Result] = None
        self.results: Dict[str, Result] = {}        # config key -> first result
        self._seen: List[str] = []                  # every key ever requested, in order
        self._requested: Dict[str, DesiredResult] = {}
        self.pending_result_callbacks: List = []
        self.new_results: List[Result] = []
        self._unprocessed: List[Result] = []
        self._pop_results: Dict[tuple, Result] = {}
        self.root_technique.set_driver(self)

    # -- identity ----------------------------------------------------------
    def config_key(self, cfg) -> str:
        if self._hash_fn is not None:
            return self._hash_fn(cfg)
        return self.manipulator.hash_config(cfg)

    def config_keys(self, cfgs) -> List[str]:
        """keys of many configurations (one batched device hash)"""
        if self._hash_fn is not None:
            return [self._hash_fn(c) for c in cfgs]
        from .engine import default_engine
        return default_engine(self.manipulator).hash_configs(cfgs) if len(cfgs) else []

    def record_seed(self, cfgs, times, keys=None) -> None:
        """bootstrap history: already-evaluated configurations (an initial design,
        or results loaded from a previous run) become results of generation 0"""
        keys = keys if keys is not None else self.config_keys(cfgs)
        for cfg, t, key in zip(cfgs, times, keys):
            if key in self._requested:
                continue
            dr = DesiredResult(cfg, key, "seed", self.generation)
            self._requested[key] = dr
            self._seen.append(key)
            self.report(dr, t)
        self.process_new_results()

    def seed_results(self, cfgs, evaluate) -> None:
        self.record_seed(cfgs, [evaluate(c) for c in cfgs])

    def seen_hashes(self) -> List[str]:
        return self._seen

    def has_results(self, cfg) -> bool:
        return self.config_key(cfg) in self.results

    # -- technique-facing --------------------------------------------------
    def make_desired_result(self, cfg, requestor: str) -> DesiredResult:
        return DesiredResult(cfg, self.config_key(cfg), requestor, self.generation)

    def register_result_callback(self, dr: DesiredResult, callback) -> None:
        if dr.result is not None:
            callback(dr.result)
        else:
            self.pending_result_callbacks.append((dr, callback))

    def result_callbacks(self) -> None:
        pending, self.pending_result_callbacks = self.pending_result_callbacks, []
        for dr, cb in pending:
            if dr.result is None and dr.key in self.results:
                dr.result = self.results[dr.key]
            if dr.result is not None:
                cb(dr.result)
            else:
                self.pending_result_callbacks.append((dr, cb))

    def best_configuration(self):
        return None if self.best_result is None else self.best_result.configuration

    def training_configs(self):
        """(configurations, times) of every result, in arrival order"""
        keys = list(self.results)
        cfgs = [self.results[k].configuration for k in keys]
        y = np.array([self.results[k].time for k in keys], dtype=np.float64)
        return cfgs, y

    def population_result(self, tech, idx) -> Optional[Result]:
        return self._pop_results.get((tech.name, idx))

    def set_population_result(self, tech, idx, result) -> None:
        self._pop_results[(tech.name, idx)] = result

    # -- generation loop ---------------------------------------------------
    def run_generation_techniques(self) -> List[DesiredResult]:
        """driver.py:160-207: ask the root technique up to `parallelism` times;
        a repeated configuration is not re-evaluated, it receives the earlier
        request's result through a callback."""
        todo = []
        for _ in range(self.parallelism):
            dr = self.root_technique.desired_result()
            if dr is None or dr is False:
                break
            first = self._requested.get(dr.key)
            if first is not None:
                def cb(result, dr=dr):
                    dr.result = result
                    dr.state = "COMPLETE"
                self.register_result_callback(first, cb)
            else:
                self._requested[dr.key] = dr
                self._seen.append(dr.key)
                todo.append(dr)
            self.test_count += 1
        return todo

    def report(self, dr: DesiredResult, time: float) -> Result:
        r = Result(dr.configuration, time, dr.requestor)
        dr.result = r
        dr.state = "COMPLETE"
        self.results.setdefault(dr.key, r)
        self._unprocessed.append(r)
        return r

    def process_new_results(self) -> None:
        """driver.py:209-225"""
        self.new_results = []
        for r in self._unprocessed:
            self.new_results.append(r)
            if self.best_result is None or self.objective.lt(r, self.best_result):
                self.best_result = r
                r.was_new_best = True
            else:
                r.was_new_best = False
        self._unprocessed = []
        self.result_callbacks()

    def main(self, evaluate: Callable[[Dict[Any, Any]], float], test_limit: int = 100,
             max_generations: int = 100000) -> Optional[Result]:
        """SearchDriver.main (driver.py:260-281) with a synchronous evaluator"""
        while self.test_count <= test_limit and self.generation < max_generations:
            todo = self.run_generation_techniques()
            for dr in todo:
                self.report(dr, evaluate(dr.configuration))
            self.process_new_results()
            self.generation += 1
            if not todo and not self.pending_result_callbacks and self.test_count and \
                    self._idle_generations():
                break
        return self.best_result

    def _idle_generations(self) -> bool:
        self._idle = getattr(self, "_idle", 0) + 1
        return self._idle > 50


class DistributedSearchDriver(SearchDriver):
    """SPMD search loop over a torch.distributed group (one process per GPU).

    Every rank runs the same technique tree with the same seeds; the GPU
    techniques shard each round's candidate pool by global index and
    all-gather their local top-k (technique.GpuBatchTechnique), so every rank
    requests the same configurations.  Rank `src` evaluates them and the
    results -- objective values and hash digests, the per-round history delta
    -- are broadcast to every rank (dist.broadcast_results; the reference's
    api.sync result injection, api.py:547-553, and ParallelTuning's batch
    dispatch, api.py:428-482).  The digests double as a consistency check:
    a rank whose requests diverge raises instead of training on wrong data.
    """

    def __init__(self, manipulator, root_technique, objective=None, parallelism: int = 4, hash_fn=None,
                 group=None, src: int = 0, device=None):
        super().__init__(manipulator, root_technique, objective, parallelism, hash_fn)
        self.group, self.src = group, src
        self.device = device

    def seed_results(self, cfgs, evaluate) -> None:
        """rank `src` evaluates the initial design; values + digests are broadcast"""
        import torch
        import torch.distributed as dist

        from .dist import broadcast_results
        from .engine import hex_to_digests
        keys = self.config_keys(cfgs)
        kd = torch.from_numpy(hex_to_digests(keys).view(np.int32).copy())
        src = dist.get_rank(self.group) == self.src
        y = torch.tensor([evaluate(c) for c in cfgs], dtype=torch.float64) if src else None
        dev = self.device if self.device is not None else torch.device("cpu")
        y, dig = broadcast_results(y, kd if src else None, len(cfgs), dev, self.src, self.group)
        if dig.shape[0] != len(cfgs) or not torch.equal(dig.cpu(), kd):
            raise RuntimeError("initial design differs between ranks")
        self.record_seed(cfgs, y.cpu().tolist(), keys)

    def main(self, evaluate: Callable[[Dict[Any, Any]], float], test_limit: int = 100,
             max_generations: int = 100000) -> Optional[Result]:
        import torch
        import torch.distributed as dist

        from .dist import broadcast_results
        from .engine import hex_to_digests

        rank = dist.get_rank(self.group)
        dev = self.device if self.device is not None else torch.device("cpu")
        while self.test_count <= test_limit and self.generation < max_generations:
            todo = self.run_generation_techniques()
            n = len(todo)
            keys = torch.from_numpy(hex_to_digests([dr.key for dr in todo]).view(np.int32).copy())
            y = torch.tensor([evaluate(dr.configuration) for dr in todo], dtype=torch.float64) \
                if rank == self.src else None
            y, dig = broadcast_results(y, keys if rank == self.src else None, n, dev, self.src, self.group)
            if dig.shape[0] != n or not torch.equal(dig.cpu(), keys):
                raise RuntimeError(f"rank {rank}: requested configurations diverged from rank {self.src}")
            for dr, t in zip(todo, y.cpu().tolist()):
                self.report(dr, t)
            self.process_new_results()
            self.generation += 1
            if not todo and not self.pending_result_callbacks and self.test_count and self._idle_generations():
                break
        return self.best_result
