"""In-memory search driver with the reference SearchDriver's surface and semantics.

The GPU techniques talk to their driver only through what the reference's
SearchDriver (opentuner/search/driver.py) and DriverBase
(opentuner/driverbase.py:5-48) expose, so the same technique code runs under
this driver and under the reference's own (refbinding.py):

  manipulator, objective, generation, tuning_run, best_result     driver.py:48-100
  get_configuration(cfg) -> Configuration (.hash, .data)           driver.py:253-258, models.py:120-135
  has_results(config)                                              driver.py:157-158
  results_query(config=None) / requests_query()                    driverbase.py:24-47
  register_result_callback / result_callbacks                      driver.py:130-155
  run_generation_techniques (duplicate requests)                   driver.py:160-207
  process_new_results (was_new_best, best_result)                  driver.py:209-225
  main (convergence by test_limit, bail_threshold)                 driver.py:113-128, 260-281
  external_main_generation (TuningRunManager slave mode)           driver.py:287-292

The SQL results database is replaced by lists: Configuration rows interned by
hash, DesiredResult and Result rows in creation order (their ids).  A
configuration's identity is its hash_config digest, computed on the device by
the technique layer's kernel (GPU path) or by a host callable `hash_fn`
(CPU-only plumbing tests supply the hashlib restatement from oracle/).

TuningRunManager mirrors opentuner/api.py:6-104 (get_next_desired_result,
get_desired_results, report_result, sync) over this driver: one
get_desired_results() call = one generation = one GPU scoring round's
selections (feature f-3).  DistributedSearchDriver / DistributedTuningRunManager
run the same loop SPMD over torch.distributed (one process per GPU).
"""
from __future__ import annotations

import collections
import logging
from typing import Any, Callable, Dict, List, Optional

import numpy as np

log = logging.getLogger(__name__)


class Configuration:
    """resultsdb/models.py:120-135: (hash, data) row, interned per hash"""
    __slots__ = ("id", "hash", "data")

    def __init__(self, id: int, hash: str, data: Dict[Any, Any]):
        self.id, self.hash, self.data = id, hash, data

    def __repr__(self):
        return f"Configuration(id={self.id}, hash={self.hash[:12]}...)"


class Result:
    """resultsdb/models.py Result: the measured objective of a configuration"""
    __slots__ = ("id", "configuration", "time", "was_new_best", "requestor", "state", "tuning_run")

    def __init__(self, configuration: Optional[Configuration] = None, time: float = float("inf"),
                 requestor: str = "", state: str = "OK", id: int = -1, tuning_run=None):
        self.id = id
        self.configuration = configuration
        self.time = float(time)
        self.was_new_best = None
        self.requestor = requestor
        self.state = state
        self.tuning_run = tuning_run


class DesiredResult:
    """resultsdb/models.py DesiredResult: one request for an evaluation"""
    __slots__ = ("id", "configuration", "requestor", "generation", "tuning_run", "result", "state", "limit",
                 "request_date")

    def __init__(self, configuration: Configuration, requestor: str = "", generation: int = 0, tuning_run=None,
                 id: int = -1):
        self.id = id
        self.configuration = configuration
        self.requestor = requestor
        self.generation = generation
        self.tuning_run = tuning_run
        self.result: Optional[Result] = None
        self.state = "UNKNOWN"
        self.limit = None
        self.request_date = None

    @property
    def key(self) -> str:
        return self.configuration.hash


class MinimizeTime:
    """objective.py:161-183: compare results on .time"""

    def set_driver(self, driver):
        self.driver = driver

    def lt(self, a: Result, b: Result) -> bool:
        return a.time < b.time

    def lte(self, a: Result, b: Result) -> bool:
        return a.time <= b.time

    def relative(self, a: Result, b: Result) -> float:
        return a.time / b.time if b.time else float("inf")

    def limit_from_config(self, config):
        return None


class SearchDriver:
    def __init__(self, manipulator, root_technique, objective=None, parallelism: int = 4,
                 hash_fn: Optional[Callable[[Dict[Any, Any]], str]] = None, bail_threshold: int = 500,
                 pipelining: int = 0, tuning_run=None, no_dups: bool = False, duplicate_log_max: int = 4096):
        import copy
        self.manipulator = manipulator
        self.objective = objective or MinimizeTime()
        self.parallelism = parallelism
        self.bail_threshold = bail_threshold
        self.pipelining = pipelining
        self.tuning_run = tuning_run
        self._hash_fn = hash_fn
        # technique instances are deep-copied into every driver (driver.py:75)
        self.root_technique = copy.deepcopy(root_technique)
        self.generation = 0
        self.test_count = 0
        self.best_result: Optional[Result] = None
        self.new_results: List[Result] = []
        self.pending_result_callbacks: List = []
        self._configs: Dict[str, Configuration] = {}       # Configuration table, by hash
        self._requests: List[DesiredResult] = []           # DesiredResult table
        self._first_request: Dict[str, DesiredResult] = {}  # hash -> earliest request
        self._results: List[Result] = []                   # Result table
        self.results: Dict[str, Result] = {}               # hash -> first result (convenience view)
        self._unprocessed: List[Result] = []
        self._todo: List[DesiredResult] = []               # REQUESTED, not yet measured
        # (test_count, requestor, first requestor, OLD | PENDING) per duplicate
        # request: the reference's log line (driver.py:186-191) as data, the
        # latest duplicate_log_max of them (duplicate_count counts them all);
        # no_dups silences the warning as the reference's --no-dups does (:185)
        self.no_dups = no_dups
        self.duplicate_log = collections.deque(maxlen=duplicate_log_max)
        self.duplicate_count = 0
        if hasattr(self.objective, "set_driver"):
            self.objective.set_driver(self)
        self.root_technique.set_driver(self)

    # -- identity / database ----------------------------------------------
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

    def _intern(self, cfg, hashv: str) -> Configuration:
        c = self._configs.get(hashv)
        if c is None:
            c = Configuration(len(self._configs), hashv, cfg)
            self._configs[hashv] = c
        return c

    def get_configuration(self, cfg) -> Configuration:
        """driver.py:253-258: hash_config, then Configuration.get (existing row or a new one)"""
        return self._intern(cfg, self.config_key(cfg))

    def configuration_from_digest(self, cfg, hashv: str) -> Configuration:
        """get_configuration for a config whose hash_config digest the device
        already computed (the GPU techniques hand their selections over this
        way, so a request costs no second hash).  A driver built with a custom
        hash_fn keys every configuration by it, so the digest is not used then
        (one Configuration row per configuration, whoever requests it)."""
        if self._hash_fn is not None:
            return self.get_configuration(cfg)
        return self._intern(cfg, hashv)

    def has_results(self, config) -> bool:
        return config.hash in self.results

    def results_query(self, config=None) -> List[Result]:
        """driverbase.py:24-44 (no generation / objective ordering: arrival order)"""
        if config is None:
            return list(self._results)
        return [r for r in self._results if r.configuration.hash == config.hash]

    def requests_query(self) -> List[DesiredResult]:
        """driverbase.py:46-47"""
        return self._requests

    def seen_hashes(self) -> List[str]:
        """hash of every requested configuration, in request order (first request only)"""
        return list(self._first_request)

    # -- technique-facing --------------------------------------------------
    def register_result_callback(self, dr: DesiredResult, callback) -> None:
        if dr.result is not None:
            callback(dr.result)
        else:
            self.pending_result_callbacks.append((dr, callback))

    def result_callbacks(self) -> None:
        """driver.py:136-155"""
        pending, self.pending_result_callbacks = self.pending_result_callbacks, []
        for dr, cb in pending:
            if dr.result is None and self.generation - dr.generation > self.pipelining:
                found = self.results.get(dr.key)
                if found is not None:
                    dr.result = found
            if dr.result is not None:
                cb(dr.result)
            else:
                self.pending_result_callbacks.append((dr, cb))

    def best_configuration(self):
        return None if self.best_result is None else self.best_result.configuration.data

    # -- bootstrap ---------------------------------------------------------
    def record_seed(self, cfgs, times, keys=None) -> None:
        """already-evaluated configurations (an initial design, or results of a
        previous run) become results of the current generation"""
        keys = keys if keys is not None else self.config_keys(cfgs)
        for cfg, t, key in zip(cfgs, times, keys):
            if key in self._first_request:
                continue
            dr = self._add_request(DesiredResult(self._intern(cfg, key), "seed", self.generation, self.tuning_run))
            self.report(dr, t)
        self.process_new_results()

    def seed_results(self, cfgs, evaluate, keys=None) -> None:
        """evaluate an initial design and record it (keys: the configurations'
        hash_config digests when the caller already has them)"""
        self.record_seed(cfgs, [evaluate(c) for c in cfgs], keys)

    # -- generation loop ---------------------------------------------------
    def _add_request(self, dr: DesiredResult) -> DesiredResult:
        dr.id = len(self._requests)
        self._requests.append(dr)
        self._first_request.setdefault(dr.key, dr)
        return dr

    def run_generation_techniques(self) -> int:
        """driver.py:160-207: ask the root technique up to `parallelism` times.
        A configuration requested before is not measured again: its request
        receives the earlier request's result through a callback.  Returns the
        number of requests made (duplicates included); the new ones wait in
        pending_desired_results()."""
        n = 0
        for _ in range(self.parallelism):
            dr = self.root_technique.desired_result()
            if dr is None or dr is False:
                break
            first = self._first_request.get(dr.key)
            self._add_request(dr)
            if first is not None:
                # driver.py:186-191: the earliest request of the configuration,
                # OLD once it has a result, PENDING before
                cls = "OLD" if first.result is not None else "PENDING"
                self.duplicate_log.append((self.test_count, dr.requestor, first.requestor, cls))
                self.duplicate_count += 1
                if not self.no_dups:
                    log.warning("duplicate configuration request #%d %s/%s %s", self.test_count, dr.requestor,
                                first.requestor, cls)

                def cb(result, dr=dr):
                    dr.result = result
                    dr.state = "COMPLETE"
                self.register_result_callback(first, cb)
            else:
                dr.state = "REQUESTED"
                self._todo.append(dr)
            self.test_count += 1
            n += 1
        return n

    def pending_desired_results(self) -> List[DesiredResult]:
        """REQUESTED and not yet measured (measurement driver's query)"""
        return [dr for dr in self._todo if dr.state == "REQUESTED"]

    def report(self, dr: DesiredResult, time: float, requestor: Optional[str] = None) -> Result:
        """measurement_driver.report_result: the Result row of a request"""
        r = Result(dr.configuration, time, requestor or dr.requestor, id=len(self._results),
                   tuning_run=self.tuning_run)
        self._results.append(r)
        dr.result = r
        dr.state = "COMPLETE"
        self.results.setdefault(dr.key, r)
        self._unprocessed.append(r)
        if dr in self._todo:
            self._todo.remove(dr)
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

    def convergence_criteria(self, test_limit: int) -> bool:
        return self.test_count > test_limit

    def main(self, evaluate: Callable[[Dict[Any, Any]], float], test_limit: int = 100,
             max_generations: int = 100000) -> Optional[Result]:
        """SearchDriver.main (driver.py:260-281) with a synchronous evaluator:
        stop after `test_limit` tests, or after more than `bail_threshold`
        consecutive generations without a single request."""
        no_tests_generations = 0
        while not self.convergence_criteria(test_limit) and self.generation < max_generations:
            if self.run_generation_techniques() > 0:
                no_tests_generations = 0
            elif no_tests_generations <= self.bail_threshold:
                no_tests_generations += 1
            else:
                break
            self.run_generation_results(evaluate)
            self.generation += 1
        return self.best_result

    def run_generation_results(self, evaluate) -> None:
        for dr in self.pending_desired_results():
            self.report(dr, evaluate(dr.configuration.data))
        self.process_new_results()

    def external_main_generation(self) -> None:
        """driver.py:287-292 (TuningRunManager slave mode)"""
        self.process_new_results()
        self.run_generation_techniques()
        self.generation += 1


class TuningRunManager:
    """opentuner/api.py:6-104 over the in-memory driver: the program under
    tuning pulls requests and reports results; the search runs one generation
    whenever no request is pending.  With GPU techniques and parallelism = the
    technique batch, one get_desired_results() is one scoring round's
    selections (f-3: batch dispatch of k proposals per round)."""

    driver_cls = SearchDriver

    def __init__(self, manipulator, root_technique, parallelism: int = 8, objective=None, hash_fn=None, **kw):
        self.search_driver = self.driver_cls(manipulator, root_technique, objective=objective,
                                             parallelism=parallelism, hash_fn=hash_fn, **kw)

    def get_next_desired_result(self) -> Optional[DesiredResult]:
        drs = self.search_driver.pending_desired_results()
        if not drs:
            self.search_driver.external_main_generation()
            drs = self.search_driver.pending_desired_results()
            if not drs:
                return None
        return drs[0]

    def get_desired_results(self) -> List[DesiredResult]:
        drs = self.search_driver.pending_desired_results()
        if not drs:
            self.search_driver.external_main_generation()
            drs = self.search_driver.pending_desired_results()
        for dr in drs:
            dr.state = "RUNNING"                # measurement_driver.claim_desired_result
        return drs

    def report_result(self, desired_result: DesiredResult, result: Result, result_input=None) -> Result:
        if desired_result in self.search_driver._todo:
            self.search_driver._todo.remove(desired_result)
        r = self.search_driver.report(desired_result, result.time)
        return r

    def sync(self, global_results) -> None:
        """api.py:87-104: results measured by other search instances (objects with
        .data, .technique, .result, e.g. GlobalResult rows) become requests +
        results of this run"""
        drv = self.search_driver
        for gr in global_results:
            config = drv.get_configuration(gr.data)
            dr = drv._add_request(DesiredResult(config, gr.technique, drv.generation, drv.tuning_run))
            self.report_result(dr, Result(time=gr.result))

    def get_best_configuration(self):
        return self.search_driver.best_configuration()

    def get_best_result(self) -> Optional[Result]:
        return self.search_driver.best_result

    def finish(self) -> None:
        self.search_driver.process_new_results()


# ---------------------------------------------------------------------------
# SPMD over torch.distributed
# ---------------------------------------------------------------------------
def agree(ok: bool, group=None, device=None) -> bool:
    """True iff every rank of the group passes ok=True (dist.agree: one
    all-reduce MIN over this rank's RCCL communicator, or gloo on the CPU).
    Every rank takes the same branch afterwards, so a failure on one rank
    never leaves the others waiting inside a later collective."""
    from .dist import agree as _agree
    return _agree(ok, group, device)


class DistributedSearchDriver(SearchDriver):
    """SPMD search loop over a torch.distributed group (one process per GPU).

    Every rank runs the same technique tree with the same seeds; the GPU
    techniques shard each round's candidate pool by global index and
    all-gather their local top-k (technique.GpuBatchTechnique), so every rank
    requests the same configurations.  Rank `src` evaluates them and the
    results -- objective values and hash digests, the per-round history delta
    -- are broadcast to every rank (dist.broadcast_results; the reference's
    api.sync result injection, api.py:547-553, and ParallelTuning's batch
    dispatch, api.py:428-482).  The digests double as a consistency check,
    agreed on collectively: if any rank's requests diverge, EVERY rank raises
    (none is left waiting in the next collective).
    """

    def __init__(self, manipulator, root_technique, objective=None, parallelism: int = 4, hash_fn=None,
                 group=None, src: int = 0, device=None, **kw):
        self.group, self.src = group, src
        self.device = device
        super().__init__(manipulator, root_technique, objective, parallelism, hash_fn, **kw)

    def _exchange(self, keys_hex: List[str], values: Optional[List[float]]):
        """broadcast (values, digests) from src; every rank checks its own keys
        against src's and all ranks agree on the outcome"""
        import torch
        import torch.distributed as dist

        from .dist import broadcast_results
        from .engine import hex_to_digests
        n = len(keys_hex)
        keys = torch.from_numpy(hex_to_digests(keys_hex).view(np.int32).copy())
        is_src = dist.get_rank(self.group) == self.src
        y = torch.tensor(values, dtype=torch.float64) if is_src else None
        dev = self.device if self.device is not None else torch.device("cpu")
        y, dig = broadcast_results(y, keys if is_src else None, n, dev, self.src, self.group)
        same = dig.shape[0] == n and torch.equal(dig.cpu(), keys)
        if not agree(same, self.group, self.device):
            raise RuntimeError(f"rank {dist.get_rank(self.group)}: requested configurations diverged from rank "
                               f"{self.src} (this rank {'agrees' if same else 'differs'})")
        return y.cpu().tolist()

    def seed_results(self, cfgs, evaluate, keys=None) -> None:
        """rank `src` evaluates the initial design; values + digests are broadcast"""
        import torch.distributed as dist
        keys = keys if keys is not None else self.config_keys(cfgs)
        src = dist.get_rank(self.group) == self.src
        y = self._exchange(keys, [evaluate(c) for c in cfgs] if src else None)
        self.record_seed(cfgs, y, keys)

    def run_generation_results(self, evaluate) -> None:
        import torch.distributed as dist
        todo = self.pending_desired_results()
        src = dist.get_rank(self.group) == self.src
        y = self._exchange([dr.key for dr in todo],
                           [evaluate(dr.configuration.data) for dr in todo] if src else None)
        for dr, t in zip(todo, y):
            self.report(dr, t)
        self.process_new_results()


class DistributedTuningRunManager(TuningRunManager):
    """TuningRunManager SPMD over torch.distributed: every rank calls
    get_desired_results() / get_next_desired_result() in step and gets the same
    requests; only rank `src` measures and calls report_result().  At the start
    of the next get_*() call the measured values of every handed-out request
    travel from src to all ranks in one broadcast_results (the api.sync path of
    ParallelTuning, api.py:547-553, over RCCL); requests src has not measured
    yet stay pending everywhere.  sync(global_results) is called on every rank
    with the same global results (read from the shared GlobalResult table)."""

    driver_cls = DistributedSearchDriver

    def __init__(self, *a, group=None, src: int = 0, device=None, **kw):
        super().__init__(*a, group=group, src=src, device=device, **kw)
        self._reported: Dict[int, float] = {}     # request id -> measured time (src)

    def report_result(self, desired_result, result, result_input=None):
        self._reported[desired_result.id] = float(result.time)
        return None

    def _exchange_reported(self) -> None:
        import torch.distributed as dist
        drv = self.search_driver
        out = [dr for dr in drv._todo if dr.state == "RUNNING"]        # identical list on every rank
        is_src = dist.get_rank(drv.group) == drv.src
        vals = [self._reported.pop(dr.id, float("nan")) for dr in out] if is_src else None
        y = drv._exchange([dr.key for dr in out], vals)
        for dr, t in zip(out, y):
            if t == t:                                                  # NaN: not measured yet
                drv.report(dr, t)

    def get_next_desired_result(self):
        self._exchange_reported()
        return super().get_next_desired_result()

    def get_desired_results(self):
        self._exchange_reported()
        return super().get_desired_results()
