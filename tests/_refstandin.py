"""Test infrastructure: a stand-in for the parts of the reference OpenTuner
that the reference-side binding (uptune_amd/refbinding.py) touches.  The
reference itself may not be imported or run here, so this
module restates its INTERFACE -- the names, call order and row types the
binding meets -- from the cited lines, in the simplest form:

  technique module   SearchPlugin.set_driver (plugin.py:37-39),
                     SearchTechnique.set_driver / desired_result (technique.py:70-111),
                     register (technique.py:287-288)
  SearchDriver       DriverBase.results_query / requests_query (driverbase.py:24-47),
                     get_configuration (driver.py:253-258), has_results (:157-158),
                     register_result_callback / result_callbacks (:130-155),
                     run_generation_techniques (:160-207), process_new_results (:209-225),
                     add_plugin (:102-107), main (:260-281)
  ORM rows           Configuration (.id .hash .data), DesiredResult, Result
                     (resultsdb/models.py:120-263)

Queries are lazy iterables over the tables, not lists (as SQLAlchemy
queries are), so the binding's generic (non-list) path is the one exercised.
Configuration identity uses the oracle's hashlib restatement of hash_config.
"""
import copy

from _spaces import oracle_space
from oracle import hashing as oh


# ---------------------------------------------------------------- ORM rows
class Configuration:
    def __init__(self, id, hash, data):
        self.id, self.hash, self.data = id, hash, data


class DesiredResult:
    def __init__(self, configuration=None, requestor=None, generation=None, request_date=None, tuning_run=None):
        self.id = None
        self.configuration = configuration
        self.configuration_id = configuration.id if configuration is not None else None
        self.requestor, self.generation, self.request_date, self.tuning_run = (requestor, generation,
                                                                              request_date, tuning_run)
        self.result = None
        self.state = "UNKNOWN"
        self.limit = None


class Result:
    def __init__(self, configuration=None, time=None, tuning_run=None):
        self.id = None
        self.configuration, self.time, self.tuning_run = configuration, time, tuning_run
        self.was_new_best = None
        self.state = "OK"


# ---------------------------------------------------------------- technique module
the_registry = []


def register(t):
    the_registry.append(t)


class SearchPlugin:
    def set_driver(self, driver):
        self.driver = driver


class SearchTechniqueBase:
    def __init__(self, name=None):
        super().__init__()
        self.name = name if name else self.__class__.__name__

    def is_ready(self):
        return True

    def handle_requested_result(self, result):
        pass


class SearchTechnique(SearchPlugin, SearchTechniqueBase):
    def __init__(self, *pargs, **kwargs):
        super().__init__(*pargs, **kwargs)
        self.driver = None
        self.manipulator = None
        self.objective = None
        self.request_count = 0

    def set_driver(self, driver):
        super().set_driver(driver)
        self.manipulator = driver.manipulator
        self.objective = driver.objective
        driver.add_plugin(self)

    def desired_result(self):
        cfg = self.desired_configuration()
        if cfg is None:
            return None
        if cfg is False:
            return False
        config = cfg if type(cfg) is Configuration else self.driver.get_configuration(cfg)
        desired = DesiredResult(configuration=config, requestor=self.name, generation=self.driver.generation,
                                request_date=None, tuning_run=self.driver.tuning_run)
        if hasattr(self, "limit"):
            desired.limit = self.limit
        self.driver.register_result_callback(desired, self.handle_requested_result)
        self.request_count += 1
        return desired

    def desired_configuration(self):
        return dict()


# ---------------------------------------------------------------- driver
class _Query:
    """lazy iterable over a table snapshot (SQLAlchemy-query-like)"""

    def __init__(self, rows):
        self._rows = rows

    def __iter__(self):
        return iter(list(self._rows))

    def all(self):
        return list(self._rows)

    def count(self):
        return len(self._rows)


class Objective:
    def set_driver(self, driver):
        self.driver = driver

    def lt(self, a, b):
        return a.time < b.time


class Manipulator:
    """reference-like manipulator: the mirror's params + hashlib hash_config"""

    def __init__(self, mirror):
        self.params = mirror.params
        self._space = oracle_space(mirror)

    def hash_config(self, cfg):
        return oh.hash_config(self._space, [cfg[p.name] for p in self.params])

    def normalize(self, cfg):
        pass


class SearchDriver:
    def __init__(self, manipulator, root_technique, parallelism=4, bail_threshold=500):
        self.manipulator = manipulator
        self.objective = Objective()
        self.parallelism = parallelism
        self.bail_threshold = bail_threshold
        self.tuning_run = "run-0"
        self.generation = 0
        self.test_count = 0
        self.best_result = None
        self.plugins = []
        self.pending_result_callbacks = []
        self._configs, self._drs, self._results = [], [], []
        self.root_technique = copy.deepcopy(root_technique)
        self.objective.set_driver(self)
        self.root_technique.set_driver(self)

    def add_plugin(self, p):
        if p in self.plugins:
            return
        self.plugins.append(p)
        p.set_driver(self)

    # DriverBase
    def results_query(self, config=None):
        return _Query([r for r in self._results if config is None or r.configuration is config])

    def requests_query(self):
        return _Query(self._drs)

    def get_configuration(self, cfg):
        self.manipulator.normalize(cfg)
        hashv = self.manipulator.hash_config(cfg)
        for c in self._configs:
            if c.hash == hashv:
                return c
        c = Configuration(len(self._configs), hashv, cfg)
        self._configs.append(c)
        return c

    def has_results(self, config):
        return self.results_query(config=config).count() > 0

    def register_result_callback(self, desired_result, callback):
        if desired_result.result is not None:
            callback(desired_result.result)
        else:
            self.pending_result_callbacks.append((desired_result, callback))

    def result_callbacks(self):
        pending, self.pending_result_callbacks = self.pending_result_callbacks, []
        for dr, cb in pending:
            if dr.result is not None:
                cb(dr.result)
                continue
            if self.generation - dr.generation > 0:
                rs = self.results_query(config=dr.configuration).all()
                if rs:
                    dr.result = rs[0]
                    cb(dr.result)
                    continue
            self.pending_result_callbacks.append((dr, cb))

    def run_generation_techniques(self):
        n = 0
        for _ in range(self.parallelism):
            dr = self.root_technique.desired_result()
            if dr is None or dr is False:
                break
            dr.id = len(self._drs)
            dups = [d for d in self._drs if d.configuration is dr.configuration]
            self._drs.append(dr)
            if dups:
                def cb(result, dr=dr):
                    dr.result = result
                    dr.state = "COMPLETE"
                self.register_result_callback(dups[0], cb)
            else:
                dr.state = "REQUESTED"
            self.test_count += 1
            n += 1
        return n

    def process_new_results(self):
        for r in [r for r in self._results if r.was_new_best is None]:
            if self.best_result is None or self.objective.lt(r, self.best_result):
                self.best_result = r
                r.was_new_best = True
            else:
                r.was_new_best = False
        self.result_callbacks()

    def main(self, evaluate, test_limit):
        no_tests = 0
        while self.test_count <= test_limit:
            if self.run_generation_techniques() > 0:
                no_tests = 0
            elif no_tests <= self.bail_threshold:
                no_tests += 1
            else:
                break
            for dr in [d for d in self._drs if d.state == "REQUESTED"]:
                r = Result(configuration=dr.configuration, time=evaluate(dr.configuration.data),
                           tuning_run=self.tuning_run)
                r.id = len(self._results)
                self._results.append(r)
                dr.result, dr.state = r, "COMPLETE"
            self.process_new_results()
            self.generation += 1
        return self.best_result
