"""Search-technique plugin interface, AUC bandit and the GPU batch techniques.

Mirrors the reference's plugin API so the GPU path drops in where the
per-candidate CPU techniques sit:

  SearchTechnique.desired_result / desired_configuration   opentuner/search/technique.py:70-121
  register / all_techniques / get_enabled                   technique.py:287, 331-355
  MetaSearchTechnique.desired_result                        opentuner/search/metatechniques.py:14-57
  BanditQueue / AUCBanditQueue                              opentuner/search/bandittechniques.py:20-146
  AUCBanditMetaTechnique                                    bandittechniques.py:150-165

`desired_configuration()` returns a config dict, None (nothing to propose ->
the bandit credits 0 and moves on) or False (waiting for results) exactly as
in the reference.  The GPU techniques (GpuDifferentialEvolution, GpuPSO,
GpuGA, GpuGGA) score a whole candidate pool per round on the device
(proposal -> hash_config -> dedup -> GP-EI -> top-k) and hand the top-k out one
per call.  Device contexts are created lazily in set_driver and are never
deep-copied (technique instances are deepcopied per driver, driver.py:75).
Device errors never propagate into the driver (the reference's controller
retries forever on exceptions, api.py:433-435): the technique logs and
returns None so the bandit moves on.
"""
from __future__ import annotations

import copy
import logging
import math
import random
from collections import deque
from typing import Any, Dict, List, Optional

import numpy as np

log = logging.getLogger(__name__)


# ---------------------------------------------------------------------------
# plugin interface + registry
# ---------------------------------------------------------------------------
class SearchTechniqueBase:
    def __init__(self, name: Optional[str] = None):
        self.name = name or self.default_name()

    def is_ready(self) -> bool:
        return True

    def default_name(self) -> str:
        return self.__class__.__name__

    def handle_requested_result(self, result) -> None:
        pass

    def set_driver(self, driver) -> None:
        raise NotImplementedError

    def desired_result(self):
        raise NotImplementedError


class SearchTechnique(SearchTechniqueBase):
    """technique.py:70-175: subclasses implement desired_configuration()."""

    def __init__(self, *pargs, **kwargs):
        super().__init__(*pargs, **kwargs)
        self.driver = None
        self.manipulator = None
        self.objective = None
        self.request_count = 0

    def set_driver(self, driver):
        self.driver = driver
        self.manipulator = driver.manipulator
        self.objective = driver.objective

    def desired_result(self):
        """technique.py:88-111: wrap desired_configuration() into a DesiredResult
        (None = nothing to propose, False = waiting for results)"""
        from .driver import Configuration, DesiredResult
        cfg = self.desired_configuration()
        if cfg is None:
            return None
        if cfg is False:
            return False
        config = cfg if isinstance(cfg, Configuration) else self.driver.get_configuration(cfg)
        desired = DesiredResult(configuration=config, requestor=self.name, generation=self.driver.generation,
                                tuning_run=getattr(self.driver, "tuning_run", None))
        if hasattr(self, "limit"):
            desired.limit = self.limit
        self.driver.register_result_callback(desired, self.handle_requested_result)
        self.request_count += 1
        return desired

    def desired_configuration(self):
        raise NotImplementedError


the_registry: List[SearchTechniqueBase] = []


def register(t: SearchTechniqueBase) -> None:
    the_registry.append(t)


def all_techniques() -> List[SearchTechniqueBase]:
    return the_registry


def get_enabled(names: List[str]) -> List[SearchTechniqueBase]:
    known = {t.name for t in the_registry}
    for n in names:
        if n not in known:
            raise Exception("Unknown technique: --technique={}".format(n))
    return [t for t in the_registry if t.name in names]


# ---------------------------------------------------------------------------
# meta techniques / bandit (stay on the CPU: O(#techniques) per request)
# ---------------------------------------------------------------------------
class MetaSearchTechnique(SearchTechniqueBase):
    """metatechniques.py:14-76"""

    def __init__(self, techniques, log_freq=500, *pargs, **kwargs):
        super().__init__(*pargs, **kwargs)
        self.techniques = techniques
        self.request_count = 0
        self.log_freq = log_freq
        self.unique_names()

    def unique_names(self):
        names = set()
        for t in self.techniques:
            while t.name in names:
                t.name += "~"
            names.add(t.name)

    def set_driver(self, driver):
        for t in self.techniques:
            t.set_driver(driver)
        self.driver = driver

    def desired_result(self):
        for technique in self.select_technique_order():
            dr = technique.desired_result()
            if dr is not None:
                if dr is False:
                    continue  # waiting for results
                self.driver.register_result_callback(
                    dr, lambda result, technique=technique: self.on_technique_result(technique, result))
                self.request_count += 1
                return dr
            self.on_technique_no_desired_result(technique)
        return None

    def on_technique_no_desired_result(self, technique):
        pass

    def on_technique_result(self, technique, result):
        pass

    def select_technique_order(self):
        return list(self.techniques)


class BanditQueue:
    """bandittechniques.py:20-79"""

    def __init__(self, keys, C=0.05, window=500, **kwargs):
        self.C = C
        self.history = deque()
        self.keys = keys
        self.use_counts = dict((k, 0) for k in keys)
        self.window = window
        self.request_count = 0

    def exploitation_term(self, key):
        return 0.0

    def exploration_term(self, key):
        if self.use_counts[key] > 0:
            return math.sqrt((2.0 * math.log(len(self.history), 2.0)) / self.use_counts[key])
        return float("inf")

    def bandit_score(self, key):
        return self.exploitation_term(key) + self.C * self.exploration_term(key)

    def ordered_keys(self, rng=random):
        keys = list(self.keys)
        rng.shuffle(keys)  # break ties randomly
        keys.sort(key=self.bandit_score)
        self.request_count += 1
        return reversed(keys)

    def on_result(self, key, value):
        self.history.append((key, value))
        self.on_push_history(key, value)
        if len(self.history) > self.window:
            self.on_pop_history(*self.history.popleft())

    def on_push_history(self, key, value):
        self.use_counts[key] += 1

    def on_pop_history(self, key, value):
        self.use_counts[key] -= 1


class AUCBanditQueue(BanditQueue):
    """Area-under-curve credit assignment (Fialho et al.): a restatement of
    bandittechniques.py:82-146 with the same scores and tie-break sequence.
    The exploitation term is the reference's O(1) incremental form: with the
    uses of `key` in the window numbered 1..pos, AUC = 2 * (sum of the
    numbers of the credited uses) / (pos * (pos + 1)).  auc_sum holds that
    sum; popping the oldest use renumbers the rest down by one, i.e. subtracts
    the number of credited uses left (auc_decay)."""

    def __init__(self, *args, **kwargs):
        super().__init__(*args, **kwargs)
        self.auc_sum = dict((t, 0) for t in self.keys)
        self.auc_decay = dict((t, 0) for t in self.keys)

    def exploitation_term(self, key):
        pos = self.use_counts[key]
        if pos:
            return self.auc_sum[key] * 2.0 / (pos * (pos + 1.0))
        return 0.0

    def on_push_history(self, key, value):
        super().on_push_history(key, value)
        if value:
            self.auc_sum[key] += self.use_counts[key]
            self.auc_decay[key] += 1

    def on_pop_history(self, key, value):
        super().on_pop_history(key, value)
        self.auc_sum[key] -= self.auc_decay[key]
        if value:
            self.auc_decay[key] -= 1


class AUCBanditMetaTechnique(MetaSearchTechnique):
    """bandittechniques.py:150-165"""

    def __init__(self, techniques, bandit_kwargs=None, seed: Optional[int] = None, **kwargs):
        super().__init__(techniques, **kwargs)
        self.bandit = AUCBanditQueue([t.name for t in techniques], **(bandit_kwargs or {}))
        self.name_to_technique = dict((t.name, t) for t in self.techniques)
        self._rng = random.Random(seed) if seed is not None else None  # None: the global `random`

    def select_technique_order(self):
        return [self.name_to_technique[k] for k in self.bandit.ordered_keys(self._rng or random)]

    def on_technique_result(self, technique, result):
        self.bandit.on_result(technique.name, result.was_new_best)

    def on_technique_no_desired_result(self, technique):
        self.bandit.on_result(technique.name, 0)


# ---------------------------------------------------------------------------
# GPU batch techniques
# ---------------------------------------------------------------------------
class SharedModel:
    """Device state the GPU techniques of one bandit share: ONE context, hence
    one history digest set and one GP fit per change of the training set (the
    reference composes DE, PSO and GA under one bandit, bandittechniques.py:311-320,
    and north_star C5 asks for a shared surrogate).  Each technique keeps its
    own population in a slot of that context (ut_population_select).

    A technique built without `shared=` makes a private SharedModel, so a
    stand-alone technique and a bandit member run the same code.  Everything
    here reads the driver only through the reference SearchDriver surface:
    requests_query() (every requested configuration's hash -> the dedup set),
    results_query() (Configuration.data + time -> the training set)."""

    def __init__(self, device: int = 0, seed: int = 0, lengthscale: float = 0.3, min_train: int = 4,
                 precision: int = 64, sigma_f2: float = 1.0, sigma_n2: float = 1e-6, jitter: float = 1e-8,
                 engine_factory=None, y_transform: Optional[str] = None):
        self.device, self.seed, self.lengthscale, self.min_train = device, seed, lengthscale, min_train
        self.precision = precision
        # y_transform: what the GP is fitted on.  None = the objective as
        # measured; "rank" = its normal scores, Phi^-1((rank + 1/2) / n) (order
        # preserving, so the incumbent stays the minimum): an objective spanning
        # many decades (Rosenbrock over [-1000, 1000]^2: 0 .. 1e14) otherwise
        # standardises to a flat landscape where EI only explores
        if y_transform not in (None, "rank"):
            raise ValueError("y_transform: None or 'rank'")
        self.y_transform = y_transform
        # engine_factory(manipulator, device, seed) -> a BatchEngine-compatible
        # object; None = uptune_amd.engine.BatchEngine (the device path).  Tests
        # substitute a CPU stand-in to exercise the plugin plumbing without a GPU.
        self.engine_factory = engine_factory
        self.hyper = dict(sigma_f2=sigma_f2, sigma_n2=sigma_n2, jitter=jitter)
        self._reset()
        self.slots: Dict[str, int] = {}

    def _reset(self):
        self.engine = None
        self._req_seen = 0          # requests_query() rows pushed to the device set (list drivers)
        self._hist = set()          # digests pushed (any driver)
        self._res_ids: List[Any] = []
        # training rows in arrival order (features, objective): the first _n
        # rows of capacity-grown buffers, so a fit that appends a few results
        # copies only those
        self._n = 0
        self._Xa = np.zeros((0, 0))
        self._ya = np.zeros(0)
        # the same rows in the fit's order (what gp_fit receives): best y first
        # as of the last refit, the results since appended in arrival order
        self._Xf = np.zeros((0, 0))
        self._yf = np.zeros(0)
        self._nf = 0
        self._perm_npad = 0
        # features of the rounds' selections, encoded on the device beside
        # them (GpuBatchTechnique._round), by hash_config digest: a result of a
        # selected configuration needs no second encode round trip
        self._feat_cache: Dict[str, np.ndarray] = {}
        self._fit_key = None
        self._fit_unverified = False
        self.fits = 0
        # list drivers (append-only results table): the usable rows found so
        # far and how far the table has been scanned
        self._scan_n = 0
        self._scan_last = None
        self._scan_rows: List[Any] = []
        self._scan_ids: List[Any] = []

    def __deepcopy__(self, memo):
        # techniques (and so their shared model) are deep-copied per driver
        # (driver.py:75): the copy starts without a device context
        new = self.__class__.__new__(self.__class__)
        memo[id(self)] = new
        new.__dict__.update({k: copy.deepcopy(v, memo) for k, v in self.__dict__.items() if k != "engine"})
        new._reset()
        return new

    def slot(self, tech) -> int:
        return self.slots.setdefault(tech.name, len(self.slots))

    def engine_for(self, tech):
        """the shared engine with `tech`'s population slot selected"""
        if self.engine is None:
            if self.engine_factory is None:
                from .engine import BatchEngine
                self.engine = BatchEngine(tech.manipulator, device=self.device, seed=self.seed)
            else:
                self.engine = self.engine_factory(tech.manipulator, self.device, self.seed)
            self.engine.gp_set_precision(self.precision)
            self.engine.history_reset(1024)
        self.engine.population_select(self.slot(tech))
        return self.engine

    def sync_history(self, driver) -> None:
        """every configuration the driver has requested joins the device dedup
        set (driver.py:157-158,177-200: history + in-flight requests)"""
        reqs = driver.requests_query()
        if isinstance(reqs, list):             # append-only table: only the new rows
            rows, self._req_seen = reqs[self._req_seen:], len(reqs)
        else:                                  # a SQL query (reference driver): all rows, filtered
            rows = reqs
        new = []
        for dr in rows:
            h = dr.configuration.hash
            if h not in self._hist:
                self._hist.add(h)
                new.append(h)
        if new:
            self.engine.history_add(new)

    def fit(self, driver) -> bool:
        """(re)fit the GP iff the driver's results changed since the last fit;
        the new training rows are encoded on the device (ut_encode_features)
        and the fit is enqueued without a host wait (ut_gp_fit_async)"""
        def usable(r):
            return getattr(r, "state", "OK") == "OK" and r.time is not None and math.isfinite(r.time)

        res = driver.results_query()
        if isinstance(res, list):
            # an in-memory table only grows: scan the rows added since the last
            # call (a table that shrank or changed under us is rescanned)
            if len(res) < self._scan_n or (self._scan_n and res[self._scan_n - 1] is not self._scan_last):
                self._scan_n, self._scan_rows, self._scan_ids = 0, [], []
            for r in res[self._scan_n:]:
                if usable(r):
                    self._scan_ids.append(getattr(r, "id", len(self._scan_rows)))
                    self._scan_rows.append(r)
            self._scan_n = len(res)
            self._scan_last = res[-1] if res else None
            rows, ids = self._scan_rows, self._scan_ids
        else:   # a SQL query (reference driver): every row, filtered
            rows = [r for r in res if usable(r)]
            ids = [getattr(r, "id", i) for i, r in enumerate(rows)]
        if len(rows) < self.min_train:
            return False
        if self._fit_unverified and self._fit_key is not None:
            # the previous fit ran asynchronously (no host wait when it was
            # enqueued): a kernel matrix that was not positive definite would
            # leave every score NaN, so check it once, before reusing it
            self._fit_unverified = False
            if not self.engine.gp_fit_ok():
                self.hyper["jitter"] = max(10.0 * self.hyper.get("jitter", 0.0), 1e-8)
                log.warning("GP fit on %d results was not positive definite: refitting with jitter %g",
                            self._fit_key[0], self.hyper["jitter"])
                self._fit_key = None
        key = (len(rows), ids[-1])
        if key == self._fit_key:
            return True
        k = self._n
        if k == 0 or ids[:k] != self._res_ids:      # not an append: re-encode everything
            k = self._n = self._nf = 0
        new = rows[k:]
        if new:
            n = k + len(new)
            self._Xa, self._ya = _rows_room(self._Xa, self._ya, k, n, self.engine.spec.n_features)
            self._Xa[k:n] = self._features(new)
            self._ya[k:n] = [float(r.time) for r in new]
            self._n = n
            self._res_ids = list(ids)   # a copy: the scan list keeps growing
        # Row order.  The GP posterior does not depend on it, but the EI bound of
        # pruned scoring (ut_gp_topk_pruned) comes from the first rows of L^-1:
        # with the best results first it sees the neighbourhood that GA / GGA
        # children (mutations of the best configuration) live in (the C5 GGA
        # round: 262,144 survivors -> 8, 75 -> 5 ms; a GA round: 2,459 -> 8,
        # scripts/exp/gga_prune_probe.py).  The rows are re-sorted only where
        # the device refits anyway (a new padded size, gp.hip NPAD = 128, or a
        # re-encode); in between the new results are appended, so the
        # incremental fit still applies.
        n = self._n
        npad = -(-n // 128) * 128
        self._Xf, self._yf = _rows_room(self._Xf, self._yf, self._nf, n, self._Xa.shape[1])
        if self._nf == 0 or npad != self._perm_npad or self._nf > n:
            perm = np.argsort(self._ya[:n], kind="stable")
            self._Xf[:n] = self._Xa[perm]
            self._yf[:n] = self._ya[perm]
            self._perm_npad = npad
        else:
            self._Xf[self._nf:n] = self._Xa[self._nf:n]
            self._yf[self._nf:n] = self._ya[self._nf:n]
        self._nf = n
        y = self._yf[:n]
        if self.y_transform == "rank":
            from scipy.special import ndtri
            from scipy.stats import rankdata
            # average ranks: tied (repeated) measurements get one normal score,
            # whatever their row order
            r = rankdata(y, method="average") - 1.0
            y = ndtri((r + 0.5) / n)
        self.engine.gp_fit(self._Xf[:n], y, lengthscale=self.lengthscale, wait=False, **self.hyper)
        self._fit_key = key
        self._fit_unverified = True
        self.fits += 1
        return True

    def note_selections(self, hexes) -> None:
        """a round's selections are requests the driver has not made yet: they
        join the dedup set now, so no technique sharing this model selects one
        of them again while it waits in a queue (a bandit runs other techniques'
        rounds between the requests of one round's batch)"""
        new = [h for h in hexes if h not in self._hist]
        if new:
            self._hist.update(new)
            self.engine.history_add(new)

    def remember_features(self, hexes, feat) -> None:
        """features [k][F] of configurations selected this round, by digest"""
        if len(self._feat_cache) > (1 << 16):   # selections never evaluated: bounded
            self._feat_cache.clear()
        for hx, f in zip(hexes, feat):
            self._feat_cache[hx] = f

    def _features(self, results) -> np.ndarray:
        """GP features of results: the round's device encoding where the result's
        configuration is one of the selections, else encoded now"""
        out = np.empty((len(results), self.engine.spec.n_features))
        miss = []
        for i, r in enumerate(results):
            f = self._feat_cache.pop(getattr(r.configuration, "hash", None), None)
            if f is None:
                miss.append(i)
            else:
                out[i] = f
        if miss:
            out[miss] = self.engine.features_host([results[i].configuration.data for i in miss])
        return out


def _rows_room(X, y, used, n, d):
    """(X, y) with room for n rows of d features, the first `used` rows kept"""
    if X.shape[0] >= n and X.shape[1] == d:
        return X, y
    cap = max(n + n // 2, 256)
    X2, y2 = np.empty((cap, d)), np.empty(cap)
    used = min(used, n, X.shape[0])
    if used and X.shape[1] == d:
        X2[:used], y2[:used] = X[:used], y[:used]
    return X2, y2


class GpuBatchTechnique(SearchTechnique):
    """Base of the device-scored population techniques.

    One round = propose `pool` candidates with the technique's operator,
    hash_config + dedup against every configuration the driver has seen,
    score with the shared GP (EI/UCB) fitted on the driver's results, keep
    the top `batch`; desired_configuration() then returns them one per call.
    """

    # DE / GA pools shard over the ranks of a process group by GLOBAL candidate
    # index; PSO moves its (small) swarm on every rank (replicas)
    sharded = True

    def __init__(self, pool: int = 1 << 14, batch: int = 8, population: int = 1024, device: int = 0,
                 seed: int = 0, lengthscale: float = 0.3, min_train: int = 4, acq: str = "ei",
                 group=None, surrogate=None, shared: Optional[SharedModel] = None, engine_factory=None,
                 prune_rows: int = 0, precision: int = 64, y_transform: Optional[str] = None, *pargs, **kwargs):
        super().__init__(*pargs, **kwargs)
        # prune_rows > 0: score rounds with ut_gp_topk_pruned (selection-exact EI
        # bound from the first prune_rows rows of L^-1 k*; fp64 fits, EI / UCB):
        # the same selections as the dense variance at a fraction of its cost
        # when the bounds are tight (or the GP is flat: exact ties by index)
        self.prune_rows = int(prune_rows)
        # surrogate: None = the GP fitted on the driver's results (EI / UCB); or a
        # tree ensemble over the same features (sklearn regressor, XGBoost JSON,
        # forest.Forest) ranking candidates by predicted objective (minimised),
        # the multi-stage tuner's model scoring (multi_stage.py:8-22, :109-123)
        self.surrogate = surrogate
        # precision: the GP contractions of a private model (64 / 32 / 16 = f16x3);
        # a shared model (the bandit's) carries its own
        self.model = shared if shared is not None else SharedModel(device=device, seed=seed,
                                                                   lengthscale=lengthscale, min_train=min_train,
                                                                   precision=precision,
                                                                   engine_factory=engine_factory,
                                                                   y_transform=y_transform)
        # multi-GPU: with torch.distributed initialised and
        # world > 1, rank r scores candidates [base + r*pool, base + (r+1)*pool)
        # of every round and the local top-k lists are all-gathered and merged
        self.group = group
        self.pool, self.batch, self.population = int(pool), int(batch), int(population)
        self.acq_kind = acq
        self.queue: List[Any] = []      # (config dict, hash hex) of the last round's selections
        self.round = 0
        self.cand_base = 0
        self._initialised = False

    def __deepcopy__(self, memo):
        # the process group is shared, never copied; the model drops its device state
        cls = self.__class__
        new = cls.__new__(cls)
        memo[id(self)] = new
        for k, v in self.__dict__.items():
            setattr(new, k, v if k == "group" else copy.deepcopy(v, memo))
        new._initialised = False
        return new

    @property
    def engine(self):
        return self.model.engine

    def _dist(self):
        """(rank, world) of the sharded round (world 1 without torch.distributed)"""
        try:
            import torch.distributed as dist
        except Exception:  # pragma: no cover
            return 0, 1
        if not dist.is_available() or not dist.is_initialized():
            return 0, 1
        return dist.get_rank(self.group), dist.get_world_size(self.group)

    def round_base(self) -> int:
        """global index of this rank's first candidate of the current round"""
        rank, _ = self._dist()
        return self.cand_base + (rank * self.pool if self.sharded else 0)

    # -- device state ------------------------------------------------------
    def _ensure_engine(self):
        eng = self.model.engine_for(self)
        if not self._initialised:
            self.init_population()
            self._initialised = True
        return eng

    def init_population(self):
        self.engine.population_init(max(self.population, 4), round_=0)

    def propose(self, m: int):
        """-> (values [P][m] device tensor, invalid mask or None)"""
        raise NotImplementedError

    def hash_proposals(self, vals, base):
        """hash_config of this round's proposals"""
        return self.engine.hash(vals)

    def best_row(self):
        """driver.best_result's configuration as a SoA value row, or None"""
        b = self.driver.best_result
        return None if b is None else self.engine.spec.encode_configs([b.configuration.data])[:, 0]

    def _local_round(self):
        """this rank's shard: propose -> hash -> dedup -> score -> local top-k"""
        import torch
        eng = self._ensure_engine()
        self.model.sync_history(self.driver)
        # the fit first: its new training rows are encoded through the device
        # (one host round trip) while the queue is still empty.  Pruned scoring
        # needs the whole fit before its K*, so the round's stages queue behind
        # it (ut_gp_join_fit): the fit's chain of small kernels runs alone
        # instead of starving beside the hash, and no host wait sits between the
        # hash and the fit (the proposals never read the GP).  Dense fp64 rounds
        # keep the fit beside their K* (only the variance GEMM waits for it).
        have_model = self.surrogate is None and self.model.fit(self.driver)
        if have_model and self.prune_rows > 0 and self.model.precision == 64:
            eng.gp_join_fit()
        base = self.round_base()
        vals, invalid = self.propose(self.pool)
        dig = self.hash_proposals(vals, base)
        dup = eng.dedup(dig)
        if invalid is not None:
            dup = torch.maximum(dup, invalid)
        if self.surrogate is not None:
            if getattr(eng, "forest", None) is None:
                eng.forest_set(self.surrogate)
            _, score = eng.forest_predict(eng.encode(vals), dup=dup)
        elif have_model:
            if self.prune_rows > 0 and self.model.precision == 64:
                idx, top, _ = eng.gp_topk_pruned(eng.encode(vals), self.batch, acq=eng.acq(self.acq_kind), dup=dup,
                                                 cand_base=base, bound_rows=self.prune_rows)
                loc = torch.where(idx >= 0, idx - base, torch.zeros_like(idx))
                return vals, idx, top, dig[loc], vals[:, loc]
            # encoding fused into the K* operand pass (no feature matrix)
            _, _, score = eng.gp_score_values(vals, acq=eng.acq(self.acq_kind), dup=dup)
        else:  # no model yet: every non-duplicate candidate is equally good (lowest index first)
            score = torch.zeros(vals.shape[1], dtype=torch.float64, device=vals.device)
        idx, top = eng.topk(score, self.batch, dup=dup, cand_base=base)   # GLOBAL candidate indices
        loc = torch.where(idx >= 0, idx - base, torch.zeros_like(idx))
        return vals, idx, top, dig[loc], vals[:, loc]

    def _round(self):
        from .engine import digests_to_hex
        rank, world = self._dist()
        if world > 1 and self.sharded:
            # a failure on any rank must not leave the others inside the
            # all-gather: agree first, then all proceed or all give up
            from .driver import agree
            err = None
            try:
                vals, idx, top, dig, rows = self._local_round()
            except Exception as ex:   # noqa: BLE001 -- re-raised below on every rank
                err = ex
            # the vote travels on the technique's GPU whether or not the round
            # failed (a failed rank must use the same communicator as the others)
            import torch
            dev = idx.device if err is None else torch.device("cuda", self.model.device)
            if not agree(err is None, self.group, dev):
                raise RuntimeError(f"{self.name}: scoring round failed on "
                                   f"{'this rank: ' + repr(err) if err is not None else 'another rank'}")
            from .dist import allgather_selection
            idx, top, rows, dig = allgather_selection(idx, top, dig, rows, self.batch, group=self.group,
                                                      with_digests=True)
        else:
            vals, idx, top, dig, rows = self._local_round()
        import torch
        eng = self.engine
        # the selections (and, for the GP's next fit, their features) reach the
        # host in ONE copy: global indices, value rows, digests, features
        feat = eng.encode(rows) if self.surrogate is None else None
        parts = [idx.contiguous().view(torch.float64), rows.contiguous().reshape(-1),
                 dig.to(torch.int32).contiguous().view(torch.float64).reshape(-1)]
        if feat is not None:
            parts.append(feat.contiguous().reshape(-1))
        host = torch.cat(parts).cpu().numpy()
        k, ncol = idx.numel(), rows.shape[0]
        o1, o2 = k + ncol * k, k + ncol * k + 4 * k
        keep = host[:k].view(np.int64) >= 0
        idx_h = host[:k].view(np.int64)[keep]
        rows_h = host[k:o1].reshape(ncol, k)[:, keep]
        hexes = digests_to_hex(host[o1:o2].view(np.int32).reshape(k, 8)[keep])
        cfgs = eng.spec.decode_values(rows_h)
        self.queue.extend(zip(cfgs, hexes))
        self.model.note_selections(hexes)
        if feat is not None:
            # a result's features are what features_host(config) encodes: keep
            # those of selections whose config re-encodes to the same value
            # bits (always, unless a value has two encodings, e.g. an enum
            # option listed twice)
            same = (eng.spec.encode_configs(cfgs).view(np.int64) == rows_h.view(np.int64)).all(axis=0)
            ft = host[o2:].reshape(-1, k)[:, keep].T
            self.model.remember_features([h for h, s in zip(hexes, same) if s], ft[same])
        self.after_round(idx_h, hexes)
        self.round += 1
        self.cand_base += (world if self.sharded else 1) * self.pool

    def after_round(self, idx, hexes):
        pass

    def desired_configuration(self):
        try:
            if not self.queue:
                self._round()
            if not self.queue:
                return None
            cfg, hx = self.queue.pop(0)
            # the digest is already known: an in-memory driver interns it as is
            # (no second hash); the reference driver hashes the dict itself
            intern = getattr(self.driver, "configuration_from_digest", None)
            return intern(cfg, hx) if intern is not None else cfg
        except Exception as ex:  # never raise into the driver loop
            log.warning("%s: device round failed: %s", self.name, ex)
            return None


class GpuDifferentialEvolution(GpuBatchTechnique):
    """Batched DifferentialEvolution(Alt) (differentialevolution.py:29-151):
    every round proposes DE/rand/1/bin trials for the population, with the
    driver's best config in the donor pool (information sharing, :112-116);
    an evaluated trial replaces its target when better (handle_requested_result,
    :131-139)."""

    def __init__(self, cr: float = 0.2, n_cross: int = 1, information_sharing: int = 1, *pargs, **kwargs):
        super().__init__(*pargs, **kwargs)
        self.cr, self.n_cross, self.information_sharing = cr, n_cross, information_sharing
        self._pending: Dict[str, int] = {}       # trial digest -> target member
        self._pop_results: Dict[int, Any] = {}   # member -> its Result (PopulationMember.config)

    def propose(self, m):
        return self.engine.propose_de(m, round_=self.round, cand_base=self.round_base(), cr=self.cr,
                                      n_cross=self.n_cross, best=self.best_row(),
                                      information_sharing=self.information_sharing), None

    def hash_proposals(self, vals, base):
        # trials keep most of their target's values: reuse its inner digests
        return self.engine.hash_de(vals, base)

    def after_round(self, idx, hexes):
        npop = self.engine.npop
        for g, hx in zip(np.asarray(idx).tolist(), hexes):   # global index g targets member g % npop
            self._pending[hx] = g % npop

    def handle_requested_result(self, result):
        import torch
        tgt = self._pending.pop(result.configuration.hash, None)
        if tgt is None or self.engine is None:
            return
        parent = self._pop_results.get(tgt)
        if parent is None or self.objective.lt(result, parent):
            eng = self.model.engine_for(self)
            vals = torch.from_numpy(eng.spec.encode_configs([result.configuration.data])).to(eng.device)
            eng.population_replace(vals, torch.tensor([tgt], device=eng.device))
            self._pop_results[tgt] = result


class GpuPSO(GpuBatchTechnique):
    """Batched PSO (pso.py:11-77); particles move toward the driver's best."""

    sharded = False   # the swarm moves on every rank: same particles, same result

    def __init__(self, omega=0.5, phi_l=0.5, phi_g=0.5, enum_mode=0, crossover="op3_cross_OX1", *pargs, **kwargs):
        super().__init__(*pargs, **kwargs)
        self.omega, self.phi_l, self.phi_g, self.enum_mode = omega, phi_l, phi_g, enum_mode
        self.crossover = crossover   # PSO(crossover=...) for permutation params (pso.py:80-84)

    def init_population(self):
        super().init_population()
        self.engine.pso_reset()

    def propose(self, m):
        gb = self.best_row()
        if gb is None:  # no result yet: particle 0 stands in for the global best
            gb = self.engine.population_get()[:, 0]
        npop = self.engine.npop
        x, v = self.engine.propose_pso(gb, min(m, npop), round_=self.round, cand_base=0, omega=self.omega,
                                       phi_l=self.phi_l, phi_g=self.phi_g, enum_mode=self.enum_mode,
                                       crossover=self.crossover)
        self.engine.pso_commit(x, v, cand_base=0)   # HybridParticle.move mutates the particle in place
        return x, None


class GpuGA(GpuBatchTechnique):
    """Batched UniformGreedyMutation / NormalGreedyMutation / GA
    (evolutionarytechniques.py:13-158)."""

    def __init__(self, mutation_rate=0.1, crossover_rate=0.0, must_mutate_count=1, normal=False, sigma=0.1,
                 crossover_strength=0.0, op=4, crossover=None, *pargs, **kwargs):
        super().__init__(*pargs, **kwargs)
        # crossover: GA(crossover='op3_cross_OX3', ...) -- applied to permutation
        # params of size > 6 when two parents are selected (:117-134, :144-148)
        self.ga = dict(mutation_rate=mutation_rate, crossover_rate=crossover_rate,
                       must_mutate_count=must_mutate_count, normal=normal, sigma=sigma,
                       crossover_strength=crossover_strength, op=op, crossover=crossover)

    def propose(self, m):
        # GreedySelectionMixin.select: the global best config (random() before any result)
        self._parent = self.best_row()
        return self.engine.propose_ga(m, self._parent, None, round_=self.round, cand_base=self.round_base(), **self.ga)

    def hash_proposals(self, vals, base):
        # children keep most of the parent's values: reuse its inner digests
        parent = getattr(self, "_parent", None)
        hp = getattr(self.engine, "hash_parent", None)
        if parent is None or hp is None:
            return self.engine.hash(vals)
        return hp(vals, parent)


class GpuGGA(GpuGA):
    """globalGA.NormalGreedyMutation(crossover_rate=0.5, crossover_strength=0.2) (globalGA.py:129)"""

    def __init__(self, *pargs, **kwargs):
        kwargs.setdefault("mutation_rate", 0.1)
        super().__init__(*pargs, crossover_rate=0.5, crossover_strength=0.2, normal=True, op=5, **kwargs)


def _shared_model(kw) -> SharedModel:
    return SharedModel(device=kw.get("device", 0), seed=kw.get("seed", 0), lengthscale=kw.get("lengthscale", 0.3),
                       min_train=kw.get("min_train", 4), precision=kw.get("precision", 64),
                       engine_factory=kw.pop("engine_factory", None), y_transform=kw.get("y_transform"))


def pso_ga_de_bandit(bandit_seed: Optional[int] = None, **kw) -> AUCBanditMetaTechnique:
    """GPU counterpart of the reference's "PSO_GA_DE" bandit (bandittechniques.py:311-320):
    the four techniques share ONE SharedModel (one device context: one GP fit
    per generation, one dedup set) with a population slot each.  bandit_seed
    fixes the bandit's tie-break shuffles (required for SPMD runs: every rank
    must order the techniques the same way)."""
    kw = dict(kw)
    shared = kw.pop("shared", None) or _shared_model(kw)
    return AUCBanditMetaTechnique([
        GpuPSO(name="gpu-pso", shared=shared, **kw),
        GpuGA(name="gpu-ga", crossover_rate=0.5, shared=shared, **kw),
        GpuDifferentialEvolution(name="gpu-de", shared=shared, **kw),
        GpuGGA(name="gpu-gga", shared=shared, **kw),
    ], name="GPU_PSO_GA_DE", seed=bandit_seed)


def bandit_a(bandit_seed: Optional[int] = None, **kw) -> AUCBanditMetaTechnique:
    """GPU counterpart of the reference's default root technique,
    "AUCBanditMetaTechniqueA" (bandittechniques.py:273-278; technique.py:349):
    DifferentialEvolutionAlt (cr 0.2), UniformGreedyMutation (mutation rate
    0.1, evolutionarytechniques.py:13-24) and NormalGreedyMutation(mutation_rate
    =0.3) on one shared model.  The fourth child, RandomNelderMead, is a
    sequential simplex technique outside the scoring path (DESIGN.md "Out of
    scope") and is not built."""
    kw = dict(kw)
    shared = kw.pop("shared", None) or _shared_model(kw)
    return AUCBanditMetaTechnique([
        GpuDifferentialEvolution(name="gpu-de-alt", cr=0.2, shared=shared, **kw),
        GpuGA(name="gpu-uniform-greedy-mutation", mutation_rate=0.1, shared=shared, **kw),
        GpuGA(name="gpu-normal-greedy-mutation", mutation_rate=0.3, normal=True, shared=shared, **kw),
    ], name="GpuAUCBanditMetaTechniqueA", seed=bandit_seed)


def bandit_b(bandit_seed: Optional[int] = None, **kw) -> AUCBanditMetaTechnique:
    """"AUCBanditMetaTechniqueB" (bandittechniques.py:279-282): DifferentialEvolutionAlt
    and UniformGreedyMutation on one shared model"""
    kw = dict(kw)
    shared = kw.pop("shared", None) or _shared_model(kw)
    return AUCBanditMetaTechnique([
        GpuDifferentialEvolution(name="gpu-de-alt", cr=0.2, shared=shared, **kw),
        GpuGA(name="gpu-uniform-greedy-mutation", mutation_rate=0.1, shared=shared, **kw),
    ], name="GpuAUCBanditMetaTechniqueB", seed=bandit_seed)


_XO = ("op3_cross_OX3", "op3_cross_OX1", "op3_cross_PMX", "op3_cross_PX", "op3_cross_CX")


def reference_registry(wrap=None, bandit_cls=None, **kw) -> List[SearchTechniqueBase]:
    """GPU counterparts of the population techniques the reference registers,
    same parameters, names prefixed "Gpu" (crossover variants suffixed, since
    the reference registers all five PSO / GA variants under one class name):

      DifferentialEvolution (cr 0.9), DifferentialEvolutionAlt (cr 0.2),
      DifferentialEvolution_20_100      differentialevolution.py:148-151
      PSO(crossover=OX3|OX1|PMX|PX|CX)  pso.py:80-84
      GA(crossover=..., mutation 0.1, crossover rate 0.8)
                                        evolutionarytechniques.py:146-150
      ga-base, UniformGreedyMutation05/10/20, NormalGreedyMutation05/10/20
                                        evolutionarytechniques.py:151-158
      GGA                               globalGA.py:129
      PSO_GA_DE bandit                  bandittechniques.py:311-320
      AUCBanditMetaTechniqueA / B       bandittechniques.py:273-282 (A without
                                        RandomNelderMead: see bandit_a)

    `wrap(cls)` maps each GPU technique class before construction (the
    reference-side binding rebases them onto its SearchTechnique)
    and `bandit_cls` replaces this module's AUCBanditMetaTechnique for the
    bandit.  `kw` goes to every technique (pool, batch, device, seed, ...).  The
    DE population size is the device population (`population=`), not 30 / 100:
    every member is scored each round."""
    W = wrap or (lambda c: c)
    kw = dict(kw)
    ef = kw.get("engine_factory")
    sm = _shared_model(kw)          # the bandit's children share one model (pops engine_factory; every
    #                                 technique, stand-alone or not, gets the requested precision)
    if ef is not None:
        kw["engine_factory"] = ef   # ... while each stand-alone technique builds its own
    DE, PSO, GA, GGA = W(GpuDifferentialEvolution), W(GpuPSO), W(GpuGA), W(GpuGGA)
    out: List[SearchTechniqueBase] = [
        DE(name="GpuDifferentialEvolution", cr=0.9, **kw),
        DE(name="GpuDifferentialEvolutionAlt", cr=0.2, **kw),
        DE(name="GpuDifferentialEvolution_20_100", cr=0.2, **kw),
    ]
    for xo in _XO:
        out.append(PSO(name="GpuPSO-" + xo[len("op3_cross_"):], crossover=xo, **kw))
    for xo in _XO:
        out.append(GA(name="GpuGA-" + xo[len("op3_cross_"):], crossover=xo, mutation_rate=0.10, crossover_rate=0.8,
                      **kw))
    out.append(GA(name="Gpuga-base", mutation_rate=0.10, **kw))
    for r in (5, 10, 20):
        out.append(GA(name="GpuUniformGreedyMutation%02d" % r, mutation_rate=r / 100.0, **kw))
    for r in (5, 10, 20):
        out.append(GA(name="GpuNormalGreedyMutation%02d" % r, mutation_rate=r / 100.0, normal=True, **kw))
    out.append(GGA(name="GpuGGA", **kw))
    children = [PSO(name="gpu-pso", shared=sm, **kw), GA(name="gpu-ga", crossover_rate=0.5, shared=sm, **kw),
                DE(name="gpu-de", shared=sm, **kw), GGA(name="gpu-gga", shared=sm, **kw)]
    out.append((bandit_cls or AUCBanditMetaTechnique)(children, name="GPU_PSO_GA_DE"))
    # AUCBanditMetaTechniqueA / B, each with a model of its own
    sa, sb = _shared_model(dict(kw)), _shared_model(dict(kw))
    for nm, kids in (("GpuAUCBanditMetaTechniqueA",
                      [DE(name="gpu-de-alt", cr=0.2, shared=sa, **kw),
                       GA(name="gpu-uniform-greedy-mutation", mutation_rate=0.1, shared=sa, **kw),
                       GA(name="gpu-normal-greedy-mutation", mutation_rate=0.3, normal=True, shared=sa, **kw)]),
                     ("GpuAUCBanditMetaTechniqueB",
                      [DE(name="gpu-de-alt", cr=0.2, shared=sb, **kw),
                       GA(name="gpu-uniform-greedy-mutation", mutation_rate=0.1, shared=sb, **kw)])):
        out.append((bandit_cls or AUCBanditMetaTechnique)(kids, name=nm))
    return out
