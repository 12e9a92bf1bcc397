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
        """technique.py:88-111 -> a DesiredResult-like record, None or False"""
        cfg = self.desired_configuration()
        if cfg is None:
            return None
        if cfg is False:
            return False
        dr = self.driver.make_desired_result(cfg, requestor=self.name)
        self.driver.register_result_callback(dr, self.handle_requested_result)
        self.request_count += 1
        return dr

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
    """Area-under-curve credit assignment (Fialho et al.), bandittechniques.py:82-146"""

    def __init__(self, *args, **kwargs):
        super().__init__(*args, **kwargs)
        self.debug = kwargs.get("debug", False)
        self.auc_sum = dict((t, 0) for t in self.keys)
        self.auc_decay = dict((t, 0) for t in self.keys)

    def exploitation_term_slow(self, key):
        score = 0.0
        pos = 0
        for t, value in self.history:
            if t is key:
                pos += 1
                if value:
                    score += pos
        if pos:
            return score * 2.0 / (pos * (pos + 1.0))
        return 0.0

    def exploitation_term_fast(self, key):
        score = self.auc_sum[key]
        pos = self.use_counts[key]
        if pos:
            return score * 2.0 / (pos * (pos + 1.0))
        return 0.0

    def exploitation_term(self, key):
        v1 = self.exploitation_term_fast(key)
        if self.debug:
            assert v1 == self.exploitation_term_slow(key)
        return v1

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
class GpuBatchTechnique(SearchTechnique):
    """Base of the device-scored population techniques.

    One round = propose `pool` candidates with the technique's operator,
    hash_config + dedup against every configuration the driver has seen,
    score with the GP (EI) fitted on the driver's results, keep the top
    `batch`; desired_configuration() then returns them one per call.
    """

    # DE / GA pools shard over the ranks of a process group by GLOBAL candidate
    # index; PSO moves its (small) swarm on every rank (replicas)
    sharded = True

    def __init__(self, pool: int = 1 << 14, batch: int = 8, population: int = 1024, device: int = 0,
                 seed: int = 0, lengthscale: float = 0.3, min_train: int = 4, acq: str = "ei",
                 group=None, surrogate=None, *pargs, **kwargs):
        super().__init__(*pargs, **kwargs)
        # surrogate: None = the GP fitted on the driver's results (EI / UCB); or a
        # tree ensemble over the same features (sklearn regressor, XGBoost JSON,
        # forest.Forest) ranking candidates by predicted objective (minimised),
        # the multi-stage tuner's model scoring (multi_stage.py:8-22, :109-123)
        self.surrogate = surrogate
        # multi-GPU: with torch.distributed initialised and
        # world > 1, rank r scores candidates [base + r*pool, base + (r+1)*pool)
        # of every round and the local top-k lists are all-gathered and merged
        self.group = group
        self.pool, self.batch, self.population = int(pool), int(batch), int(population)
        self.device, self.seed, self.lengthscale, self.min_train = device, seed, lengthscale, min_train
        self.acq_kind = acq
        self.engine = None
        self.queue: List[Dict[str, Any]] = []
        self.round = 0
        self.cand_base = 0
        self._hist_seen = 0

    def __deepcopy__(self, memo):
        # device handles are never copied (driver.py:75 deep-copies techniques)
        cls = self.__class__
        new = cls.__new__(cls)
        memo[id(self)] = new
        for k, v in self.__dict__.items():
            setattr(new, k, None if k == "engine" else (v if k == "group" else copy.deepcopy(v, memo)))
        return new

    def _dist(self):
        """(rank, world) of the sharded round (world 1 without torch.distributed)"""
        try:
            import torch.distributed as dist
        except Exception:  # pragma: no cover
            return 0, 1
        if not self.sharded or not dist.is_available() or not dist.is_initialized():
            return 0, 1
        return dist.get_rank(self.group), dist.get_world_size(self.group)

    def round_base(self) -> int:
        """global index of this rank's first candidate of the current round"""
        rank, _ = self._dist()
        return self.cand_base + rank * self.pool

    # -- device state ------------------------------------------------------
    def _ensure_engine(self):
        if self.engine is None:
            from .engine import BatchEngine
            self.engine = BatchEngine(self.manipulator, device=self.device, seed=self.seed)
            self.engine.history_reset(1024)
            self.init_population()
        return self.engine

    def init_population(self):
        self.engine.population_init(max(self.population, 4), round_=0)

    def _sync_history(self):
        """push digests of newly seen configurations to the device set"""
        seen = self.driver.seen_hashes()
        if len(seen) > self._hist_seen:
            self.engine.history_add(seen[self._hist_seen:])
            self._hist_seen = len(seen)

    def _fit(self) -> bool:
        cfgs, y = self.driver.training_configs()
        if len(y) < self.min_train:
            return False
        # the driver's results are append-only: encode only the new ones
        X = getattr(self, "_X", None)
        if X is None or X.shape[0] > len(cfgs):
            X = np.zeros((0, self.engine.spec.n_features))
        if X.shape[0] < len(cfgs):
            X = np.vstack([X, self.engine.features_host(cfgs[X.shape[0]:])])
        self._X = X
        self.engine.gp_fit(X, y, lengthscale=self.lengthscale, sigma_f2=1.0, sigma_n2=1e-6, jitter=1e-8)
        return True

    def propose(self, m: int):
        """-> (values [P][m] device tensor, invalid mask or None)"""
        raise NotImplementedError

    def _round(self):
        import torch
        eng = self._ensure_engine()
        self._sync_history()
        rank, world = self._dist()
        base = self.round_base()
        vals, invalid = self.propose(self.pool)
        dig = eng.hash(vals)
        dup = eng.dedup(dig)
        if invalid is not None:
            dup = torch.maximum(dup, invalid)
        if self.surrogate is not None:
            if getattr(eng, "forest", None) is None:
                eng.forest_set(self.surrogate)
            _, score = eng.forest_predict(eng.encode(vals), dup=dup)
        elif self._fit():
            feat = eng.encode(vals)
            _, _, score = eng.gp_score(feat, acq=eng.acq(self.acq_kind), dup=dup)
        else:  # no model yet: every non-duplicate candidate is equally good (lowest index first)
            score = torch.zeros(vals.shape[1], dtype=torch.float64, device=vals.device)
        idx, top = eng.topk(score, self.batch, dup=dup, cand_base=base)   # GLOBAL candidate indices
        loc = torch.where(idx >= 0, idx - base, torch.zeros_like(idx))
        rows = vals[:, loc]
        if world > 1:
            from .dist import allgather_selection
            idx, top, rows = allgather_selection(idx, top, dig[loc], rows, self.batch, group=self.group)
        keep = idx >= 0
        idx, rows = idx[keep], rows[:, keep]
        self.queue.extend(eng.decode(rows))
        self.after_round(vals, idx)
        self.round += 1
        self.cand_base += world * self.pool

    def after_round(self, vals, idx):
        pass

    def desired_configuration(self):
        try:
            if not self.queue:
                self._round()
            if not self.queue:
                return None
            return self.queue.pop(0)
        except Exception as ex:  # never raise into the driver loop
            log.warning("%s: device round failed: %s", self.name, ex)
            return None


class GpuDifferentialEvolution(GpuBatchTechnique):
    """Batched DifferentialEvolution(Alt) (differentialevolution.py:29-151):
    every round proposes DE/rand/1/bin trials for the population; evaluated
    trials replace their target when better (handle_requested_result, :131-139)."""

    def __init__(self, cr: float = 0.2, n_cross: int = 1, information_sharing: int = 1, *pargs, **kwargs):
        super().__init__(*pargs, **kwargs)
        self.cr, self.n_cross, self.information_sharing = cr, n_cross, information_sharing
        self._pending: Dict[str, int] = {}

    def propose(self, m):
        # share information with other techniques: the driver's best config joins
        # the donor pool information_sharing times (differentialevolution.py:112-116)
        best = self.driver.best_configuration()
        b = None if best is None else self.engine.spec.encode_configs([best])[:, 0]
        return self.engine.propose_de(m, round_=self.round, cand_base=self.round_base(), cr=self.cr,
                                      n_cross=self.n_cross, best=b,
                                      information_sharing=self.information_sharing), None

    def after_round(self, vals, idx):
        npop = self.engine.npop
        for j, g in enumerate(idx.cpu().numpy().tolist()):   # global index g targets member g % npop
            cfg = self.queue[len(self.queue) - len(idx) + j]
            self._pending[self.driver.config_key(cfg)] = g % npop

    def handle_requested_result(self, result):
        import torch
        key = self.driver.config_key(result.configuration)
        tgt = self._pending.pop(key, None)
        if tgt is None or self.engine is None:
            return
        parent = self.driver.population_result(self, tgt)
        if parent is None or self.objective.lt(result, parent):
            vals = torch.from_numpy(self.engine.spec.encode_configs([result.configuration])).to(self.engine.device)
            self.engine.population_replace(vals, torch.tensor([tgt], device=self.engine.device))
            self.driver.set_population_result(self, tgt, result)


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
        best = self.driver.best_configuration()
        if best is None:  # no result yet: particle 0 stands in for the global best
            gb = self.engine.population_get()[:, 0]
        else:
            gb = self.engine.spec.encode_configs([best])[:, 0]
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
        best = self.driver.best_configuration()
        p1 = None if best is None else self.engine.spec.encode_configs([best])[:, 0]
        return self.engine.propose_ga(m, p1, None, round_=self.round, cand_base=self.round_base(), **self.ga)


class GpuGGA(GpuGA):
    """globalGA.NormalGreedyMutation(crossover_rate=0.5, crossover_strength=0.2) (globalGA.py:288)"""

    def __init__(self, *pargs, **kwargs):
        kwargs.setdefault("mutation_rate", 0.1)
        super().__init__(*pargs, crossover_rate=0.5, crossover_strength=0.2, normal=True, op=5, **kwargs)


def pso_ga_de_bandit(bandit_seed: Optional[int] = None, **kw) -> AUCBanditMetaTechnique:
    """GPU counterpart of the reference's "PSO_GA_DE" bandit (bandittechniques.py:311-320).
    bandit_seed fixes the bandit's tie-break shuffles (required for SPMD runs:
    every rank must order the techniques the same way)."""
    return AUCBanditMetaTechnique([
        GpuPSO(name="gpu-pso", **kw),
        GpuGA(name="gpu-ga", crossover_rate=0.5, **kw),
        GpuDifferentialEvolution(name="gpu-de", **kw),
        GpuGGA(name="gpu-gga", **kw),
    ], name="GPU_PSO_GA_DE", seed=bandit_seed)


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

    `wrap(cls)` maps each GPU technique class before construction (the
    reference-side binding rebases them onto its SearchTechnique)
    and `bandit_cls` replaces this module's AUCBanditMetaTechnique for the
    bandit.  `kw` goes to every technique (pool, batch, device, seed, ...).  The
    DE population size is the device population (`population=`), not 30 / 100:
    every member is scored each round."""
    W = wrap or (lambda c: c)
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
    children = [PSO(name="gpu-pso", **kw), GA(name="gpu-ga", crossover_rate=0.5, **kw), DE(name="gpu-de", **kw),
                GGA(name="gpu-gga", **kw)]
    out.append((bandit_cls or AUCBanditMetaTechnique)(children, name="GPU_PSO_GA_DE"))
    return out
