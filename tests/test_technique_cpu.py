"""Plugin layer on the CPU: AUC bandit bookkeeping, meta-technique ordering and
credit, the driver's dedup/result feedback, and the C1 plumbing config
(2-D Rosenbrock under an AUC bandit).

The bandit is restated from opentuner/search/bandittechniques.py:20-165; the
checks below are the reference's own invariants (exploitation_term_fast ==
exploitation_term_slow, asserted there under debug=True, :123-126) plus
hand-computed AUC values.  Config identity in the CPU tests comes from the
oracle's hashlib restatement of hash_config (test infrastructure only).
"""
import copy
import math
import random

import pytest

from oracle import hashing as OH
from oracle import space as OS
from uptune_amd import technique as T
from uptune_amd.driver import MinimizeTime, Result, SearchDriver
from uptune_amd.manipulator import ConfigurationManipulator, FloatParameter


def test_auc_hand_computed():
    q = T.AUCBanditQueue(["a", "b"])
    for k, v in [("a", 1), ("b", 0), ("a", 0), ("a", 1)]:
        q.on_result(k, v)
    # a: positions 1 (hit), 2, 3 (hit) -> (1 + 3) * 2 / (3 * 4)
    assert q.exploitation_term("a") == pytest.approx(8 / 12)
    assert q.exploitation_term("b") == 0.0
    # exploration: sqrt(2 log2(|history|) / uses)
    assert q.exploration_term("a") == pytest.approx(math.sqrt(2 * math.log(4, 2) / 3))
    assert q.bandit_score("b") == pytest.approx(0.05 * math.sqrt(2 * 2 / 1))


def _auc_direct(history, key):
    """AUC straight from its definition over the window: number the uses of
    `key` 1..pos in order, sum the numbers of the credited ones, times
    2 / (pos (pos + 1)) (the reference's exploitation_term_slow invariant,
    bandittechniques.py:107-126)"""
    score = pos = 0
    for k, v in history:
        if k == key:
            pos += 1
            if v:
                score += pos
    return score * 2.0 / (pos * (pos + 1.0)) if pos else 0.0


@pytest.mark.parametrize("window", [3, 7, 500])
def test_auc_incremental_equals_definition_with_window(window):
    rng = random.Random(window)
    keys = ["k%d" % i for i in range(5)]
    q = T.AUCBanditQueue(keys, window=window)
    for _ in range(400):
        q.on_result(rng.choice(keys), rng.random() < 0.3)
        for k in keys:
            assert q.exploitation_term(k) == pytest.approx(_auc_direct(q.history, k), abs=1e-12)
        assert len(q.history) <= window
        assert sum(q.use_counts.values()) == len(q.history)


def test_unused_key_explored_first():
    q = T.AUCBanditQueue(["a", "b", "c"])
    for _ in range(5):
        q.on_result("a", 1)
        q.on_result("b", 1)
    order = list(q.ordered_keys(random.Random(0)))
    assert order[0] == "c"                      # infinite exploration term
    assert q.exploration_term("c") == float("inf")


class _Fixed(T.SearchTechnique):
    """returns queued values: a config dict, None or False"""

    def __init__(self, seq, **kw):
        super().__init__(**kw)
        self.seq = list(seq)
        self.results = []

    def desired_configuration(self):
        return self.seq.pop(0) if self.seq else None

    def handle_requested_result(self, result):
        self.results.append(result)


class _RandomSearch(T.SearchTechnique):
    def __init__(self, seed, **kw):
        super().__init__(**kw)
        self.rng = random.Random(seed)

    def desired_configuration(self):
        return {p.name: self.rng.uniform(p.min_value, p.max_value) for p in self.manipulator.params}


def _space2():
    return ConfigurationManipulator([FloatParameter(0, -1000.0, 1000.0), FloatParameter(1, -1000.0, 1000.0)])


def _hash_fn(manip):
    ospace = [OS.Param(p.name, OS.FLOAT, p.min_value, p.max_value) for p in manip.params]
    return lambda cfg: OH.hash_config(ospace, [cfg[p.name] for p in manip.params])


def _rosen(cfg):
    x0, x1 = cfg[0], cfg[1]
    return 100.0 * (x1 - x0 * x0) ** 2 + (x0 - 1.0) ** 2


def test_meta_order_skip_and_credit():
    m = _space2()
    waiting = _Fixed([False, False], name="waiting")
    empty = _Fixed([], name="empty")
    giver = _Fixed([{0: 1.0, 1: 1.0}, {0: 2.0, 1: 2.0}], name="giver")
    meta = T.AUCBanditMetaTechnique([waiting, empty, giver], seed=0)
    d = SearchDriver(m, meta, parallelism=1, hash_fn=_hash_fn(m))
    root = d.root_technique
    dr = root.desired_result()
    assert dr.requestor == "giver"
    # "empty" returned None and was credited 0; "waiting" returned False and was not
    hist_keys = [k for k, _ in root.bandit.history]
    assert "waiting" not in hist_keys
    assert hist_keys.count("empty") == (1 if "empty" in hist_keys else 0)
    d._add_request(dr)
    d.report(dr, 3.0)
    d.process_new_results()
    assert ("giver", True) in [(k, bool(v)) for k, v in root.bandit.history]
    g = root.name_to_technique["giver"]
    assert len(g.results) == 1 and g.results[0].was_new_best


def test_driver_duplicate_request_not_reevaluated():
    m = _space2()
    cfg = {0: 5.0, 1: 25.0}
    tech = _Fixed([dict(cfg), dict(cfg), {0: 1.0, 1: 1.0}], name="dups")
    d = SearchDriver(m, tech, parallelism=3, hash_fn=_hash_fn(m))
    calls = []

    def ev(c):
        calls.append(c)
        return _rosen(c)

    d.main(ev, test_limit=2)
    assert len(calls) == 2                       # the repeated config ran once
    assert d.test_count == 3
    # the duplicate request's own callback fires at the next result pass, as in
    # the reference (result_callbacks re-queues it until dr.result is set by the
    # first request's callback, driver.py:136-155)
    d.process_new_results()
    got = d.root_technique.results
    assert len(got) == 3                         # but every request received a result
    assert sorted(r.time for r in got) == sorted([_rosen(cfg), _rosen(cfg), 0.0])
    assert d.best_result.time == 0.0


def test_c1_rosenbrock_plumbing():
    """C1: FloatParameter(0|1, -1000, 1000), bandit over techniques, test-limit"""
    m = _space2()
    meta = T.AUCBanditMetaTechnique([_RandomSearch(1, name="r1"), _RandomSearch(2, name="r2"),
                                     _Fixed([], name="none")], bandit_kwargs={"window": 10 ** 6}, seed=3)
    d = SearchDriver(m, meta, parallelism=4, hash_fn=_hash_fn(m))
    best = d.main(_rosen, test_limit=400)
    assert d.test_count > 400
    assert len(d.results) == d.test_count        # random floats never repeat
    times = [r.time for r in d.results.values()]
    assert best.time == min(times)
    b = d.root_technique.bandit
    assert set(b.use_counts) == {"r1", "r2", "none"}
    assert sum(b.use_counts.values()) == len(b.history) <= b.window
    # new-best credits are exactly the results flagged was_new_best
    assert sum(1 for _, v in b.history if v) == sum(1 for r in d.results.values() if r.was_new_best)


def test_register_and_get_enabled():
    t = _Fixed([], name="registered-test-tech")
    T.register(t)
    try:
        assert T.get_enabled(["registered-test-tech"]) == [t]
        with pytest.raises(Exception):
            T.get_enabled(["no-such-technique"])
    finally:
        T.the_registry.remove(t)


def test_gpu_techniques_deepcopy_and_no_device():
    """technique instances are deep-copied per driver (driver.py:75): the device
    handle is never copied; without a GPU the technique logs and returns None
    (the driver retries forever on exceptions, api.py:433-435)."""
    meta = T.pso_ga_de_bandit(pool=256, batch=4, population=64)
    meta2 = copy.deepcopy(meta)
    assert [t.name for t in meta2.techniques] == ["gpu-pso", "gpu-ga", "gpu-de", "gpu-gga"]
    assert all(t.engine is None for t in meta2.techniques)
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present: covered by tests/test_gpu_technique.py")
    m = _space2()
    d = SearchDriver(m, meta2, parallelism=2, hash_fn=_hash_fn(m))
    assert d.root_technique.desired_result() is None


def test_reference_registry_mirrors_reference_techniques():
    """reference_registry(): one GPU technique per population technique the
    reference registers (differentialevolution.py:148-151, pso.py:80-84,
    evolutionarytechniques.py:146-158, globalGA.py:129, bandittechniques.py:311-320);
    built without touching a device."""
    from uptune_amd._lib import CROSSOVERS
    reg = T.reference_registry(pool=256, batch=4)
    names = [t.name for t in reg]
    assert len(names) == len(set(names)) == 24
    by = {t.name: t for t in reg}
    assert by["GpuDifferentialEvolution"].cr == 0.9 and by["GpuDifferentialEvolutionAlt"].cr == 0.2
    for xo in ("OX1", "OX3", "PMX", "PX", "CX"):
        assert by["GpuPSO-" + xo].crossover in CROSSOVERS
        g = by["GpuGA-" + xo].ga
        assert g["crossover"] in CROSSOVERS and g["crossover_rate"] == 0.8 and g["mutation_rate"] == 0.1
    assert by["GpuNormalGreedyMutation20"].ga["normal"] and not by["GpuUniformGreedyMutation05"].ga["normal"]
    assert by["GpuGGA"].ga["crossover_strength"] == 0.2
    assert all(getattr(t, "engine", None) is None for t in reg if isinstance(t, T.GpuBatchTechnique))
    assert by["GPU_PSO_GA_DE"].bandit is not None
    # the default root technique, AUCBanditMetaTechniqueA (bandittechniques.py:273-278),
    # without RandomNelderMead; its children share one model
    a = by["GpuAUCBanditMetaTechniqueA"]
    kids = {t.name: t for t in a.techniques}
    assert kids["gpu-de-alt"].cr == 0.2
    assert kids["gpu-uniform-greedy-mutation"].ga["mutation_rate"] == 0.1
    assert not kids["gpu-uniform-greedy-mutation"].ga["normal"]
    assert kids["gpu-normal-greedy-mutation"].ga["mutation_rate"] == 0.3
    assert kids["gpu-normal-greedy-mutation"].ga["normal"]
    assert len({id(t.model) for t in a.techniques}) == 1
    assert [t.name for t in by["GpuAUCBanditMetaTechniqueB"].techniques] == ["gpu-de-alt",
                                                                           "gpu-uniform-greedy-mutation"]
    assert T.bandit_a(pool=256).bandit.C == 0.05 and T.bandit_a(pool=256).bandit.window == 500
    # the reference-side binding rebases every class through `wrap`
    class _Tag:
        pass

    reg2 = T.reference_registry(wrap=lambda c: type("W" + c.__name__, (c, _Tag), {}), pool=256)
    bandits = [t for t in reg2 if isinstance(t, T.AUCBanditMetaTechnique)]
    assert len(bandits) == 3
    assert all(isinstance(t, _Tag) for t in reg2 if t not in bandits)
    assert all(isinstance(c, _Tag) for b in bandits for c in b.techniques)


def test_c1_bandit_a_over_the_oracle_engine():
    """C1's root technique (AUCBanditMetaTechniqueA's device counterpart,
    technique.bandit_a) through the driver with the CPU stand-in engine
    (tests/_oracle_engine.py: the oracle's propose / hash / GP): every child runs,
    nothing is evaluated twice, and the bandit's credits are the new bests"""
    from _oracle_engine import OracleEngine
    m = _space2()
    meta = T.bandit_a(bandit_seed=5, pool=256, batch=4, population=30, seed=11, lengthscale=0.3,
                      y_transform="rank", engine_factory=OracleEngine)
    d = SearchDriver(m, meta, parallelism=4, hash_fn=_hash_fn(m))
    best = d.main(_rosen, test_limit=160)
    assert d.test_count >= 160
    assert len(d.results) == d.test_count
    b = d.root_technique.bandit
    assert set(b.use_counts) == {"gpu-de-alt", "gpu-uniform-greedy-mutation", "gpu-normal-greedy-mutation"}
    assert all(v > 0 for v in b.use_counts.values())
    assert best.time == min(r.time for r in d.results.values())
    assert sum(1 for _, v in b.history if v) == sum(1 for r in d.results.values() if r.was_new_best)
