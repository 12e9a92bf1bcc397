"""GPU techniques behind the plugin API: the PSO/GA/DE/GGA bandit
(bandittechniques.py:311-320 "PSO_GA_DE") tuning an 8-D Rosenbrock through the
driver, every proposal scored on the device (hash_config, dedup, GP-EI, top-k).
"""
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu


def _space(P=8):
    from uptune_amd.manipulator import ConfigurationManipulator, FloatParameter, IntegerParameter
    ps = [FloatParameter("x%d" % i, -2.0, 2.0) for i in range(P - 1)] + [IntegerParameter("n", 0, 20)]
    return ConfigurationManipulator(ps)


def _rosen(cfg, P=8):
    x = [cfg["x%d" % i] for i in range(P - 1)]
    return sum(100.0 * (x[i + 1] - x[i] ** 2) ** 2 + (x[i] - 1.0) ** 2 for i in range(P - 2)) + 0.01 * cfg["n"]


def test_bandit_over_gpu_techniques_tunes():
    from oracle import hashing as OH
    from oracle import space as OS
    from uptune_amd import technique as T
    from uptune_amd.driver import SearchDriver

    m = _space()
    meta = T.pso_ga_de_bandit(pool=4096, batch=4, population=256, seed=7)
    d = SearchDriver(m, meta, parallelism=4)
    best = d.main(_rosen, test_limit=240)
    names = {t.name: t for t in d.root_technique.techniques}
    assert all(t.engine is not None for t in names.values())
    assert d.test_count > 240
    # no configuration was evaluated twice: dedup against history worked on the device
    assert len(d.results) == len(d.seen_hashes())
    # every sub-technique was used and produced results
    counts = d.root_technique.bandit.use_counts
    assert all(counts[n] > 0 for n in names), counts
    first = next(iter(d.results.values()))
    assert best.time < first.time
    # one shared model: one context (one engine), a population slot per technique,
    # and at most one GP fit per generation (a refit only when results changed)
    model = names["gpu-de"].model
    assert all(t.model is model for t in names.values())
    assert len({id(t.engine) for t in names.values()}) == 1
    assert sorted(model.slots.values()) == [0, 1, 2, 3]
    assert 0 < model.fits <= d.generation
    # device hash of every evaluated config equals the hashlib restatement
    ospace = [OS.Param(p.name, OS.FLOAT if type(p).__name__ == "FloatParameter" else OS.INT,
                       p.min_value, p.max_value) for p in m.params]
    for key, r in list(d.results.items())[:32]:
        assert key == OH.hash_config(ospace, [r.configuration.data[p.name] for p in m.params])


def test_gpu_de_replaces_population_rows():
    from uptune_amd import technique as T
    from uptune_amd.driver import SearchDriver

    m = _space()
    de = T.GpuDifferentialEvolution(pool=1024, batch=8, population=64, name="de")
    d = SearchDriver(m, de, parallelism=8)
    d.main(_rosen, test_limit=64)
    tech = d.root_technique
    pop = tech.engine.population_get().cpu().numpy()
    # each recorded population result is the row now stored at that slot
    replaced = list(tech._pop_results.items())
    assert replaced
    for idx, r in replaced:
        row = tech.engine.spec.encode_configs([r.configuration.data])[:, 0]
        assert (pop[:, idx] == row).all()


def test_gpu_technique_returns_none_on_device_error():
    """C-ABI errors are caught (api.py:433-435 retries forever on exceptions)"""
    from uptune_amd import technique as T
    from uptune_amd.driver import SearchDriver

    m = _space()
    ga = T.GpuGA(pool=256, batch=4, population=32, name="ga")
    ga.ga["max_retries"] = 99  # > 15: UT_EINVAL from ut_propose_ga
    d = SearchDriver(m, ga, parallelism=1)
    assert d.root_technique.desired_result() is None
