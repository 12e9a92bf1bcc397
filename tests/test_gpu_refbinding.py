"""The reference-side binding and the TuningRunManager batch path on the real
device engine (libuthot.so): the scenarios of tests/test_refbinding_cpu.py and
tests/test_tuning_manager_cpu.py with engine_factory=None."""
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

import _refstandin as R  # noqa: E402
from uptune_amd import refbinding  # noqa: E402
from uptune_amd import technique as T  # noqa: E402
from uptune_amd.manipulator import (BooleanParameter, ConfigurationManipulator, EnumParameter,  # noqa: E402
                                    FloatParameter, IntegerParameter)


def _mirror():
    return ConfigurationManipulator([FloatParameter("x", -2.0, 2.0), FloatParameter("y", -2.0, 2.0),
                                     IntegerParameter("n", 0, 50), EnumParameter("mode", ["a", "b", "c"]),
                                     BooleanParameter("flag")])


def _obj(cfg):
    x, y = cfg["x"], cfg["y"]
    return (100.0 * (y - x * x) ** 2 + (x - 1.0) ** 2 + 0.01 * abs(cfg["n"] - 17)
            + (0.5 if cfg["mode"] != "b" else 0.0) + (0.25 if cfg["flag"] else 0.0))


@pytest.fixture()
def registry():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    R.the_registry.clear()
    ts = refbinding.register_all(R, bandit_cls=T.AUCBanditMetaTechnique, pool=4096, batch=4, population=256, seed=5,
                                 lengthscale=0.5)
    yield ts
    R.the_registry.clear()


@pytest.mark.parametrize("name", ["GpuDifferentialEvolution", "GpuPSO-PMX", "GpuGA-CX", "GPU_PSO_GA_DE",
                                  "GpuAUCBanditMetaTechniqueA"])
def test_reference_driver_on_device(registry, name, caplog):
    tech = {t.name: t for t in registry}[name]
    m = R.Manipulator(_mirror())
    d = R.SearchDriver(m, tech, parallelism=4)
    with caplog.at_level("WARNING"):
        d.main(_obj, test_limit=40)
    assert "round failed" not in caplog.text
    assert d.test_count > 40
    assert all(type(dr) is R.DesiredResult for dr in d._drs)
    hashes = [dr.configuration.hash for dr in d._drs]
    assert len(hashes) == len(set(hashes))
    # the device digests are the reference manipulator's hash_config (hashlib)
    for dr in d._drs:
        assert dr.configuration.hash == m.hash_config(dr.configuration.data)
    assert d.best_result.time < max(r.time for r in d._results)
    if name in ("GPU_PSO_GA_DE", "GpuAUCBanditMetaTechniqueA"):
        model = d.root_technique.techniques[0].gpu.model
        assert 0 < model.fits <= d.generation


def test_tuning_run_manager_on_device():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from uptune_amd.driver import Result, TuningRunManager
    mirror = _mirror()
    bandit = T.pso_ga_de_bandit(bandit_seed=1, pool=4096, batch=8, population=256, seed=2, lengthscale=0.5)
    api = TuningRunManager(mirror, bandit, parallelism=8)
    seen = set()
    for _ in range(6):
        drs = api.get_desired_results()
        assert 0 < len(drs) <= 8
        for dr in drs:
            assert dr.configuration.hash not in seen
            seen.add(dr.configuration.hash)
            api.report_result(dr, Result(time=_obj(dr.configuration.data)))
    api.finish()
    assert api.get_best_result() is not None and len(api.search_driver.results_query()) == len(seen)
