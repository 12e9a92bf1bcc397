"""f-3: batch dispatch through the reference's TuningRunManager API
(opentuner/api.py:6-104; uptune's ParallelTuning.get_config / api.sync,
python/uptune/api.py:428-446, :547-553) -- uptune_amd.driver.TuningRunManager
and its SPMD form, with the GPU technique layer on the oracle-backed CPU
engine (tests/_oracle_engine.py).  Also: a scoring round that fails on ONE
rank is agreed on collectively, so no rank is left inside the all-gather
(technique.py:408)."""
import os
import socket

import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

import _refstandin as R
from _oracle_engine import OracleEngine
from uptune_amd import technique as T
from uptune_amd.driver import DistributedTuningRunManager, Result, TuningRunManager
from uptune_amd.manipulator import ConfigurationManipulator, FloatParameter, IntegerParameter


def _mirror():
    return ConfigurationManipulator([FloatParameter("x", -2.0, 2.0), FloatParameter("y", -2.0, 2.0),
                                     IntegerParameter("n", 0, 50)])


def _obj(cfg):
    return 100.0 * (cfg["y"] - cfg["x"] ** 2) ** 2 + (cfg["x"] - 1.0) ** 2 + 0.01 * cfg["n"]


def _hash_fn(mirror):
    m = R.Manipulator(mirror)
    return m.hash_config


def _de(**kw):
    return T.GpuDifferentialEvolution(name="de", pool=512, batch=4, population=64, seed=3, lengthscale=0.5,
                                      engine_factory=OracleEngine, **kw)


class _GR:
    """a GlobalResult-like row (database/globalmodels.py:22-36): data, technique, result"""

    def __init__(self, data, technique, result):
        self.data, self.technique, self.result = data, technique, result


def test_get_desired_results_is_one_scoring_round():
    mirror = _mirror()
    api = TuningRunManager(mirror, _de(), parallelism=4, hash_fn=_hash_fn(mirror))
    seen = set()
    best = []
    for gen in range(6):
        drs = api.get_desired_results()
        assert len(drs) == 4                                   # the round's top-4, in one generation
        assert len({dr.generation for dr in drs}) == 1
        for dr in drs:
            assert dr.configuration.hash not in seen           # dedup vs everything requested so far
            seen.add(dr.configuration.hash)
            api.report_result(dr, Result(time=_obj(dr.configuration.data)))
        if api.get_best_result() is not None:     # best_result moves at the next generation (api.py:55-70)
            best.append(api.get_best_result().time)
    api.finish()
    best.append(api.get_best_result().time)
    tech = api.search_driver.root_technique
    assert tech.round == 6 and tech.model.fits >= 4
    assert best[-1] <= best[0]
    assert api.get_best_configuration() == api.get_best_result().configuration.data


def test_sync_injects_foreign_results():
    """api.sync (api.py:87-104): results measured by another search instance
    become this run's requests + results; they train the GP and join the
    dedup set, so this instance never asks for them again"""
    mirror = _mirror()
    api = TuningRunManager(mirror, _de(), parallelism=4, hash_fn=_hash_fn(mirror))
    other = TuningRunManager(mirror, _de(information_sharing=0), parallelism=4, hash_fn=_hash_fn(mirror))
    foreign = []
    for dr in other.get_desired_results():
        t = _obj(dr.configuration.data)
        other.report_result(dr, Result(time=t))
        foreign.append(_GR(dr.configuration.data, "other-node", t))
    api.sync(foreign)
    drv = api.search_driver
    assert len(drv.results_query()) == 4 and {r.requestor for r in drv.results_query()} == {"other-node"}
    fh = {drv.config_key(g.data) for g in foreign}
    for _ in range(4):
        for dr in api.get_desired_results():
            assert dr.configuration.hash not in fh
            api.report_result(dr, Result(time=_obj(dr.configuration.data)))
    assert api.get_best_result().time <= min(g.result for g in foreign)


# ---------------------------------------------------------------- SPMD (gloo, world 2)
def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _manager_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    mirror = _mirror()
    api = DistributedTuningRunManager(mirror, _de(), parallelism=4, hash_fn=_hash_fn(mirror))
    measured = 0
    for gen in range(5):
        drs = api.get_desired_results()
        if rank == 0:
            for dr in drs:
                measured += 1
                api.report_result(dr, Result(time=_obj(dr.configuration.data)))
    api.get_desired_results()          # exchange the last generation's results
    drv = api.search_driver
    q.put((rank, measured, [(r.configuration.hash, r.time) for r in drv.results_query()]))
    dist.destroy_process_group()


def _spmd(target, world=2, *extra):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=target, args=(r, world, port, q) + extra) for r in range(world)]
    for p in ps:
        p.start()
    out = sorted((q.get(timeout=180) for _ in range(world)), key=lambda t: t[0])
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    return out


def test_distributed_manager_rank0_measures_all_ranks_learn():
    (r0, m0, h0), (r1, m1, h1) = _spmd(_manager_worker)
    assert m0 == 20 and m1 == 0
    assert h0 == h1 and len(h0) == 20


def _fail_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    mirror = _mirror()
    from uptune_amd.driver import SearchDriver
    d = SearchDriver(mirror, _de(), parallelism=4, hash_fn=_hash_fn(mirror))
    tech = d.root_technique
    out = []
    for r in range(3):
        if r == 1 and rank == 1:        # inject a device failure on rank 1 only, round 2
            tech.propose = lambda m: (_ for _ in ()).throw(RuntimeError("injected device failure"))
        elif r == 2:
            tech.propose = T.GpuDifferentialEvolution.propose.__get__(tech)
        tech.queue.clear()
        out.append(tech.desired_configuration() is None)
    q.put((rank, out))
    dist.destroy_process_group()


def test_round_failure_on_one_rank_is_collective():
    """rank 1 fails inside its shard of round 2: BOTH ranks return None for
    that round (agreed by all_reduce before the all-gather) and both carry on
    with round 3 -- nobody hangs in a collective the other rank skipped"""
    out = _spmd(_fail_worker)
    assert out[0][1] == out[1][1] == [False, True, False]


def test_failed_async_fit_is_detected_and_refit(caplog):
    """a GP fit enqueued without a host wait whose kernel matrix is
    not positive definite must not poison later rounds silently: the next
    round checks it (gp_fit_ok), logs, and refits with more jitter"""
    import logging

    from uptune_amd.driver import SearchDriver
    mirror = _mirror()
    # lengthscale 1e3, no noise, no jitter: K ~ all ones, singular
    sm = T.SharedModel(seed=3, lengthscale=1e3, min_train=4, sigma_n2=0.0, jitter=0.0, engine_factory=OracleEngine)
    de = T.GpuDifferentialEvolution(name="de", pool=256, batch=4, population=64, seed=3, shared=sm)
    drv = SearchDriver(mirror, de, parallelism=4)
    with caplog.at_level(logging.WARNING, logger="uptune_amd.technique"):
        drv.main(_obj, test_limit=40, max_generations=10)
    eng = drv.root_technique.model.engine     # the driver's (deep) copy of the technique
    js = eng.calls["jitter"]
    assert js[0] == 0.0 and max(js) >= 1e-8            # escalated after the failed fit
    assert any("not positive definite" in r.message for r in caplog.records)
    assert eng.gp_fit_ok()                             # the refit succeeded
    assert drv.test_count >= 24                        # rounds kept producing configurations
