"""World-size-2 gloo run of DistributedSearchDriver (uptune_amd/driver.py), the
SPMD search loop behind C5: rank 0 evaluates every generation and broadcasts
(objective values, digests); the other ranks never call the objective, yet end
with the same result history, configuration for configuration, as rank 0 and as
a single-process SearchDriver.  If any rank's requests diverge, every rank raises.

The techniques are CPU random searches and config identity is the oracle's
hashlib hash_config (test infrastructure), so no GPU is involved.
"""
import os
import random
import socket

import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import hashing as OH
from oracle import space as OS
from uptune_amd import technique as T
from uptune_amd.driver import DistributedSearchDriver, SearchDriver
from uptune_amd.manipulator import ConfigurationManipulator, FloatParameter


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


def _tree(seed_shift=0):
    return T.AUCBanditMetaTechnique([_RandomSearch(1 + seed_shift, name="r1"), _RandomSearch(2, name="r2")],
                                    bandit_kwargs={"window": 10 ** 6}, seed=3)


_SEED_CFGS = [{0: float(i), 1: float(i * i)} for i in range(-3, 4)]


def _history(d):
    return [(k, r.time) for k, r in d.results.items()]


def _worker(rank, world, port, diverge, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    m = _space2()
    calls = []

    def ev(cfg):
        calls.append(cfg)
        return _rosen(cfg)

    d = DistributedSearchDriver(m, _tree(1 if (diverge and rank == 1) else 0), parallelism=4, hash_fn=_hash_fn(m))
    try:
        d.seed_results(_SEED_CFGS, ev)
        best = d.main(ev, test_limit=60, max_generations=1 if diverge else 100000)
        q.put((rank, "ok", len(calls), _history(d), best.time, d.test_count))
    except RuntimeError as ex:
        q.put((rank, "diverged", len(calls), str(ex), None, None))
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(world, diverge):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, diverge, q)) for r in range(world)]
    for p in ps:
        p.start()
    out = sorted((q.get(timeout=180) for _ in range(world)), key=lambda t: t[0])
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    return out


def test_rank0_evaluates_and_all_ranks_share_history():
    out = _run(2, diverge=False)
    (r0, s0, calls0, hist0, best0, n0), (r1, s1, calls1, hist1, best1, n1) = out
    assert s0 == s1 == "ok"
    assert calls1 == 0                       # only rank 0 runs the objective
    assert calls0 == len(hist0) > len(_SEED_CFGS)
    assert hist1 == hist0 and best1 == best0 and n1 == n0

    # the same search as one process: identical history
    m = _space2()
    d = SearchDriver(m, _tree(), parallelism=4, hash_fn=_hash_fn(m))
    d.record_seed(_SEED_CFGS, [_rosen(c) for c in _SEED_CFGS], d.config_keys(_SEED_CFGS))
    best = d.main(_rosen, test_limit=60)
    assert _history(d) == hist0 and best.time == best0


def test_diverging_rank_raises_on_every_rank():
    """a divergence seen by one rank is agreed on collectively (all_reduce of
    the check): EVERY rank raises, none is left waiting in the next collective
    (the src rank used to block in the next broadcast)"""
    out = _run(2, diverge=True)
    assert out[0][1] == out[1][1] == "diverged"
    assert "this rank agrees" in out[0][3] and "this rank differs" in out[1][3]
    assert out[1][2] == 0
