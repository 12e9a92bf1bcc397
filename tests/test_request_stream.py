"""The tutorial run's request stream replayed through the build's driver
(VERDICT r4 missing #1): the only reference data that pins dedup and
was_new_best semantics beyond the hash layout.

samples/tutorials/tuneup.opentuner.db holds a real OpenTuner run of
IntegerParameter('BLOCK_SIZE', 1, 10) under AUCBanditMetaTechniqueA: 12
desired_result rows over 9 configurations in 3 generations of 4 requests, 7
result rows, and samples/tutorials/tuneup.opentuner.log the duplicate-request
lines driver.py:186-191 printed.  The fixture (tests/golden/
tutorial_request_stream.json, made by make_golden.py tutorial_request_stream
from scalar columns and the log text) is replayed: a scripted bandit hands the
recorded requestor of every request its recorded configuration (the
configuration's BLOCK_SIZE is the value whose Python-2-layout hash_config is
the stored Configuration.hash, tutorial_db_hashes.json), the objective returns
the recorded time, and uptune_amd.driver.SearchDriver runs the generations.
The driver must then reproduce, with no other input:
  * which requests are duplicates, which earlier request each one's result
    comes from (desired_result.result_id), and the OLD / PENDING class the
    reference logged (opentuner/search/driver.py:177-200);
  * the result rows in collection order with was_new_best
    (driver.py:209-225);
  * the bandit's parameters (bandit_info: C = 0.05, window = 500) as the
    build's defaults (bandittechniques.py:20-30).
The CPU test hashes with the oracle's Py2 restatement; the GPU test with the
device's Py2 layout, and checks the device dedup set's verdicts too."""
import json
import os

import pytest

from uptune_amd.driver import SearchDriver
from uptune_amd.manipulator import ConfigurationManipulator, IntegerParameter
from uptune_amd.technique import AUCBanditMetaTechnique, AUCBanditQueue, SearchTechnique


def _fixture(golden_dir):
    fx = json.load(open(os.path.join(golden_dir, "tutorial_request_stream.json")))
    rows = json.load(open(os.path.join(golden_dir, "tutorial_db_hashes.json")))["rows"]
    fx["config"] = {r["id"]: r for r in rows}   # configuration id -> (hash, BLOCK_SIZE)
    return fx


class _Scripted(SearchTechnique):
    """answers with the configurations the tutorial run requested under this name;
    `seen` (GPU test): the device dedup verdict of each request, before it joins
    the history set"""

    def __init__(self, name, sizes, seen=None):
        super().__init__(name=name)
        self.sizes = list(sizes)
        self.seen = seen

    def desired_configuration(self):
        cfg = {"BLOCK_SIZE": self.sizes.pop(0)}
        if self.seen is not None:
            self.seen(cfg)
        return cfg


class _ScriptedBandit(AUCBanditMetaTechnique):
    """AUC bandit whose arm order per request is the recorded requestor (the
    credit assignment still runs on the driver's was_new_best)"""

    def __init__(self, techniques, order, **kw):
        super().__init__(techniques, **kw)
        self.order = list(order)

    def select_technique_order(self):
        return [self.name_to_technique[self.order.pop(0)]]


def _replay(fx, hash_fn, seen=None):
    reqs = fx["desired_result"]
    size = {cid: r["BLOCK_SIZE"] for cid, r in fx["config"].items()}
    arms = fx["bandit_sub_technique"]
    techs = [_Scripted(a, [size[r["configuration_id"]] for r in reqs if r["requestor"] == a], seen) for a in arms]
    root = _ScriptedBandit(techs, [r["requestor"] for r in reqs], name="AUCBanditMetaTechniqueA")
    time_of = {size[r["configuration_id"]]: r["time"] for r in fx["result"]}
    manip = ConfigurationManipulator([IntegerParameter("BLOCK_SIZE", 1, 10)])
    gens = max(r["generation"] for r in reqs) + 1
    drv = SearchDriver(manip, root, parallelism=len(reqs) // gens, hash_fn=hash_fn)
    for _ in range(gens):
        assert drv.run_generation_techniques() == len(reqs) // gens
        drv.run_generation_results(lambda cfg: time_of[cfg["BLOCK_SIZE"]])
        drv.generation += 1
    return drv


def _check(drv, fx):
    reqs, res = fx["desired_result"], fx["result"]
    # the requests: requestor, generation, configuration (Configuration.hash)
    got = drv.requests_query()
    assert len(got) == len(reqs)
    for g, r in zip(got, reqs):
        assert (g.requestor, g.generation) == (r["requestor"], r["generation"])
        assert g.configuration.hash == fx["config"][r["configuration_id"]]["hash"]
        assert g.state == "COMPLETE"
    # the results, in collection order, and the request each one answered
    results = drv.results_query()
    assert [(r.configuration.hash, r.time) for r in results] == \
        [(fx["config"][r["configuration_id"]]["hash"], r["time"]) for r in res]
    assert [int(r.was_new_best) for r in results] == [r["was_new_best"] for r in res]
    assert [g.result.id + 1 for g in got] == [r["result_id"] for r in reqs]
    # duplicates: requests 3, 7, 8, 9, 12 (ids), with the reference's log lines
    first = {}
    dup_ids = []
    for r in reqs:
        if r["configuration_id"] in first:
            dup_ids.append(r["id"])
        first.setdefault(r["configuration_id"], r["id"])
    assert dup_ids == [3, 7, 8, 9, 12]
    want = [(d["test_count"], d["requestor"], d["first_requestor"], d["class"]) for d in fx["log_duplicates"]]
    assert list(drv.duplicate_log) == want and drv.duplicate_count == len(want)
    assert drv.best_result.time == min(r["time"] for r in res)


def test_bandit_defaults_equal_tutorial_bandit_info(golden_dir):
    fx = _fixture(golden_dir)
    q = AUCBanditQueue(fx["bandit_sub_technique"])
    assert (q.C, q.window) == (fx["bandit_info"]["c"], fx["bandit_info"]["window"])
    assert fx["bandit_sub_technique"] == ["DifferentialEvolutionAlt", "UniformGreedyMutation", "NormalGreedyMutation",
                                          "RandomNelderMead"]


def test_request_stream_replay_cpu(golden_dir):
    """driver semantics with the oracle's Py2-layout hash_config"""
    from oracle import hashing as oh
    from oracle.space import INT, Param
    space = [Param("BLOCK_SIZE", INT, 1, 10)]
    fx = _fixture(golden_dir)
    drv = _replay(fx, lambda cfg: oh.hash_config(space, [cfg["BLOCK_SIZE"]], py2=True))
    _check(drv, fx)


@pytest.mark.gpu
def test_request_stream_replay_gpu(golden_dir):
    """the same replay keyed by the device's Py2-layout hash_config, and the
    device history set's dedup verdict of every request (checked against the
    requests the reference found duplicate)"""
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from uptune_amd.engine import BatchEngine, hex_to_digests
    fx = _fixture(golden_dir)
    eng = BatchEngine(ConfigurationManipulator([IntegerParameter("BLOCK_SIZE", 1, 10)]), device=0, py2_layout=True)
    eng.history_reset(0)
    verdicts = []

    def seen(cfg):
        h = eng.hash_configs([cfg])
        d = torch.from_numpy(hex_to_digests(h).view("int32").copy()).cuda()
        verdicts.append(bool(eng.dedup(d).cpu()[0]))
        eng.history_add(d)

    drv = _replay(fx, lambda cfg: eng.hash_configs([cfg])[0], seen)
    _check(drv, fx)
    assert [i + 1 for i, v in enumerate(verdicts) if v] == [3, 7, 8, 9, 12]
