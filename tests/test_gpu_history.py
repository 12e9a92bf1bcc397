"""Device dedup against ingested history: the
reference's results DB, GlobalResult DB, archive CSV and pending configs all
land in the GPU history set.  Needs a GPU."""
import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

from oracle import hashing as oh  # noqa: E402
from oracle.space import INT, Param  # noqa: E402


def _engine(manip, py2=False, seed=0):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from uptune_amd.engine import BatchEngine
    return BatchEngine(manip, device=0, seed=seed, py2_layout=py2)


def test_resume_from_opentuner_db(golden_dir):
    """tutorial DB (OpenTuner layout): BLOCK_SIZE configs with a Result are seen"""
    from uptune_amd import history as H
    from uptune_amd.manipulator import ConfigurationManipulator, IntegerParameter
    rows = json.load(open(os.path.join(golden_dir, "tutorial_db_hashes.json")))["rows"]
    db = os.path.join(golden_dir, "tutorial_opentuner.db")
    e = _engine(ConfigurationManipulator([IntegerParameter("BLOCK_SIZE", 1, 10)]), py2=True)
    e.history_reset(0)
    assert H.ingest_history(e, opentuner_db=db) == 7
    with_result = set(H.opentuner_result_hashes(db))
    by_hash = {r["hash"]: r["BLOCK_SIZE"] for r in rows}
    seen_sizes = {by_hash[h] for h in with_result}
    cfgs = [{"BLOCK_SIZE": b} for b in range(1, 11)]
    assert e.hash_configs([{"BLOCK_SIZE": r["BLOCK_SIZE"]} for r in rows]) == [r["hash"] for r in rows]
    assert H.seen_mask(e, cfgs) == [b in seen_sizes for b in range(1, 11)]


def test_archive_and_pending(golden_dir):
    from uptune_amd import history as H
    from uptune_amd import schema as S
    tokens = [["IntegerParameter", "x", [2, 15]], ["IntegerParameter", "y", [2, 12]],
              ["IntegerParameter", "a", [2, 15]], ["IntegerParameter", "b", [2, 12]]]
    e = _engine(S.create_params(tokens))
    arch = H.read_archive(os.path.join(golden_dir, "causal_archive.csv"), e.spec)
    space = [Param(n, INT, lo, hi) for _, n, (lo, hi) in tokens]
    # device digests of the archive rows == hash_config restated
    assert e.hash_configs(arch) == [oh.hash_config(space, [c[p.name] for p in space]) for c in arch]
    pending = [{"x": 3, "y": 3, "a": 3, "b": 3}]
    e.history_reset(0)
    n = H.ingest_history(e, archive_csv=os.path.join(golden_dir, "causal_archive.csv"), pending=pending)
    assert n == 51
    fresh = [{"x": 15, "y": 12, "a": 15, "b": 12}, {"x": 2, "y": 2, "a": 2, "b": 2}]
    fresh = [c for c in fresh if c not in arch]
    probe = arch[:10] + pending + fresh + fresh[:1]
    want = [True] * 11 + [False] * len(fresh) + [True]   # the repeat of fresh[0] is an in-batch duplicate
    assert H.seen_mask(e, probe) == want
