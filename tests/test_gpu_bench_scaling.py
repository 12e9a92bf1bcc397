"""bench.py's multi-rank path, as the driver's scaling run will launch it
(`bench.py --gpus N`), rehearsed on one GPU with gloo records
(UT_DIST_BACKEND=gloo: N rank processes share cuda:0; the merge still runs
as the HIP kernel):

  * --scaling strong: the global pool is fixed, rank r scores
    [r*M/N, (r+1)*M/N).  The 8-rank line selects exactly what the 1-rank
    line selects (equal `selection_sha` of the last timed round's merged
    (index, digest) list, and of the score-determined parity round's) and both pass the oracle parity block -- SURVEY.md
    §8(e)'s "the same top-k at 1/2/4/8 GPUs", checked on the bench's own
    output (the analog of the reference's parallel_factor instances that
    exchange results every round, python/uptune/api.py:400-401,547-553);
  * --scaling weak: a 2-rank line with m per rank equals the 1-rank line
    with 2m;
  * each rank caches inner digests for its own shard's DE targets only, so
    an 8-rank strong line holds less device memory per rank than 1 rank.
"""
import json
import os
import subprocess
import sys

import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(*args, timeout=420):
    env = dict(os.environ, UT_DIST_BACKEND="gloo")
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "2", "--warmup", "1", "--no-cpu-baseline",
           "--parity-sample", "2048", *args]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, (cmd, r.stdout[-2000:], r.stderr[-4000:])
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    return json.loads(lines[0])


@pytest.mark.timeout(900)
def test_strong_scaling_selections_equal_at_1_and_8_ranks():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    M = 1 << 16
    one = _bench("--gpus", "1", "--scaling", "strong", "--m", str(M))
    eight = _bench("--gpus", "8", "--scaling", "strong", "--m", str(M))
    assert one["world"] == 1 and eight["world"] == 8
    assert one["scaling"] == eight["scaling"] == "strong"
    assert one["config"]["global_pool"] == eight["config"]["global_pool"] == M
    assert eight["config"]["candidates_per_gpu"] == M // 8
    assert one["parity"]["all_ok"] and eight["parity"]["all_ok"], (one["parity"], eight["parity"])
    assert one["selection_sha"] == eight["selection_sha"]
    # the score-determined round (ell = 2: every selected score distinct), so the
    # equal shas check the cross-rank score merge, not only the index tie-break
    sd1, sd8 = one["parity"]["score_determined"], eight["parity"]["score_determined"]
    assert sd1["distinct_selected_scores"] == sd8["distinct_selected_scores"] == 256
    assert sd1["selection_sha"] == sd8["selection_sha"]
    # the shard-local inner-digest cache: an eighth of the pool's targets per rank
    assert 0 < eight["hbm_bytes_per_rank"] < one["hbm_bytes_per_rank"]


@pytest.mark.timeout(900)
def test_weak_scaling_line_equals_one_rank_with_the_whole_pool():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    m = 1 << 15
    two = _bench("--gpus", "2", "--m", str(m))
    one = _bench("--gpus", "1", "--m", str(2 * m))
    assert two["scaling"] == "weak" and two["world"] == 2
    assert two["config"]["global_pool"] == one["config"]["global_pool"] == 2 * m
    assert two["parity"]["all_ok"] and one["parity"]["all_ok"]
    assert two["selection_sha"] == one["selection_sha"]
    assert two["parity"]["score_determined"]["selection_sha"] == one["parity"]["score_determined"]["selection_sha"]
