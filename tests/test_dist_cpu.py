"""World-size-2 gloo run of the multi-GPU exchange (uptune_amd/dist.py):
sharded local top-k -> all_gather -> merge equals the single-pool top-k,
including cross-shard duplicate digests and score ties; history broadcast."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import select as osel


def _pool(m=4000, seed=0):
    rng = np.random.default_rng(seed)
    scores = np.round(rng.standard_normal(m), 1)          # heavy ties
    dig = rng.integers(0, 2**31, size=(m, 8), dtype=np.int64).astype(np.int32)
    # plant duplicates: later candidates repeat earlier configs (same digest, same score)
    for a, b in [(5, 3100), (17, 2500), (2600, 3999), (100, 101)]:
        dig[b] = dig[a]
        scores[b] = scores[a]
    scores[::53] = np.nan
    return scores, dig


def _global_ref(scores, dig, k):
    hexes = [row.tobytes() for row in dig]
    dup = osel.dedup(hexes, set())
    return osel.topk(list(scores), k, dup=dup)


def _worker(rank, world, port, k, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from uptune_amd.dist import allgather_topk, broadcast_history
    scores, dig = _pool()
    m = len(scores)
    lo, hi = rank * m // world, (rank + 1) * m // world
    # local shard: in-shard dedup + local top-k (what ut_score_round_* returns)
    hexes = [row.tobytes() for row in dig[lo:hi]]
    dup = osel.dedup(hexes, set())
    loc = osel.topk(list(scores[lo:hi]), k, dup=dup, cand_base=lo)
    li = torch.tensor(loc, dtype=torch.int64)
    ls = torch.tensor([scores[g] if g >= 0 else float("-inf") for g in loc], dtype=torch.float64)
    ld = torch.tensor(np.stack([dig[g] if g >= 0 else np.zeros(8, np.int32) for g in loc]), dtype=torch.int32)
    gi, gs, gd, _ = allgather_topk(li, ls, ld, k)
    # the merged digests are the selected candidates' (zero for empty slots)
    assert all((gd[j].numpy() == (dig[g] if g >= 0 else 0)).all() for j, g in enumerate(gi.tolist()))
    X = torch.arange(12, dtype=torch.float64).reshape(3, 4) if rank == 0 else None
    y = torch.tensor([1.0, 2.0, 3.0]) if rank == 0 else None
    dd = torch.arange(24, dtype=torch.int32).reshape(3, 8) if rank == 0 else None
    X, y, dd = broadcast_history(X, y, dd, 3, 4, "cpu")
    q.put((rank, gi.tolist(), float(X.sum()), float(y.sum()), int(dd.sum())))
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("world,k", [(2, 64), (2, 7), (4, 32)])
def test_sharded_topk_equals_global(world, k):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, k, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    scores, dig = _pool()
    want = _global_ref(scores, dig, k)
    for rank, got, xs, ys, ds in res:
        assert got == want
        assert (xs, ys, ds) == (66.0, 6.0, 276)


def test_merge_topk_unit():
    from uptune_amd.dist import merge_topk
    s = torch.tensor([0.9, 0.5, 0.9, 0.7, float("-inf")], dtype=torch.float64)
    i = torch.tensor([7, 3, 2, 9, -1])
    d = torch.tensor([[1] * 8, [2] * 8, [3] * 8, [1] * 8, [0] * 8], dtype=torch.int32)
    gi, gs = merge_topk(s, i, d, 4)
    # digest [1]*8 appears as idx 7 and 9 -> 7 survives
    assert gi.tolist() == [2, 7, 3, -1]


def _sel_worker(rank, world, port, k, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from uptune_amd.dist import allgather_selection, broadcast_results
    scores, dig = _pool()
    m = len(scores)
    lo, hi = rank * m // world, (rank + 1) * m // world
    values = np.arange(3 * m, dtype=np.float64).reshape(3, m)   # row j of candidate g = j*m + g
    hexes = [row.tobytes() for row in dig[lo:hi]]
    dup = osel.dedup(hexes, set())
    loc = osel.topk(list(scores[lo:hi]), k, dup=dup, cand_base=lo)
    li = torch.tensor(loc, dtype=torch.int64)
    ls = torch.tensor([scores[g] if g >= 0 else float("-inf") for g in loc], dtype=torch.float64)
    ld = torch.tensor(np.stack([dig[g] if g >= 0 else np.zeros(8, np.int32) for g in loc]), dtype=torch.int32)
    rows = torch.tensor(np.stack([values[:, g] if g >= 0 else np.zeros(3) for g in loc], axis=1))
    gi, gs, grows = allgather_selection(li, ls, ld, rows, k)
    y = torch.tensor([0.5, 1.5]) if rank == 0 else None
    d = torch.arange(16, dtype=torch.int32).reshape(2, 8) if rank == 0 else None
    y, d = broadcast_results(y, d, 2, torch.device("cpu"))
    q.put((rank, gi.tolist(), grows.numpy().tolist(), float(y.sum()), int(d.sum())))
    dist.destroy_process_group()


def test_allgather_selection_rows_and_results_broadcast():
    k, world = 40, 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_sel_worker, args=(r, world, port, k, q)) for r in range(world)]
    for p in ps:
        p.start()
    out = sorted(q.get(timeout=120) for _ in range(world))
    for p in ps:
        p.join(timeout=60)
    scores, dig = _pool()
    want = _global_ref(scores, dig, k)
    m = len(scores)
    for rank, gi, rows, ysum, dsum in out:
        assert gi == want
        # every rank gets the selected candidates' value rows, in merged order
        assert rows == [[j * m + g for g in want] for j in range(3)]
        assert ysum == 2.0 and dsum == sum(range(16))


def test_merge_topk_random_vs_python():
    """the fixed-size merge equals the plain definition: drop empty slots, keep
    the smallest index of each digest, order by (-score, index), pad with -1"""
    from uptune_amd.dist import merge_topk
    rng = np.random.default_rng(5)
    for trial in range(50):
        R, k = int(rng.integers(1, 9)), int(rng.integers(1, 12))
        n = R * k
        idx = rng.choice(10 * n, size=n, replace=False).astype(np.int64)
        idx[rng.random(n) < 0.2] = -1
        sc = rng.choice([0.1, 0.5, 0.9, float("-inf")], size=n)        # ties on purpose
        dg = rng.integers(0, 4, size=(n, 8)).astype(np.int32)          # collisions on purpose
        dg[:, 1:] = dg[:, :1]
        best = {}
        for j in range(n):
            if idx[j] < 0:
                continue
            key = tuple(dg[j])
            if key not in best or idx[j] < idx[best[key]]:
                best[key] = j
        rows = sorted(best.values(), key=lambda j: (-sc[j], idx[j]))[:k]
        want_i = [int(idx[j]) for j in rows] + [-1] * (k - len(rows))
        want_s = [float(sc[j]) for j in rows] + [float("-inf")] * (k - len(rows))
        gi, gs = merge_topk(torch.from_numpy(sc), torch.from_numpy(idx), torch.from_numpy(dg), k)
        assert gi.tolist() == want_i, trial
        assert gs.tolist() == want_s, trial


def _enomem_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from uptune_amd import dist as D
    out = {}
    idx = torch.arange(4, dtype=torch.int64) + 10 * rank
    sc = torch.tensor([4.0, 3.0, 2.0, 1.0], dtype=torch.float64) + rank
    dig = (torch.arange(32, dtype=torch.int32) + 100 * rank).reshape(4, 8)
    if rank == 1:
        D._FAIL_NEXT_ALLOC = 1          # this rank's receive buffers fail once
    try:
        D.allgather_topk(idx, sc, dig, 4)
        out["first"] = "no error"
    except Exception as ex:
        out["first"] = str(ex)
    # the next exchange succeeds on both ranks (no rank was left in a collective)
    mi, ms = D.allgather_topk(idx, sc, dig, 4)[:2]
    out["second"] = mi.tolist()
    dist.destroy_process_group()
    q.put((rank, out))


def test_allgather_allocation_failure_on_one_rank_returns_enomem_on_both():
    """VERDICT r5 #7 on the gloo exchange: an allocation failure injected on
    rank 1 makes BOTH ranks raise UT_ENOMEM (the agreement before the
    all_gather), no rank hangs, and the next exchange works"""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_enomem_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in ps:
        p.join(timeout=60)
    assert "UT_ENOMEM" in res[1]["first"] and "no memory for the records" in res[1]["first"], res
    assert "UT_ENOMEM" in res[0]["first"] and "another rank" in res[0]["first"], res
    assert res[0]["second"] == res[1]["second"] == [10, 0, 11, 1], res   # (-score, index) order
