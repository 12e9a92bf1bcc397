"""The multi-GPU exchange on the device (uptune_amd/csrc/comm.hip through
uptune_amd/dist.py):

  * the HIP merge kernel (ut_topk_merge) equals the merge's definition
    (dist.merge_topk, and a plain-Python restatement) on random pools with
    score ties, empty slots, NaN scores, digest collisions and value rows;
  * libuthot's own RCCL communicator (ut_comm_*) at world size 1 -- the only
    RCCL world a one-GPU box allows (RCCL refuses two ranks on one device);
  * bench-style rounds (DE round -> local top-k -> exchange -> the MERGED
    selections join every rank's history) at world 1 and world 2 (gloo
    records, merge on the device, both ranks on cuda:0) select the same
    candidates with the same dup masks in every round on a discrete space
    where later rounds' dup masks depend on the history -- the contract that
    the same top-k comes out at 1/2/4/8 GPUs (python/uptune/api.py:547-553
    exchanges results between parallel instances each round).
"""
import os
import socket

import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _py_merge(sc, idx, dg, k):
    """the definition: drop empty / NaN slots, keep the smallest index of each
    digest, order by (-score, index), pad with -1"""
    best = {}
    for j in range(len(idx)):
        if idx[j] < 0 or sc[j] != sc[j]:
            continue
        key = tuple(dg[j])
        if key not in best or idx[j] < idx[best[key]]:
            best[key] = j
    rows = sorted(best.values(), key=lambda j: (-sc[j], idx[j]))[:k]
    return rows


def test_topk_merge_kernel_vs_definition():
    _need_gpu()
    from uptune_amd.dist import device_ctx, merge_topk
    c = device_ctx(torch.device("cuda", 0))
    rng = np.random.default_rng(11)
    for trial in range(60):
        R, k = int(rng.integers(1, 9)), int(rng.integers(1, 300))
        n = R * k
        idx = rng.choice(10 * n + 10, size=n, replace=False).astype(np.int64)
        idx[rng.random(n) < 0.2] = -1
        sc = rng.choice([0.1, 0.5, 0.9, -1.5, float("-inf"), float("nan")], size=n, p=[.3, .2, .2, .2, .05, .05])
        dg = rng.integers(0, 6, size=(n, 8)).astype(np.int32)          # collisions on purpose
        if trial % 2:
            dg[:, 1:] = dg[:, :1]
        ncols = int(rng.integers(0, 4))
        rows = rng.standard_normal((ncols, n)) if ncols else None
        dev = torch.device("cuda", 0)
        oi, os_, od, orow = c.topk_merge(torch.from_numpy(idx).to(dev), torch.from_numpy(sc).to(dev),
                                         torch.from_numpy(dg).to(dev), k,
                                         rows=None if rows is None else torch.from_numpy(rows).to(dev))
        sel = _py_merge(sc, idx, dg, k)
        want_i = [int(idx[j]) for j in sel] + [-1] * (k - len(sel))
        want_s = [float(sc[j]) for j in sel] + [float("-inf")] * (k - len(sel))
        assert oi.cpu().tolist() == want_i, trial
        assert os_.cpu().tolist() == want_s, trial
        want_d = np.zeros((k, 8), np.int32)
        want_d[:len(sel)] = dg[sel]
        np.testing.assert_array_equal(od.cpu().numpy(), want_d)
        if ncols:
            want_r = np.zeros((ncols, k))
            want_r[:, :len(sel)] = rows[:, sel]
            np.testing.assert_array_equal(orow.cpu().numpy(), want_r)
        # the torch definition (the CPU test double) agrees
        ti, ts = merge_topk(torch.from_numpy(sc), torch.from_numpy(idx), torch.from_numpy(dg), k)
        assert ti.tolist() == want_i


def test_topk_merge_edges():
    _need_gpu()
    from uptune_amd import _lib as L
    from uptune_amd.dist import device_ctx
    c = device_ctx(torch.device("cuda", 0))
    dev = torch.device("cuda", 0)
    e64 = torch.empty(0, dtype=torch.int64, device=dev)
    oi, os_, od, _ = c.topk_merge(e64, torch.empty(0, dtype=torch.float64, device=dev),
                                  torch.empty((0, 8), dtype=torch.int32, device=dev), 5)
    assert oi.cpu().tolist() == [-1] * 5 and os_.cpu().tolist() == [float("-inf")] * 5
    assert int(od.abs().sum()) == 0
    with pytest.raises(L.UthotError):   # k out of range fails loudly
        c.topk_merge(e64, torch.empty(0, dtype=torch.float64, device=dev),
                     torch.empty((0, 8), dtype=torch.int32, device=dev), 0)


def test_rccl_c_abi_world1():
    """ut_comm_init / allgather_topk / bcast_results / allreduce / barrier over
    a one-rank RCCL communicator driven through the C ABI (no torch.distributed)"""
    _need_gpu()
    from uptune_amd import _lib as L
    from uptune_amd.dist import DeviceComm
    dev = torch.device("cuda", 0)
    comm = DeviceComm(dev, 0, 1, DeviceComm.unique_id())
    try:
        k = 6
        idx = torch.tensor([4, 9, -1, 2, 7, 11], dtype=torch.int64, device=dev)
        sc = torch.tensor([0.5, 0.9, 3.0, 0.9, float("nan"), 0.1], dtype=torch.float64, device=dev)
        dg = torch.arange(48, dtype=torch.int32, device=dev).reshape(6, 8)
        dg[5] = dg[0]                                   # 11 repeats 4's configuration
        rows = torch.arange(12, dtype=torch.float64, device=dev).reshape(2, 6)
        oi, os_, od, orow = comm.allgather_topk(idx, sc, dg, k, rows=rows)
        assert oi.cpu().tolist() == [2, 9, 4, -1, -1, -1]
        assert os_.cpu().tolist()[:3] == [0.9, 0.9, 0.5]
        assert od[0].cpu().tolist() == dg[3].cpu().tolist() and int(od[3:].abs().sum()) == 0
        assert orow.cpu().tolist() == [[3.0, 1.0, 0.0, 0, 0, 0], [9.0, 7.0, 6.0, 0, 0, 0]]
        y, d = comm.bcast_results(torch.tensor([1.5, 2.5], dtype=torch.float64), dg[:2], 2, src=0)
        assert y.cpu().tolist() == [1.5, 2.5] and torch.equal(d, dg[:2])
        y, d = comm.bcast_results(torch.zeros(0, dtype=torch.float64), dg[:0], 0, src=0)
        assert y.numel() == 0 and d.shape == (0, 8)
        # a source whose rows do not match n enters the collective with the
        # failure sentinel and raises (no rank is left waiting), and the
        # communicator stays usable
        with pytest.raises(L.UthotError):
            comm.bcast_results(torch.tensor([1.5, 2.5], dtype=torch.float64), dg[:2], 3, src=0)
        y, d = comm.bcast_results(torch.tensor([4.5], dtype=torch.float64), dg[:1], 1, src=0)
        assert y.cpu().tolist() == [4.5] and torch.equal(d, dg[:1])
        t = torch.tensor([3.0, -1.0], dtype=torch.float64, device=dev)
        assert comm.allreduce_(t, L.UT_RED_MAX).cpu().tolist() == [3.0, -1.0]
        assert comm.agree(True) and not comm.agree(False)
        comm.barrier()
        r, w = torch.zeros(1, dtype=torch.int32), torch.zeros(1, dtype=torch.int32)
        import ctypes as C
        a, b = C.c_int32(), C.c_int32()
        L.check(comm.ctx, comm.lib.ut_comm_info(comm.ctx, C.byref(a), C.byref(b)), "ut_comm_info")
        assert (a.value, b.value) == (0, 1)
    finally:
        comm.close()


# ---------------------------------------------------------------------------
# bench-style rounds: rank-invariant selections and dup masks
# ---------------------------------------------------------------------------
M_PER_RANK, K, ROUNDS, SEED = 1536, 48, 4, 21


def _manip():
    from uptune_amd.manipulator import ConfigurationManipulator, EnumParameter, IntegerParameter
    # 4^5 * 3 = 3072 configurations: a round's pool repeats itself and the
    # history, so the dup masks of later rounds depend on earlier selections
    return ConfigurationManipulator([IntegerParameter("i%d" % j, 0, 3) for j in range(5)] +
                                    [EnumParameter("e", ["a", "b", "c"])])


def _rounds(rank, world, exchange):
    """ROUNDS DE rounds of the bench loop on this rank's shard; the merged
    selections join the history.  -> per round (merged idx, merged digests,
    this shard's dup mask)"""
    from uptune_amd.engine import BatchEngine
    eng = BatchEngine(_manip(), device=0, seed=SEED)
    m = M_PER_RANK
    npop = m * 2                     # the same population at every world size
    eng.population_init(npop)
    tr = eng.population_get()[:, :200]
    X = eng.encode(tr).T.contiguous().cpu().numpy()
    y = np.sum((X - 0.3) ** 2, axis=1)
    eng.history_reset(4096)
    eng.history_add(eng.hash(tr))
    out = []
    acq = eng.acq("ei")
    for r in range(ROUNDS):
        eng.gp_fit(X, y, lengthscale=0.8, sigma_f2=1.0, sigma_n2=1e-6, jitter=1e-8)
        for part in range(2 // world):         # world 1 scores both halves of the pool
            base = (rank + part) * m
            vals = eng.propose_de(m, round_=r, cand_base=base, cr=0.5)
            dig = eng.hash_de(vals, base)
            dup = eng.dedup(dig)
            _, _, score = eng.gp_score_values(vals, acq=acq, dup=dup)
            i, s = eng.topk(score, K, dup=dup, cand_base=base)
            loc = torch.where(i >= 0, i - base, torch.zeros_like(i))
            sd = torch.where((i >= 0).unsqueeze(1), dig[loc], torch.zeros_like(dig[loc]))
            if part == 0:
                li, ls, ld, masks = i, s, sd, [dup.cpu().numpy()]
            else:   # world 1: the two halves merged on the device, as two ranks would
                from uptune_amd.dist import device_ctx
                li, ls, ld, _ = device_ctx(eng.device).topk_merge(torch.cat([li, i]), torch.cat([ls, s]),
                                                                  torch.cat([ld, sd]), K)
                masks.append(dup.cpu().numpy())
        mi, ms, md = exchange(li, ls, ld) if world > 1 else (li, ls, ld)
        eng.history_add(md)
        out.append((mi.cpu().tolist(), md.cpu().numpy().tolist(), np.concatenate(masks).tolist()))
    eng.close()
    return out


def _worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from uptune_amd.dist import allgather_topk

    def ex(i, s, d):
        a, b, c, _ = allgather_topk(i, s, d, K)
        return a, b, c
    try:
        q.put((rank, _rounds(rank, world, ex)))
    finally:
        dist.destroy_process_group()


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_bench_rounds_rank_invariant():
    _need_gpu()
    import torch.multiprocessing as mp
    one = _rounds(0, 1, None)
    # the history matters: later rounds have duplicates of earlier selections
    assert sum(sum(r[2]) for r in one) > 0
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    out = sorted((q.get(timeout=240) for _ in range(2)), key=lambda t: t[0])
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in range(ROUNDS):
        # same merged selection and digests on both ranks and at world 1
        assert out[0][1][r][0] == out[1][1][r][0] == one[r][0], r
        assert out[0][1][r][1] == out[1][1][r][1] == one[r][1], r
        # the two shards' dup masks = the world-1 pool's mask
        assert out[0][1][r][2] + out[1][1][r][2] == one[r][2], r
