"""The RCCL ("nccl" backend) path of uptune_amd.dist with DEVICE tensors:
on an RCCL group every exchange goes through libuthot's own communicator
(ut_comm_*, bootstrapped over the torch group) and the HIP merge kernel.

The one-GPU boxes cannot run two RCCL ranks (RCCL refuses two ranks on one
device), so this runs the nccl code paths at world size 1 in a spawned
process: allgather_topk / allgather_selection / broadcast_results / agree
move cuda tensors through RCCL collectives, and a DistributedSearchDriver
generation loop over the GPU bandit runs on the nccl group.  The world-2
semantics are covered by the gloo tests (tests/test_dist_cpu.py,
tests/test_dist_driver_cpu.py, tests/test_tuning_manager_cpu.py,
tests/test_gpu_c5.py)."""
import os
import socket

import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(port, q):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    out = {}
    try:
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
        out["backend"] = dist.get_backend()
        from uptune_amd.dist import allgather_selection, allgather_topk, broadcast_results
        from uptune_amd.driver import agree
        idx = torch.tensor([5, 2, -1, 9], dtype=torch.int64, device=dev)
        sc = torch.tensor([3.0, 7.0, float("-inf"), 7.0], dtype=torch.float64, device=dev)
        dig = torch.arange(32, dtype=torch.int32, device=dev).reshape(4, 8)
        mi, ms, md, _ = allgather_topk(idx, sc, dig, 4)
        from uptune_amd import dist as D
        out["via"] = sorted(type(c).__name__ for c in D._COMMS.values())
        out["topk"] = (mi.device.type, mi.cpu().tolist(), ms.cpu().tolist())
        # an allocation failure while the record buffers grow (rows: wider
        # records) returns UT_ENOMEM after the ranks' vote, not a hang inside
        # the all-gather; the next call allocates and succeeds
        comm = list(D._COMMS.values())[0]
        comm.lib.ut_debug_fail_alloc(comm.ctx, 1)
        try:
            allgather_topk(idx, sc, dig, 4, rows=torch.ones((3, 4), dtype=torch.float64, device=dev))
            out["enomem"] = "no error"
        except Exception as ex:
            out["enomem"] = str(ex)
        comm.lib.ut_debug_fail_alloc(comm.ctx, 0)
        rows = torch.arange(12, dtype=torch.float64, device=dev).reshape(3, 4)
        si, ss, sr, sd = allgather_selection(idx, sc, dig, rows, 4, with_digests=True)
        out["sel"] = (si.cpu().tolist(), sr.device.type, sr.cpu().tolist(), sd.shape[0])
        y, d = broadcast_results(torch.tensor([1.5, 2.5], dtype=torch.float64), dig[:2].cpu(), 2, dev)
        out["bcast"] = (y.device.type, y.cpu().tolist(), d.cpu().tolist() == dig[:2].cpu().tolist())
        out["agree"] = (agree(True, None, dev), agree(False, None, dev))
        # a short SPMD search loop on the nccl group (rank 0 evaluates, results broadcast over RCCL)
        from uptune_amd import technique as T
        from uptune_amd.driver import DistributedSearchDriver
        from uptune_amd.manipulator import ConfigurationManipulator, FloatParameter
        m = ConfigurationManipulator([FloatParameter("x%d" % i, -2.0, 2.0) for i in range(6)])
        meta = T.pso_ga_de_bandit(bandit_seed=1, pool=2048, batch=4, population=256, seed=1, lengthscale=0.5)
        drv = DistributedSearchDriver(m, meta, parallelism=4, device=dev)

        def f(c):
            return sum((c["x%d" % i] - 0.5) ** 2 for i in range(6))
        drv.main(f, test_limit=40)
        out["loop"] = (drv.test_count, len(drv.results_query()), drv.best_result.time)
        D.release_comms()
        dist.destroy_process_group()
    except Exception as ex:  # reported to the parent
        out["error"] = repr(ex)
    q.put(out)


def test_rccl_collectives_and_loop_world1():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_worker, args=(_port(), q))
    p.start()
    out = q.get(timeout=150)
    p.join(timeout=60)
    assert "error" not in out, out.get("error")
    assert out["backend"] == "nccl"
    assert out["via"] == ["DeviceComm"]       # the C-ABI communicator carried the exchange
    dev, mi, ms = out["topk"]
    assert dev == "cuda" and mi == [2, 9, 5, -1] and ms[:3] == [7.0, 7.0, 3.0]
    si, rdev, rows, nd = out["sel"]
    assert si == [2, 9, 5, -1] and rdev == "cuda" and nd == 4
    assert rows[0][:3] == [1.0, 3.0, 0.0]
    bdev, y, same = out["bcast"]
    assert bdev == "cuda" and y == [1.5, 2.5] and same
    assert out["agree"] == (True, False)
    assert "UT_ENOMEM" in out["enomem"] and "no memory for the records" in out["enomem"], out["enomem"]
    tc, nres, best = out["loop"]
    assert tc > 40 and 0.8 * tc <= nres <= tc and best < 6 * 2.5 ** 2
