"""Multi-GPU exchange for the scoring round (one process per GPU).

SURVEY.md §8(e): the candidate pool is sharded by GLOBAL candidate index
(rank r owns [r*m, (r+1)*m)); population, training set, GP factor and history
are replicated.  Two real exchanges exist per round:

  * all-gather of every rank's local top-k records (score, index, digest,
    optionally the selected value rows) and a deterministic merge --
    cross-shard duplicates (equal digests) keep the smallest global index,
    ties on score break by the smallest index, so the merged top-k is
    identical to the single-GPU result for the same pool;
  * broadcast from the evaluating rank of the per-round history delta
    (objective values and digests) -- the analog of the reference's per-round
    api.sync result injection (python/uptune/api.py:547-553,
    opentuner/api.py:87-104).

Device path (the product): libuthot's C ABI drives RCCL itself
(`ut_comm_*`, csrc/comm.hip) on a communicator bootstrapped over the
torch.distributed group (one 128-byte id broadcast), and the merge is the HIP
kernel `ut_topk_merge`.  torch.distributed carries only that id and the
host-side control (barriers, the CPU test double).

CPU test double: with the "gloo" backend the records travel as CPU tensors
through torch.distributed; the merge then runs as the HIP kernel when the
tensors live on a GPU (the 1-GPU multi-rank rehearsal) and as `merge_topk`
(plain torch, the kernel's definition) only for CPU tensors -- the
world-size-2 tests in tests/test_dist_*.py.
"""
from __future__ import annotations

import ctypes as C
from typing import Dict, Optional, Tuple

import torch
import torch.distributed as dist

from . import _lib as L


# ---------------------------------------------------------------------------
# the merge: torch definition (CPU test double) and the HIP kernel
# ---------------------------------------------------------------------------
def merge_topk(scores: torch.Tensor, idx: torch.Tensor, digests: torch.Tensor, k: int, return_pos: bool = False):
    """Merge gathered local top-k lists (the definition ut_topk_merge implements).

    scores [R*k] f64, idx [R*k] i64 (-1 = empty slot), digests [R*k][8] i32.
    Returns (idx [k], score [k]) sorted by (-score, idx), empty slots -1 /
    -inf (+ the input position of each output slot, 0 for empty slots, with
    return_pos=True).  Cross-shard duplicates (equal digests) keep the
    smallest global index; NaN scores count as empty (the local top-k never
    selects them).

    Fixed-size tensor ops only -- no boolean indexing, no .item().
    """
    n = idx.numel()
    dev = idx.device
    big = torch.iinfo(torch.int64).max
    valid = (idx >= 0) & ~torch.isnan(scores)
    key = torch.where(valid, idx, torch.full_like(idx, big))
    d64 = digests.to(torch.int32).contiguous().view(n, 8).view(torch.int64)      # [n][4]
    # lexicographic (digest, index) order by stable sorts, least significant first
    o = torch.argsort(key, stable=True)
    for c in (3, 2, 1, 0):
        o = o[torch.argsort(d64[o, c], stable=True)]
    ds, vs = d64[o], valid[o]
    dup = torch.zeros(n, dtype=torch.bool, device=dev)
    if n > 1:   # a valid record equal to its predecessor: a later (larger-index) copy
        dup[1:] = (ds[1:] == ds[:-1]).all(dim=1) & vs[1:] & vs[:-1]
    keep = torch.empty_like(vs)
    keep[o] = vs & ~dup
    s = torch.where(keep, scores, torch.full_like(scores, float("-inf")))
    i = torch.where(keep, idx, torch.full_like(idx, big))
    # (-score, idx) order: stable by index, then stable by descending score
    o = torch.argsort(i, stable=True)
    o = o[torch.argsort(-s[o], stable=True)]
    top = o[:k]
    out_i = torch.where(keep[top], idx[top], torch.full_like(idx[top], -1))
    out_s = torch.where(keep[top], scores[top], torch.full_like(scores[top], float("-inf")))
    pos = torch.where(keep[top], top, torch.zeros_like(top))
    if out_i.numel() < k:
        pad = k - out_i.numel()
        out_i = torch.cat([out_i, torch.full((pad,), -1, dtype=idx.dtype, device=dev)])
        out_s = torch.cat([out_s, torch.full((pad,), float("-inf"), dtype=scores.dtype, device=dev)])
        pos = torch.cat([pos, torch.zeros((pad,), dtype=pos.dtype, device=dev)])
    return (out_i, out_s, pos) if return_pos else (out_i, out_s)


def _ptr(t: Optional[torch.Tensor]):
    return None if t is None else C.c_void_p(t.data_ptr())


class DeviceCtx:
    """A libuthot context on one GPU, bound to torch's current stream there
    (so its kernels and collectives are ordered with the engine's and torch's
    work).  Runs the merge kernel; DeviceComm adds the RCCL communicator."""

    def __init__(self, device):
        self.lib = L.lib()
        if not torch.cuda.is_available():
            raise L.UthotError("uptune_amd.dist device path needs a ROCm GPU")
        self.device = torch.device(device) if not isinstance(device, torch.device) else device
        if self.device.index is None:
            self.device = torch.device("cuda", torch.cuda.current_device())
        ctx = C.c_void_p()
        L.check(None, self.lib.ut_ctx_create(self.device.index, 0, C.byref(ctx)), "ut_ctx_create")
        self.ctx = ctx
        s = torch.cuda.current_stream(self.device)
        L.check(self.ctx, self.lib.ut_set_stream(self.ctx, C.c_void_p(s.cuda_stream)), "ut_set_stream")

    def close(self):
        if getattr(self, "ctx", None):
            self.lib.ut_ctx_destroy(self.ctx)
            self.ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _outs(self, k: int, ncols: int):
        dev = self.device
        oi = torch.empty(k, dtype=torch.int64, device=dev)
        os_ = torch.empty(k, dtype=torch.float64, device=dev)
        od = torch.empty((k, 8), dtype=torch.int32, device=dev)
        orows = torch.empty((ncols, k), dtype=torch.float64, device=dev) if ncols else None
        return oi, os_, od, orows

    def topk_merge(self, idx: torch.Tensor, score: torch.Tensor, digest: torch.Tensor, k: int,
                   rows: Optional[torch.Tensor] = None):
        """ut_topk_merge on n gathered records (device tensors):
        -> (idx [k], score [k], digest [k][8], rows [ncols][k] or None)"""
        n = idx.numel()
        idx = idx.to(self.device, torch.int64).contiguous()
        score = score.to(self.device, torch.float64).contiguous()
        digest = digest.to(self.device, torch.int32).contiguous().reshape(n, 8)
        ncols = 0 if rows is None else int(rows.shape[0])
        if rows is not None:
            rows = rows.to(self.device, torch.float64).contiguous()
        oi, os_, od, orows = self._outs(k, ncols)
        L.check(self.ctx, self.lib.ut_topk_merge(self.ctx, n, int(k), _ptr(idx), _ptr(score), _ptr(digest),
                                                 _ptr(rows), n, ncols, _ptr(oi), _ptr(os_), _ptr(od), _ptr(orows),
                                                 k), "ut_topk_merge")
        return oi, os_, od, orows


class DeviceComm(DeviceCtx):
    """This rank's RCCL communicator, driven through the C ABI (ut_comm_*)."""

    def __init__(self, device, rank: int, world: int, uid: bytes):
        super().__init__(device)
        if len(uid) != L.UT_COMM_ID_BYTES:
            raise ValueError("communicator id must be %d bytes" % L.UT_COMM_ID_BYTES)
        buf = C.create_string_buffer(bytes(uid), L.UT_COMM_ID_BYTES)
        L.check(self.ctx, self.lib.ut_comm_init(self.ctx, int(rank), int(world), buf), "ut_comm_init")
        self.rank, self.world = int(rank), int(world)

    @staticmethod
    def unique_id() -> bytes:
        buf = C.create_string_buffer(L.UT_COMM_ID_BYTES)
        L.check(None, L.lib().ut_comm_unique_id(buf), "ut_comm_unique_id")
        return buf.raw

    @classmethod
    def from_group(cls, group=None, device=None) -> "DeviceComm":
        """bootstrap over a torch.distributed group: its rank 0 creates the id,
        one broadcast_object_list hands it to every rank (collective)"""
        rank, world = dist.get_rank(group), dist.get_world_size(group)
        obj = [cls.unique_id() if rank == 0 else None]
        src = dist.get_global_rank(group, 0) if group is not None else 0
        dist.broadcast_object_list(obj, src=src, group=group,
                                   device=(torch.device("cpu") if dist.get_backend(group) == "gloo" else None))
        return cls(device if device is not None else torch.cuda.current_device(), rank, world, obj[0])

    def close(self):
        if getattr(self, "ctx", None):
            self.lib.ut_comm_destroy(self.ctx)
        super().close()

    def allgather_topk(self, idx: torch.Tensor, score: torch.Tensor, digest: torch.Tensor, k: int,
                       rows: Optional[torch.Tensor] = None):
        """ut_comm_allgather_topk: -> merged (idx, score, digest, rows or None), same on every rank"""
        kk = idx.numel()
        if kk != k:
            raise ValueError(f"allgather_topk: {kk} local records for k = {k}")
        idx = idx.to(self.device, torch.int64).contiguous()
        score = score.to(self.device, torch.float64).contiguous()
        digest = digest.to(self.device, torch.int32).contiguous().reshape(k, 8)
        ncols = 0 if rows is None else int(rows.shape[0])
        if rows is not None:
            rows = rows.to(self.device, torch.float64).contiguous()
        oi, os_, od, orows = self._outs(k, ncols)
        L.check(self.ctx, self.lib.ut_comm_allgather_topk(self.ctx, int(k), _ptr(idx), _ptr(score), _ptr(digest),
                                                          _ptr(rows), k, ncols, _ptr(oi), _ptr(os_), _ptr(od),
                                                          _ptr(orows), k), "ut_comm_allgather_topk")
        return oi, os_, od, orows

    def bcast_results(self, y: Optional[torch.Tensor], digests: Optional[torch.Tensor], n: int, src: int = 0):
        """ut_comm_bcast_results: src's (y [n], digests [n][8]) on every rank;
        a rank whose own n differs still receives src's rows (check the length)"""
        is_src = self.rank == src
        cap = max(int(n), 1)
        # a source whose rows do not match n still enters the collective (with
        # n = -1: the library sends the failure sentinel, so every rank raises
        # instead of waiting for a payload that never comes)
        bad = is_src and (y is None or digests is None or int(y.numel()) != int(n) or
                          tuple(digests.reshape(-1, 8).shape) != (int(n), 8))
        if is_src and not bad:
            yb = y.to(self.device, torch.float64).contiguous().reshape(-1)
            db = digests.to(self.device, torch.int32).contiguous().reshape(-1, 8)
        else:
            yb = torch.empty(cap, dtype=torch.float64, device=self.device)
            db = torch.empty((cap, 8), dtype=torch.int32, device=self.device)
        got = C.c_int64()
        n_arg = (-1 if bad else int(n)) if is_src else 0
        rc = self.lib.ut_comm_bcast_results(self.ctx, int(src), n_arg, _ptr(yb), _ptr(db),
                                            yb.numel() if is_src and not bad else cap, C.byref(got))
        ns = max(int(got.value), 0)
        if rc == -1 and ns > cap and not is_src:
            # src sent more rows than this rank expected (the collective completed;
            # rows past cap were dropped): return src's length, so the caller's
            # length check reports the divergence
            pad = ns - cap
            yb = torch.cat([yb, torch.full((pad,), float("nan"), dtype=torch.float64, device=self.device)])
            db = torch.cat([db, torch.zeros((pad, 8), dtype=torch.int32, device=self.device)])
        else:
            L.check(self.ctx, rc, "ut_comm_bcast_results")
        return yb[:ns], db[:ns]

    def allreduce_(self, t: torch.Tensor, op: int) -> torch.Tensor:
        """in-place all-reduce of a float64 device tensor"""
        assert t.dtype == torch.float64 and t.is_contiguous() and t.device == self.device
        L.check(self.ctx, self.lib.ut_comm_allreduce_f64(self.ctx, _ptr(t), t.numel(), int(op)),
                "ut_comm_allreduce_f64")
        return t

    def agree(self, ok: bool) -> bool:
        t = torch.tensor([1.0 if ok else 0.0], dtype=torch.float64, device=self.device)
        return bool(self.allreduce_(t, L.UT_RED_MIN).item() > 0.5)

    def barrier(self):
        L.check(self.ctx, self.lib.ut_comm_barrier(self.ctx), "ut_comm_barrier")


_CTX: Dict[int, DeviceCtx] = {}
_COMMS: Dict[Tuple[int, int], DeviceComm] = {}


def device_ctx(device) -> DeviceCtx:
    """the per-device merge context (the 1-GPU gloo rehearsal merges here)"""
    d = torch.device(device)
    key = d.index if d.index is not None else torch.cuda.current_device()
    c = _CTX.get(key)
    if c is None:
        c = _CTX[key] = DeviceCtx(torch.device("cuda", key))
    return c


def device_comm(group=None, device=None) -> DeviceComm:
    """this rank's RCCL communicator for `group` on `device`, created on first
    use (a collective: every rank of the group reaches its first exchange in
    the same order, so they bootstrap together)"""
    d = torch.device("cuda", torch.cuda.current_device()) if device is None else torch.device(device)
    if d.index is None:
        d = torch.device("cuda", torch.cuda.current_device())
    key = (id(group) if group is not None else 0, d.index)
    c = _COMMS.get(key)
    if c is None:
        c = _COMMS[key] = DeviceComm.from_group(group, d)
    return c


def release_comms() -> None:
    """destroy every communicator (before destroy_process_group)"""
    for c in list(_COMMS.values()):
        c.close()
    _COMMS.clear()


def uses_rccl(group=None) -> bool:
    """the device path: the group's backend is RCCL ("nccl") -> ut_comm_*"""
    return dist.get_backend(group) != "gloo"


def _comm_device(group, device):
    """gloo moves CPU tensors (the test double); the device path moves device tensors"""
    return torch.device("cpu") if dist.get_backend(group) == "gloo" else device


_FAIL_NEXT_ALLOC = 0   # tests: the next N receive allocations of _gather_gloo fail (as ut_debug_fail_alloc)


def _gather_gloo(t: torch.Tensor, group, dim: int = 0) -> torch.Tensor:
    """all_gather of t over gloo.  The receive buffers are allocated first and
    the ranks agree on success (an all-reduce MIN) before the collective, as
    ut_comm_allgather_topk does when its record buffers grow: a rank that could
    not allocate makes every rank raise UT_ENOMEM instead of leaving its peers
    inside all_gather."""
    global _FAIL_NEXT_ALLOC
    world = dist.get_world_size(group)
    t = t.cpu().contiguous()
    parts = None
    try:
        if _FAIL_NEXT_ALLOC > 0:
            _FAIL_NEXT_ALLOC -= 1
            raise MemoryError("injected allocation failure (dist._FAIL_NEXT_ALLOC)")
        parts = [torch.empty_like(t) for _ in range(world)]
    except (MemoryError, RuntimeError):
        parts = None
    ok = torch.tensor([0 if parts is None else 1], dtype=torch.int32)
    dist.all_reduce(ok, op=dist.ReduceOp.MIN, group=group)
    if not int(ok.item()):
        raise L.UthotError("allgather_topk failed: UT_ENOMEM: " + ("no memory for the records" if parts is None
                                                                  else "another rank could not allocate the records"))
    dist.all_gather(parts, t, group=group)
    return torch.cat(parts, dim=dim)


def _merge_gathered(gs, gi, gd, grows, k, device):
    """merge gathered records: the HIP kernel for a GPU caller, the torch
    definition only for CPU tensors (tests)"""
    if device.type == "cuda":
        return device_ctx(device).topk_merge(gi, gs, gd, k, rows=grows)
    mi, ms, pos = merge_topk(gs, gi, gd, k, return_pos=True)
    return mi, ms, gd[pos], (grows[:, pos] if grows is not None else None)


def allgather_topk(idx: torch.Tensor, score: torch.Tensor, digest: torch.Tensor, k: int,
                   group: Optional[dist.ProcessGroup] = None, rows: Optional[torch.Tensor] = None):
    """all-gather every rank's local (idx, score, digest[, rows [ncols][k]])
    top-k and merge -> (idx [k], score [k], digest [k][8], rows or None),
    identical on every rank; no host synchronisation on the device path."""
    dev = idx.device
    if dev.type == "cuda" and uses_rccl(group):
        return device_comm(group, dev).allgather_topk(idx, score, digest, k, rows=rows)
    kk = idx.numel()
    rec = torch.cat([idx.to(torch.int64).reshape(kk, 1).cpu(),
                     score.to(torch.float64).contiguous().view(torch.int64).reshape(kk, 1).cpu(),
                     digest.to(torch.int32).contiguous().reshape(kk, 8).view(torch.int64).cpu()], dim=1)
    g = _gather_gloo(rec, group)
    gr = None if rows is None else _gather_gloo(rows.to(torch.float64), group, dim=1).to(dev)
    gi = g[:, 0].contiguous().to(dev)
    gs = g[:, 1].contiguous().view(torch.float64).to(dev)
    gd = g[:, 2:].contiguous().view(torch.int32).to(dev)
    return _merge_gathered(gs, gi, gd, gr, k, dev)


def allgather_selection(idx: torch.Tensor, score: torch.Tensor, digest: torch.Tensor, rows: torch.Tensor, k: int,
                        group: Optional[dist.ProcessGroup] = None, with_digests: bool = False):
    """One scoring round's exchange for the technique layer: every rank's local
    top-k (global idx, score, digest) AND the selected value rows [ncols][k]
    travel in one all-gather of packed records and are merged identically on
    every rank, so every rank queues the same configurations.  Returns
    (idx [k], score [k], rows [ncols][k]) on the input device (+ digests
    [k][8] with with_digests=True); empty slots have idx -1."""
    mi, ms, md, mr = allgather_topk(idx, score, digest, k, group=group, rows=rows)
    if with_digests:
        return mi, ms, mr, md
    return mi, ms, mr


def broadcast_history(X: Optional[torch.Tensor], y: Optional[torch.Tensor], digests: Optional[torch.Tensor],
                      n: int, d: int, device, src: int = 0, group: Optional[dist.ProcessGroup] = None
                      ) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    """Broadcast a bootstrap history of n rows (features [n][d] f64, y [n] f64,
    digests [n][8] i32) from `src` to every rank; non-src ranks pass None.
    Device tensors over RCCL go through ut_comm_bcast."""
    rank = dist.get_rank(group)
    dev = torch.device(device)
    if rank == src:
        X = X.to(dev, torch.float64).contiguous()
        y = y.to(dev, torch.float64).contiguous()
        digests = digests.to(dev, torch.int32).contiguous()
    else:
        X = torch.empty((n, d), dtype=torch.float64, device=dev)
        y = torch.empty((n,), dtype=torch.float64, device=dev)
        digests = torch.empty((n, 8), dtype=torch.int32, device=dev)
    if dev.type == "cuda" and uses_rccl(group):
        comm = device_comm(group, dev)
        for t in (X, y, digests):
            L.check(comm.ctx, comm.lib.ut_comm_bcast(comm.ctx, _ptr(t), t.numel() * t.element_size(), int(src)),
                    "ut_comm_bcast")
        return X, y, digests
    for t in (X, y, digests):
        c = t.cpu()            # the same tensor for CPU inputs
        dist.broadcast(c, src, group=group)
        if t.device.type != "cpu":
            t.copy_(c)
    return X, y, digests


def broadcast_results(y: Optional[torch.Tensor], digests: Optional[torch.Tensor], n: int, device, src: int = 0,
                      group: Optional[dist.ProcessGroup] = None) -> Tuple[torch.Tensor, torch.Tensor]:
    """The per-round history delta of the search loop: objective values [n] f64
    and digests [n][8] i32 of the configurations evaluated on `src`, sent to
    every rank (api.sync's result injection, api.py:547-553).

    src's count travels first, so a rank whose own `n` differs still receives
    the payload in step and can report the divergence instead of breaking the
    collective; the returned tensors are src's (check their length against
    `n`).  Device path: ut_comm_bcast_results (RCCL); gloo: two broadcasts
    (count, then one [count][5] f64 payload)."""
    dev = torch.device(device) if device is not None else torch.device("cpu")
    if dev.type == "cuda" and uses_rccl(group):
        return device_comm(group, dev).bcast_results(y, digests, n, src=src)
    is_src = dist.get_rank(group) == src
    cnt = torch.tensor([n if is_src else -1], dtype=torch.int64)
    dist.broadcast(cnt, src, group=group)
    ns = int(cnt.item())
    if ns == 0:
        return (torch.empty((0,), dtype=torch.float64, device=dev),
                torch.empty((0, 8), dtype=torch.int32, device=dev))
    if is_src:
        pay = torch.cat([y.cpu().to(torch.float64).reshape(ns, 1),
                         digests.cpu().to(torch.int32).contiguous().view(torch.float64).reshape(ns, 4)], dim=1)
    else:
        pay = torch.empty((ns, 5), dtype=torch.float64)
    dist.broadcast(pay, src, group=group)
    y = pay[:, 0].contiguous().to(dev)
    digests = pay[:, 1:].contiguous().view(torch.int32).reshape(ns, 8).to(dev)
    return y, digests


def agree(ok: bool, group=None, device=None) -> bool:
    """True iff every rank of the group passes ok=True.  Every rank takes the
    same branch afterwards, so a failure on one rank never leaves the others
    waiting inside a later collective.  On an RCCL group the vote travels over
    this rank's communicator on `device` (or the current GPU when the caller
    has none -- a failed round still votes on the device every healthy rank
    uses); on gloo it is a CPU all_reduce."""
    if uses_rccl(group):
        d = device if device is not None else torch.device("cuda", torch.cuda.current_device())
        return device_comm(group, d).agree(ok)
    t = torch.tensor([1 if ok else 0], dtype=torch.int32)
    dist.all_reduce(t, op=dist.ReduceOp.MIN, group=group)
    return bool(int(t.item()))
