"""Multi-GPU exchange for the scoring round (one process per GPU).

SURVEY.md §8(e): the candidate pool is sharded by GLOBAL candidate index
(rank r owns [r*m, (r+1)*m)); population, training set, GP factor and history
are replicated.  Two real exchanges exist per round:

  * all_gather of every rank's local top-k records (score, index, digest) and a
    deterministic merge -- cross-shard duplicates (equal digests) keep the
    smallest global index, ties on score break by the smallest index, so the
    merged top-k is identical to the single-GPU result for the same pool;
  * broadcast from rank 0 of the per-round history delta (new evaluated rows,
    their objective values and digests) -- the analog of the reference's
    per-round api.sync result injection (python/uptune/api.py:547-553,
    opentuner/api.py:87-104).

Backend "nccl" is RCCL over xGMI on ROCm; the same code runs with "gloo" on
CPU tensors (tests/test_dist_cpu.py).  Payloads are a few KB (latency
bound), so there is no bucketing.
"""
from __future__ import annotations

from typing import Optional, Tuple

import torch
import torch.distributed as dist


def merge_topk(scores: torch.Tensor, idx: torch.Tensor, digests: torch.Tensor, k: int
               ) -> Tuple[torch.Tensor, torch.Tensor]:
    """Merge gathered local top-k lists.

    scores [R*k] f64, idx [R*k] i64 (-1 = empty slot), digests [R*k][8] i32.
    Returns (idx [k], score [k]) sorted by (-score, idx), empty slots -1.
    Cross-shard duplicates (equal digests) keep the smallest global index.

    Fixed-size tensor ops only -- no boolean indexing, no .item(): the merge
    never waits for the device, so the host keeps enqueueing the next round
    while this one computes (the N > 1 bench loop stays asynchronous).
    """
    n = idx.numel()
    dev = idx.device
    big = torch.iinfo(torch.int64).max
    valid = idx >= 0
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
    if out_i.numel() < k:
        pad = k - out_i.numel()
        out_i = torch.cat([out_i, torch.full((pad,), -1, dtype=idx.dtype, device=dev)])
        out_s = torch.cat([out_s, torch.full((pad,), float("-inf"), dtype=scores.dtype, device=dev)])
    return out_i, out_s


def allgather_topk(idx: torch.Tensor, score: torch.Tensor, digest: torch.Tensor, k: int,
                   group: Optional[dist.ProcessGroup] = None) -> Tuple[torch.Tensor, torch.Tensor]:
    """all_gather the local (idx, score, digest) top-k of every rank and merge:
    one all_gather of packed [k][6] int64 records (index, score bits, digest
    as 4 words), then merge_topk -- no host synchronisation."""
    world = dist.get_world_size(group)
    dev = idx.device
    cd = _comm_device(group, dev)
    kk = idx.numel()
    rec = torch.cat([idx.to(torch.int64).reshape(kk, 1),
                     score.to(torch.float64).contiguous().view(torch.int64).reshape(kk, 1),
                     digest.to(torch.int32).contiguous().reshape(kk, 8).view(torch.int64)], dim=1).to(cd)
    parts = [torch.empty_like(rec) for _ in range(world)]
    dist.all_gather(parts, rec, group=group)
    g = torch.cat(parts)
    gd = g[:, 2:].contiguous().view(torch.int32)
    mi, ms = merge_topk(g[:, 1].contiguous().view(torch.float64), g[:, 0].contiguous(), gd, k)
    return mi.to(dev), ms.to(dev)


def broadcast_history(X: Optional[torch.Tensor], y: Optional[torch.Tensor], digests: Optional[torch.Tensor],
                      n: int, d: int, device, src: int = 0, group: Optional[dist.ProcessGroup] = None
                      ) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    """Broadcast a history delta of n rows (features [n][d] f64, y [n] f64,
    digests [n][8] i32) from `src` to every rank; non-src ranks pass None."""
    rank = dist.get_rank(group)
    if rank == src:
        X = X.to(device, torch.float64).contiguous()
        y = y.to(device, torch.float64).contiguous()
        digests = digests.to(device, torch.int32).contiguous()
    else:
        X = torch.empty((n, d), dtype=torch.float64, device=device)
        y = torch.empty((n,), dtype=torch.float64, device=device)
        digests = torch.empty((n, 8), dtype=torch.int32, device=device)
    dist.broadcast(X, src, group=group)
    dist.broadcast(y, src, group=group)
    dist.broadcast(digests, src, group=group)
    return X, y, digests


def _comm_device(group, device):
    """gloo moves CPU tensors (and runs the CPU tests); nccl (= RCCL) moves
    device tensors over xGMI"""
    return torch.device("cpu") if dist.get_backend(group) == "gloo" else device


def allgather_selection(idx: torch.Tensor, score: torch.Tensor, digest: torch.Tensor, rows: torch.Tensor, k: int,
                        group: Optional[dist.ProcessGroup] = None, with_digests: bool = False):
    """One scoring round's exchange for the technique layer: every rank's local
    top-k (global idx, score, digest) AND the selected value rows [ncols][k]
    are all-gathered; the merge (merge_topk) is identical on every rank and the
    rows of the merged selection are taken from the gathered rows, so every
    rank queues the same configurations.  Returns (idx [k], score [k],
    rows [ncols][k]) on the input device (+ digests [k][8] with
    with_digests=True); empty slots have idx -1."""
    dev = idx.device
    cd = _comm_device(group, dev)
    world = dist.get_world_size(group)
    parts = []
    for t in (idx.to(torch.int64), score.to(torch.float64), digest.to(torch.int32), rows.to(torch.float64)):
        t = t.to(cd).contiguous()
        g = [torch.empty_like(t) for _ in range(world)]
        dist.all_gather(g, t, group=group)
        parts.append(g)
    gi = torch.cat(parts[0])
    gs = torch.cat(parts[1])
    gd = torch.cat(parts[2])
    grows = torch.cat(parts[3], dim=1)
    mi, ms = merge_topk(gs, gi, gd, k)
    pos = {int(g): p for p, g in enumerate(gi.tolist()) if g >= 0}
    take = torch.tensor([pos[int(g)] if g >= 0 else 0 for g in mi.tolist()], dtype=torch.int64, device=cd)
    out_rows = grows[:, take]
    if with_digests:
        return mi.to(dev), ms.to(dev), out_rows.to(dev), gd[take].to(dev)
    return mi.to(dev), ms.to(dev), out_rows.to(dev)


def broadcast_results(y: Optional[torch.Tensor], digests: Optional[torch.Tensor], n: int, device, src: int = 0,
                      group: Optional[dist.ProcessGroup] = None) -> Tuple[torch.Tensor, torch.Tensor]:
    """The per-round history delta of the search loop: objective values [n] f64
    and digests [n][8] i32 of the configurations evaluated on `src`, sent to
    every rank (api.sync's result injection, api.py:547-553).

    Two broadcasts: src's count, then one [count][5] f64 payload (the value and
    the digest's 32 bytes reinterpreted as 4 f64).  The count travels first so
    that a rank whose own `n` differs still receives the payload in step and can
    report the divergence instead of breaking the collective; the returned
    tensors are src's (check their length against `n`)."""
    cd = _comm_device(group, device)
    is_src = dist.get_rank(group) == src
    cnt = torch.tensor([n if is_src else -1], dtype=torch.int64, device=cd)
    dist.broadcast(cnt, src, group=group)
    ns = int(cnt.item())
    if ns == 0:
        return (torch.empty((0,), dtype=torch.float64, device=cd),
                torch.empty((0, 8), dtype=torch.int32, device=cd))
    if is_src:
        pay = torch.cat([y.to(cd, torch.float64).reshape(ns, 1),
                         digests.to(cd, torch.int32).contiguous().view(torch.float64).reshape(ns, 4)], dim=1)
    else:
        pay = torch.empty((ns, 5), dtype=torch.float64, device=cd)
    if ns > 0:
        dist.broadcast(pay, src, group=group)
    y = pay[:, 0].contiguous()
    digests = pay[:, 1:].contiguous().view(torch.int32).reshape(ns, 8)
    return y, digests
