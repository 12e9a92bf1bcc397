#!/usr/bin/env python
"""Throughput of the batch candidate-scoring hot path on MI355X.

Workload (BASELINE.json configs[1], "C2" in SURVEY.md §8(d)):
  Rosenbrock-64 space: 64 FloatParameters named 0..63 in [-1000, 1000]
  DE-Alt proposal (cr = 0.2, n_cross = 1, F = U/2 + 0.5) over a population of
  m candidates per GPU, hash_config + dedup against the history,
  GP surrogate n = 1024 (SE-ARD, ell = 0.2, sf2 = 1, sn2 = 1e-6) refit every
  round, EI (xi = 0) + top-k (k = 256), fp64.
One step = one round: GP fit + propose + hash + dedup + encode + GP score +
top-k (+ all-gather merge of the local top-k over RCCL when N > 1).

    python bench.py [--gpus N --steps K --warmup W]

N > 1: one process per GPU.  Under torch.distributed.run (WORLD_SIZE set)
each process is one rank; run directly with --gpus N, the script starts the N
rank processes itself (before anything touches a GPU) and relays rank 0's line.
Each rank scores its own shard of global candidate indices: --scaling weak
(default) fixes m per GPU (global pool N*m), --scaling strong fixes the global
pool m (rank r scores [r*m/N, (r+1)*m/N)).  The local top-k lists travel
through libuthot's own RCCL communicator (ut_comm_allgather_topk: all-gather +
HIP merge kernel) and the merged selections join every rank's history, so
every rank selects the same candidates, and `selection_sha` (the last timed
round's merged (index, digest) list) is the same at every N for one global
pool: strong lines at N = 1, 2, 4, 8 carry equal shas, and a weak line at N
equals the one-rank line of --m N*m.  torch.distributed (gloo) only bootstraps
the communicator and carries the barriers.  UT_DIST_BACKEND=gloo rehearses N
ranks on fewer GPUs (records over gloo, merge on the device).
`hbm_bytes_per_rank` is the device memory libuthot holds per rank (max over
ranks; each rank caches inner digests for its own shard's DE targets only).

`roofline` is the round's dominant kernel: the variance GEMM (fp64 / fp32 /
f16x3 dense lines), K* where it carries more work (C4), and in a pruned line
(--prune) the K* with the mean in its epilogue -- flops of its fp64
contraction only (in categorical mode the one-hot blocks' int8 code product
beside it is not counted), timed without the wait for the fit (`fit_wait`).

After the timed rounds (outside the timed region) rank 0 checks the last
round's selections against the oracle (`parity`: DE trials, hash_config
digests, EI) and runs one extra round at a lengthscale whose EI top-k is
score-determined, checking it against the oracle EI of a random sample of the
other candidates.  Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

# MI355X peaks (MI355X_MICROARCH.md chip table; FP64 matrix = FP64 vector
# spec 78.6 TF -- SURVEY.md §8(d))
PEAK_FP64_TFLOPS = 78.6
PEAK_FP32_TFLOPS = 157.3
PEAK_FP16_TFLOPS = 2516.6   # dense fp16 MFMA (256 CU x 4 SIMD x 1024 flop/clk x 2.4 GHz)
PEAK_I8_TOPS = 5033.2       # dense int8 MFMA (2x the fp16 rate: 32x32x32 i8 in the cycles of 32x32x16 f16)
I8_PRODUCTS = 21            # digit-plane products per algorithmic multiply-add at precision 8 (gp_i8.hip)
PEAK_HBM_GBS = 8000.0


def rosenbrock_decoded(X01):
    xs = X01 * 2000.0 - 1000.0
    return np.sum(100.0 * (xs[:, 1:] - xs[:, :-1] ** 2) ** 2 + (xs[:, :-1] - 1.0) ** 2, axis=1)


def training_set(n, d, seed):
    rng = np.random.default_rng(seed)
    X = rng.uniform(size=(n, d))
    return X, rosenbrock_decoded(X)


def selection_sha(idx, dig):
    """sha256 of a round's merged selections (global indices, then digests)"""
    import hashlib
    return hashlib.sha256(idx.detach().cpu().numpy().astype("<i8").tobytes() +
                          dig.detach().cpu().numpy().view(np.uint32).astype(">u4").tobytes()).hexdigest()


def host_info():
    """CPU model, logical CPUs of the machine, and the threads this job may use
    (OMP_NUM_THREADS, else the affinity mask: 16 per GPU on the MI355X boxes)"""
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:  # pragma: no cover
        aff = os.cpu_count()
    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or aff
    return {"cpu_model": model, "nproc": os.cpu_count(), "affinity_cpus": aff, "threads": min(threads, aff)}


def cpu_baseline_b1(m_sample, n, d, k, threads, seed=1):
    """B1: the same C2 round vectorised on `threads` host
    cores -- C++/OpenMP DE + hash_config + dedup, BLAS GP (oracle/cpu_batch.*)"""
    from oracle import cpu_batch
    return cpu_batch.b1_baseline(m_sample, n, d, k, seed=seed, threads=threads)


def cpu_baseline(m_sample, n, d, k, seed=1):
    """The oracle (CPU restatement of the reference path) on a bounded sample,
    single-threaded like the reference search loop (api.py:428-446)."""
    try:
        from threadpoolctl import threadpool_limits
    except Exception:  # pragma: no cover
        threadpool_limits = None
    from oracle import de as ode
    from oracle import gp as ogp
    from oracle import hashing as oh
    from oracle import select as osel
    from oracle.space import FLOAT, Param, features

    space = [Param(i, FLOAT, -1000.0, 1000.0) for i in range(d)]
    X, y = training_set(n, d, seed + 100)
    ctx = threadpool_limits(limits=1) if threadpool_limits else None
    if ctx:
        ctx.__enter__()
    try:
        pop = ode.population_init(space, m_sample, seed)
        t0 = time.perf_counter()
        g = ogp.GP(X, y, lengthscale=0.2, sigma_f2=1.0, sigma_n2=1e-6)
        trial = ode.propose_de_vec(space, pop, seed, 0, 0, m_sample, 0.2, 1)
        hx = [oh.hash_config(space, list(trial[:, j])) for j in range(m_sample)]
        dup = osel.dedup(hx, set())
        mu, var = g.posterior(features(space, trial).T)
        ei = ogp.acquisition(mu, var, g.f_best)
        osel.topk(list(ei), k, dup=dup)
        dt = time.perf_counter() - t0
    finally:
        if ctx:
            ctx.__exit__(None, None, None)
    return {"value": m_sample / dt, "unit": "candidates/s", "cores": 1, "kind": "port",
            "sample": f"oracle/ (NumPy+hashlib restatement), {m_sample} R64 candidates, n={n} GP fit + DE + "
                      f"hash_config + dedup + posterior + EI + top-{k}, 1 thread, {dt:.2f} s"}


def load_pmc(kernel_key):
    """the rocprofv3 record of a kernel (profiles/pmc_summary.json: HBM bytes
    per launch from the FETCH_SIZE / WRITE_SIZE passes, average duration from
    the --kernel-trace --stats pass of the same command)"""
    path = os.path.join(ROOT, "profiles", "pmc_summary.json")
    try:
        with open(path) as f:
            d = json.load(f)
        return d.get(kernel_key) or {}, d.get("_note", "")
    except Exception:
        return {}, ""


SHA256_CEIL_GCPS = 28.5   # measured chip ceiling of SHA-256 compressions (scripts/exp/sha_rate.hip)


def profile_suffix(ell):
    """record-key suffix of a profiled C2 pass: "" at the headline's ell = 0.2,
    "_l2" for the secondary line's ell = 2 (scripts/r06_prof.sh)"""
    return "" if ell == 0.2 else "_l2"


def load_clock():
    """profiles/clock_summary.json: per kernel the duration, clock and MFMA busy
    of the rocprofv3 counter pass (dispatches serialized: each kernel alone)"""
    try:
        with open(os.path.join(ROOT, "profiles", "clock_summary.json")) as f:
            return json.load(f)
    except Exception:
        return {}


def kernel_table(m, n, d, outer_blocks, prec=64, suffix=""):
    """Per-kernel rooflines of the default C2 round from the committed rocprofv3
    record (profiles/pmc_summary.json: HBM bytes from the FETCH_SIZE /
    WRITE_SIZE passes; profiles/clock_summary.json: durations from the counter
    pass, where rocprofv3 serializes the dispatches -- else the --kernel-trace
    --stats average of the concurrent round).  Algorithmic work per launch
    (SURVEY.md §8(d)):
      k_de: 40 d B per candidate (target, 3 donors, trial); k_hash (outer):
      outer_blocks compressions per candidate; K*: 2 n dpad flops; encode: 16 F B.
    prec 8: K* is k_gp_kstar_q (gp_kq.hip: the distance contraction on the int8
    MFMA, 21 digit products per multiply-add, the exp and six digit planes in its
    epilogue; record key kstar8; its peak = int8 peak / 21, as the variance's;
    UT_KSTAR_Q=0: k_gp_kstar<int8_t> on the fp64 MFMA).  suffix "_l2": the ell =
    2 records."""
    out = {}
    try:
        with open(os.path.join(ROOT, "profiles", "pmc_summary.json")) as f:
            pmc = json.load(f)
    except Exception:
        return out
    clk = load_clock()
    srcs = set()

    def rec(key):
        key = key + suffix
        r = pmc.get(key) or {}
        c = clk.get(key) or {}
        if c:
            t = c.get("duration_ms", 0.0) * 1e-3
            srcs.add("%s: clock_summary.json (counter pass %s, serialized) + pmc_summary.json (%s)" %
                     (key, c.get("source", "?"), r.get("source", "?")))
        else:
            t = (r.get("avg_ns") or 0.0) * 1e-9
            if r:
                srcs.add("%s: pmc_summary.json (%s; duration = --kernel-trace --stats average, concurrent)" %
                         (key, r.get("source", "?")))
        return t, r.get("hbm_bytes_per_launch")

    def hbm(key, alg_bytes):
        t, traffic = rec(key)
        if t <= 0:
            return
        out[key] = {"bound": "hbm", "ms": t * 1e3, "achieved_GBps": alg_bytes / t / 1e9,
                    "frac": alg_bytes / t / 1e9 / PEAK_HBM_GBS, "algorithmic_bytes": alg_bytes,
                    "traffic_bytes": traffic, "traffic_GBps": (traffic / t / 1e9) if traffic else None}

    def mfma(key, flops, peak=PEAK_FP64_TFLOPS):
        t, traffic = rec(key)
        if t <= 0:
            return
        out[key] = {"bound": "mfma", "ms": t * 1e3, "achieved_TFps": flops / t / 1e12,
                    "frac": flops / t / 1e12 / peak, "peak_TFps": peak, "flops": flops, "traffic_bytes": traffic,
                    # (K* at precision 8 stores six digit planes per k*: 6 n B per candidate)
                    "traffic_frac_of_hbm_peak": (traffic / t / 1e9 / PEAK_HBM_GBS) if traffic else None}

    hbm("propose", 40.0 * d * m)
    hbm("encode", 16.0 * d * m)
    kq = prec == 8 and os.environ.get("UT_KSTAR_Q", "1") != "0"
    mfma("kstar8" if prec == 8 else "kstar", 2.0 * n * (d + (-d) % 16) * m,   # the variance GEMM is `roofline`
         PEAK_I8_TOPS / I8_PRODUCTS if kq else PEAK_FP64_TFLOPS)
    t, traffic = rec("hash")
    if t > 0:
        c = float(outer_blocks) * m
        out["hash"] = {"bound": "int VALU (SHA-256)", "ms": t * 1e3, "achieved_Gcompressions_ps": c / t / 1e9,
                       "frac": c / t / 1e9 / SHA256_CEIL_GCPS, "compressions": c, "traffic_bytes": traffic,
                       "ceiling": f"{SHA256_CEIL_GCPS} G compressions/s (measured, scripts/exp/sha_rate.hip)"}
    for key, r in out.items():
        if key + suffix in clk:
            r["clock_ghz"] = clk[key + suffix].get("clock_ghz")
            r["mfma_busy"] = clk[key + suffix].get("mfma_busy")
    out["_source"] = sorted(srcs)
    return out


def spawn_ranks(n):
    """--gpus N without a launcher: start N rank processes (one GPU each) before
    this process touches a GPU, relay rank 0's output, and fail if any rank
    fails (the others are stopped then, so none waits in a collective)."""
    import socket
    import subprocess
    import tempfile
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    out0 = tempfile.TemporaryFile(mode="w+")
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env,
                                      stdout=out0 if r == 0 else subprocess.DEVNULL))
    rc = 0
    live = list(procs)
    while live:
        time.sleep(0.2)
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code != 0 and rc == 0:
                rc = code
                print(f"bench: rank {procs.index(p)} exited with {code}; stopping the other ranks",
                      file=sys.stderr, flush=True)
                for q in live:
                    q.terminate()
                for q in live:
                    try:
                        q.wait(timeout=20)
                    except subprocess.TimeoutExpired:
                        q.kill()
                live = []
    out0.seek(0)
    sys.stdout.write(out0.read())
    sys.stdout.flush()
    return rc


def oracle_space_of(manip):
    """uptune_amd manipulator -> oracle Param list (the checker's view of the space)"""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from tests._spaces import oracle_space
    return oracle_space(manip)


def parity_de_round(eng, space, idx, top, dig, npop, seed, round_, X, y, ell, jitter, k):
    """The checker (outside the timed region): a DE round's merged selections
    (global indices idx, scores top, digests dig) against the oracle --
    the trials the oracle proposes at those indices (differentialevolution.py:105-129
    restated in oracle/de.py) equal the device's, their hash_config digests
    (manipulator.py:233-243) equal the round's, and the round's scores equal
    the oracle GP's EI (oracle/gp.py) within 1e-5 relative.
    -> (report dict, oracle trials [ncols][k'], oracle EI [k'])"""
    import torch
    from oracle import de as ode
    from oracle import gp as ogp
    from oracle import hashing as oh
    from oracle.space import features, from_f64
    from uptune_amd.engine import digests_to_hex
    ii = idx.cpu().numpy()
    sel = np.flatnonzero(ii >= 0)
    g = ii[sel]
    want = ode.propose_de_at(space, g, npop, seed, round_, 0.2, 1)
    got = torch.stack([eng.propose_de(1, round_=round_, cand_base=int(j), cr=0.2, n_cross=1)[:, 0] for j in g],
                      dim=1).cpu().numpy() if len(g) else np.zeros_like(want)
    hexes = [oh.hash_config(space, [from_f64(p, want[c, j]) for c, p in enumerate(space)]) for j in range(len(g))]
    ghex = digests_to_hex(dig[torch.as_tensor(sel, device=dig.device)]) if len(g) else []
    gp = ogp.GP(X, y, lengthscale=ell, sigma_f2=1.0, sigma_n2=1e-6, jitter=jitter)
    mu, var = gp.posterior(features(space, want).T)
    ei = ogp.acquisition(mu, var, gp.f_best)
    s = top.cpu().numpy()[sel]
    rel = float(np.max(np.abs(s - ei) / np.maximum(np.abs(ei), 1e-300))) if len(g) else 0.0
    return ({"rows": int(len(g)), "trials_equal": bool(np.array_equal(got, want)),
             "digests_equal": bool(ghex == hexes), "ei_max_rel_err": rel, "round": int(round_)}, want, ei)


def parity_ga_round(eng, space, idx, top, dig, parent, seed, round_, X, y, ell, jitter):
    """The checker for a C4 GA round (outside the timed region): the oracle's
    UniformGreedyMutation children at the selected global indices
    (evolutionarytechniques.py:29-61 restated in oracle/ga.py) equal the
    device's, their hash_config digests equal the round's, and the scores equal
    the oracle GP's EI within 1e-5 relative."""
    import torch
    from oracle import ga as oga
    from oracle import gp as ogp
    from oracle import hashing as oh
    from oracle.space import features, from_f64
    from uptune_amd.engine import digests_to_hex
    ii = idx.cpu().numpy()
    sel = np.flatnonzero(ii >= 0)
    g = ii[sel]
    want, winv = oga.propose_ga_vec(space, parent, None, seed, round_, 0, 0, mutation_rate=0.1, g=g)
    got = torch.cat([eng.propose_ga(1, parent1=parent, round_=round_, cand_base=int(j), mutation_rate=0.1)[0]
                     for j in g], dim=1).cpu().numpy() if len(g) else np.zeros_like(want)
    hexes = [oh.hash_config(space, [from_f64(p, want[c, j]) for c, p in enumerate(space)]) for j in range(len(g))]
    ghex = digests_to_hex(dig[torch.as_tensor(sel, device=dig.device)]) if len(g) else []
    gp = ogp.GP(X, y, lengthscale=ell, sigma_f2=1.0, sigma_n2=1e-6, jitter=jitter)
    mu, var = gp.posterior(features(space, want).T)
    ei = ogp.acquisition(mu, var, gp.f_best)
    s = top.cpu().numpy()[sel]
    rel = float(np.max(np.abs(s - ei) / np.maximum(np.abs(ei), 1e-300))) if len(g) else 0.0
    return {"rows": int(len(g)), "trials_equal": bool(np.array_equal(got, want)), "valid": bool(not winv.any()),
            "digests_equal": bool(ghex == hexes), "ei_max_rel_err": rel, "round": int(round_)}


def kstar_fp64_features(eng, d):
    """the features K* contracts in fp64: every feature, or in categorical mode
    (ENUM / BOOL one-hot blocks as int8 codes) the numeric ones only"""
    if eng.gp_kstar_mode() != "categorical":
        return d
    from uptune_amd import _lib as L
    return sum(p.n_feat for p in eng.spec.params if p.kind not in (L.UT_BOOL, L.UT_ENUM))


def main():
    if "WORLD_SIZE" not in os.environ:
        pre = argparse.ArgumentParser(add_help=False)
        pre.add_argument("--gpus", type=int, default=1)
        n_req = pre.parse_known_args()[0].gpus
        if n_req > 1:
            sys.exit(spawn_ranks(n_req))
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--m", "--candidates", dest="m", type=int, default=1 << 20,
                    help="candidates per GPU per round (--scaling weak) or the global pool of a round "
                         "(--scaling strong)")
    ap.add_argument("--scaling", default="weak", choices=("weak", "strong"),
                    help="weak: every rank scores m candidates of a global pool of N*m (the population has N*m "
                         "members); strong: the global pool is m (population m) and rank r scores "
                         "[r*m/N, (r+1)*m/N) -- the same workload, and the same selections (selection_sha), "
                         "at every N")
    ap.add_argument("--n", type=int, default=1024, help="GP training points")
    ap.add_argument("--d", type=int, default=64)
    ap.add_argument("--k", type=int, default=256)
    ap.add_argument("--cpu-sample", type=int, default=32768,
                    help="candidates in the 1-thread oracle baseline sample (about 4 s of single-thread work)")
    ap.add_argument("--b1-sample", type=int, default=1 << 18,
                    help="candidates in the B1 batch baseline sample (C++/OpenMP + BLAS on the host cores)")
    ap.add_argument("--ell", type=float, default=None,
                    help="the GP lengthscale of the timed rounds (default: the config's -- C2 0.2, C3 1, C4 2)")
    ap.add_argument("--no-secondary", dest="secondary", action="store_false",
                    help="C2: skip the secondary line (the same rounds timed at ell = 2, score-determined)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-parity", action="store_true", help="skip the oracle check of the selections")
    ap.add_argument("--parity-sample", type=int, default=1 << 16,
                    help="random other candidates whose oracle EI must not beat the score-determined top-k")
    ap.add_argument("--precision", type=int, default=None, choices=(64, 32, 16, 8),
                    help="GP contractions on fp64 MFMA (1e-5 parity) or fp32 MFMA (1e-3 parity); 16 = f16x3: "
                         "the variance contraction as 3 fp16 MFMA products of hi/lo splits (fp32 tier, 1e-3); "
                         "8 = the fp64 tier (1e-5) on the int8 MFMA: six-digit slices, per-candidate error "
                         "bound, fp64 recompute of the candidates it does not clear (the default; --prune: 64)")
    ap.add_argument("--config", default="c2", choices=("c2", "c3", "c4"),
                    help="c2 = BASELINE configs[1] (R64, m=1M, n=1024: the headline); c3 = configs[2] per GPU "
                         "(HPL-64 mixed space, 16M/8 = 2M candidates per GPU, n=4096); c4 = configs[3] "
                         "(gcc 339-flag space, GA proposals, dedup against the 3,680 recorded configs, m=4M)")
    ap.add_argument("--prune", type=int, default=0, metavar="ROWS",
                    help="selection-exact EI-bound pruning (ut_score_round_de_pruned) with the first ROWS rows of "
                         "L^-1 k* as the bound; a secondary line, fp64 only (the dense round stays the headline)")
    ap.add_argument("--prune-pass", type=int, default=32, choices=(32, 64),
                    help="--prune's bound pass over every candidate: 32 = K* past the bound rows on the f32 MFMA "
                         "with v_exp_f32, every rounding bounded (ut_gp_set_prune_pass; the default), 64 = fp64")
    args = ap.parse_args()
    if args.precision is None:
        args.precision = 64 if args.prune else 8
    if args.prune and args.precision != 64:
        ap.error("--prune needs --precision 64")
    if args.config == "c3":
        if args.m == 1 << 20:
            args.m = 1 << 21
        if args.n == 1024:
            args.n = 4096
    if args.config == "c4" and args.m == 1 << 20:
        args.m = 1 << 22

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world != args.gpus:
        ap.error(f"--gpus {args.gpus} but the launcher started WORLD_SIZE={world} ranks")
    ndev = torch.cuda.device_count()
    # UT_DIST_BACKEND=gloo rehearses the N > 1 path with several ranks on fewer
    # GPUs (they share them round-robin); the multi-GPU runs use RCCL, one GPU per rank
    backend = os.environ.get("UT_DIST_BACKEND", "nccl")
    if world > 1 and backend == "nccl" and world > ndev:
        ap.error(f"{world} RCCL ranks need {world} GPUs, {ndev} visible (UT_DIST_BACKEND=gloo shares GPUs)")
    local = int(os.environ.get("LOCAL_RANK", "0")) % max(ndev, 1)
    torch.cuda.set_device(local)
    n_gpus = min(world, max(ndev, 1))      # distinct devices of the job
    if world > 1:   # host-side control (bootstrap, barriers, timing max); the data path is below
        dist.init_process_group("gloo")

    from uptune_amd.dist import DeviceComm, allgather_topk
    from uptune_amd.engine import BatchEngine
    from uptune_amd.manipulator import ConfigurationManipulator, FloatParameter

    n, d, k = args.n, args.d, args.k
    # the shard of global candidate indices this rank scores:
    # weak scaling fixes the per-rank m (global pool N*m), strong scaling the
    # global pool (rank r: [r*M/N, (r+1)*M/N))
    if args.scaling == "strong":
        npop = args.m
        if npop < world:
            ap.error(f"--scaling strong needs --m >= the {world} ranks")
        cand_base = rank * npop // world
        m = (rank + 1) * npop // world - cand_base
    else:
        m = args.m
        npop = m * world                   # replicated population, deterministic init on every rank
        cand_base = rank * m
    if args.config == "c3":
        from uptune_amd import spaces
        manip = spaces.hpl64()
    elif args.config == "c4":
        from uptune_amd import spaces
        manip = spaces.gcc()
    else:
        manip = ConfigurationManipulator([FloatParameter(i, -1000.0, 1000.0) for i in range(d)])
    eng = BatchEngine(manip, device=local, seed=1)
    eng.gp_set_precision(args.precision)
    if args.prune:
        eng.gp_set_prune_pass(args.prune_pass)
    eng.population_init(npop)
    # the results history holds the evaluated configurations: the n training
    # points (C2/C3) or the 3,680 recorded gcc configs (C4), plus every round's
    # selections (appended on the device after the round, as an evaluation
    # would); capacity reserved up front so no growth happens in the timed loop
    eng.history_reset(4 * (n + 3680 + (args.warmup + args.steps) * k))
    if args.config == "c3":
        # training points: n HPL-64 configs (device op1_randomize), features encoded on
        # the device; synthetic objective = squared distance of the features from 0.3
        d = eng.spec.n_features
        tr = BatchEngine(manip, device=local, seed=101)
        tr.population_init(n)
        tv = tr.population_get()
        X = tr.encode(tv).T.contiguous().cpu().numpy()
        eng.history_add(eng.hash(tv))
        y = np.sum((X - 0.3) ** 2, axis=1)
        tr.close()
    elif args.config == "c4":
        # the recorded gcc configs (samples/gcc-options/matmul-record.csv, as the
        # fixture tests/golden/gcc_history.npz): all 3,680 are the dedup history,
        # the first n with their recorded qor are the GP training set, the best
        # recorded config is the GA parent (GreedySelectionMixin.select)
        z = np.load(os.path.join(ROOT, "tests", "golden", "gcc_history.npz"))
        hist, qor = z["values"], z["qor"]
        hv = torch.from_numpy(np.ascontiguousarray(hist)).to(eng.device)
        eng.history_add(eng.hash(hv))
        d = eng.spec.n_features
        ok_rows = torch.from_numpy(np.flatnonzero(np.isfinite(qor))[:n]).to(eng.device)   # 149 runs failed: inf
        X = eng.encode(hv[:, ok_rows].contiguous()).T.contiguous().cpu().numpy()
        y = qor[ok_rows.cpu().numpy()].astype(np.float64)
        parent = hist[:, int(np.argmin(qor))].copy()
        assert np.all(np.isfinite(y)) and X.shape[0] == n
    else:
        X, y = training_set(n, d, 101)
        hv = torch.from_numpy(np.ascontiguousarray((X * 2000.0 - 1000.0).T)).to(eng.device)   # decoded configs
        eng.history_add(eng.hash(hv))
    acq = eng.acq("ei", xi=0.0)
    ell = args.ell if args.ell is not None else {"c2": 0.2, "c3": 1.0, "c4": 2.0}[args.config]

    comm = None
    exchange_note = None
    if world > 1 and backend == "nccl":
        try:
            comm = DeviceComm.from_group(None, eng.device)   # libuthot's RCCL communicator (id over gloo)
        except Exception as ex:   # keep the run: records over gloo, the merge still on the device
            exchange_note = f"RCCL communicator init failed ({ex!r}); records over gloo + HIP merge"
            print(f"bench rank {rank}: {exchange_note}", file=sys.stderr, flush=True)
        ok = torch.tensor([0 if comm is None else 1], dtype=torch.int32)
        dist.all_reduce(ok, op=dist.ReduceOp.MIN)   # every rank takes the same exchange path
        if int(ok.item()) == 0 and comm is not None:
            comm.close()
            comm = None
            exchange_note = exchange_note or "another rank's RCCL init failed; records over gloo + HIP merge"

    def exchange(idx, top, dig):
        """merged top-k of every rank (identical on all ranks); world 1: the local list"""
        if world == 1:
            return idx, top, dig
        if comm is not None:
            i, s_, d_, _ = comm.allgather_topk(idx, top, dig, k)
        else:
            i, s_, d_, _ = allgather_topk(idx, top, dig, k)
        return i, s_, d_

    def step_c4(r):
        """GA round (ut_score_round_ga): UniformGreedyMutation proposals from the
        best recorded config -> hash_config (the parent's inner digests reused) +
        dedup vs history + batch on a second stream, beside encode (fused) ->
        GP-EI -> top-k"""
        eng.gp_fit(X, y, lengthscale=ell, sigma_f2=1.0, sigma_n2=1e-6, jitter=1e-8, wait=False)
        idx, top, sdig, _ = eng.score_round_ga(m, k, parent1=parent, round_=r, cand_base=cand_base,
                                               mutation_rate=0.1, acq=acq, want_values=False)
        idx, top, sdig = exchange(idx, top, sdig)
        eng.history_add(sdig)                             # the merged selections join every rank's history
        return idx, top, sdig

    prune_stats = []

    def step(r, ell=ell):
        if args.config == "c4":
            return step_c4(r)
        eng.gp_fit(X, y, lengthscale=ell, sigma_f2=1.0, sigma_n2=1e-6, wait=False)   # overlaps propose + hash
        if args.prune:
            idx, top, dig, _, st = eng.score_round_de_pruned(m, k, round_=r, cand_base=cand_base, cr=0.2, n_cross=1,
                                                             acq=acq, want_values=False, bound_rows=args.prune)
            prune_stats.append(st)
        else:
            idx, top, dig, _ = eng.score_round_de(m, k, round_=r, cand_base=cand_base, cr=0.2, n_cross=1, acq=acq,
                                                  want_values=False)
        idx, top, dig = exchange(idx, top, dig)           # RCCL all-gather + HIP merge (world > 1)
        eng.history_add(dig)                              # the merged selections join every rank's history
        return idx, top, dig

    def timed_rounds(first, steps, ell_):
        """`steps` rounds from round `first` at lengthscale ell_, bracketed by a
        barrier + device sync on both sides; -> (seconds, max over ranks;
        per-stage device ms; i8 stats of the last round; its selections)"""
        eng.set_timing(True)
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for s in range(steps):
            out = step(first + s, ell=ell_)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        el = time.perf_counter() - t0
        # per-stage device times of the timed rounds (HIP events recorded on the
        # library's streams during the rounds, read once here)
        st_ms = {}
        for st in ("propose", "hash", "dedup", "encode", "prep", "fit_wait", "kstar", "bound", "prune", "var",
                   "var_wait", "finalize", "recompute", "topk", "outputs", "between"):
            try:
                st_ms[st] = eng.stage_time(st)
            except Exception:
                pass
        eng.set_timing(False)
        i8s = eng.gp_i8_stats() if args.precision == 8 else None
        if world > 1:
            t = torch.tensor([el], dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            el = float(t.item())
        return el, st_ms, i8s, out

    for w in range(args.warmup):
        step(w)
    torch.cuda.synchronize()
    elapsed, stages, i8_timed, (idx, top, sdig) = timed_rounds(args.warmup, args.steps, ell)

    # the secondary C2 line: the same round timed at ell = 2,
    # where k* spans (1e-3, 1), every K* digit plane carries data, EI values
    # spread and the top-k is decided by the scores (at the headline's ell =
    # 0.2 every k* underflows to ~1e-58: zero digit planes, index-order top-k)
    sec = None
    r_next = args.warmup + args.steps
    if args.secondary and args.config == "c2" and not args.prune and ell != 2.0:
        for w in range(max(1, args.warmup // 2)):
            step(r_next + w, ell=2.0)
        r_next += max(1, args.warmup // 2)
        sel2, st2, i8_2, out2 = timed_rounds(r_next, args.steps, 2.0)
        sec = {"lengthscale": 2.0, "first_round": r_next, "elapsed": sel2, "stages": st2, "i8": i8_2, "out": out2}
        r_next += args.steps

    # ---- the checker, outside the timed region ------------------------------
    parity = None
    if not args.no_parity and args.config == "c4" and rank == 0:
        rep = parity_ga_round(eng, oracle_space_of(manip), idx, top, sdig, parent, 1, args.warmup + args.steps - 1,
                              X, y, ell, 1e-8)
        parity = {"last_round": rep, "all_ok": rep["trials_equal"] and rep["valid"] and rep["digests_equal"] and
                  rep["ei_max_rel_err"] <= 1e-5}
    if not args.no_parity and args.config in ("c2", "c3"):
        r_last = args.warmup + args.steps - 1
        space = oracle_space_of(manip)
        jit = 0.0
        rep = None
        if rank == 0:
            rep, _, _ = parity_de_round(eng, space, idx, top, sdig, npop, 1, r_last, X, y, ell, jit, k)
        parity = {"last_round": rep}
        if args.config == "c2":
            # a round whose top-k the scores decide (ell = 2.0: EI values spread,
            # where the headline's ell = 0.2 makes every k* underflow to ~1e-58
            # and the selection is decided by index order): the secondary
            # line's last timed round, else one extra round
            if sec is not None:
                r_x = r_next - 1
                ix, tx, dx = sec["out"]
            else:
                r_x = r_next
                ix, tx, dx = step(r_x, ell=2.0)
            torch.cuda.synchronize()
            if rank == 0:
                rep2, _, ei_sel = parity_de_round(eng, space, ix, tx, dx, npop, 1, r_x, X, y, 2.0, jit, k)
                from oracle import de as ode
                from oracle import gp as ogp
                from oracle.space import features
                rng = np.random.default_rng(12345)
                chosen = set(ix.cpu().numpy().tolist())
                samp = rng.choice(npop, size=min(args.parity_sample, npop), replace=False)
                samp = np.array([g for g in samp if g not in chosen], dtype=np.int64)
                gp = ogp.GP(X, y, lengthscale=2.0, sigma_f2=1.0, sigma_n2=1e-6)
                mu, var = gp.posterior(features(space, ode.propose_de_at(space, samp, npop, 1, r_x, 0.2, 1)).T)
                ei_s = ogp.acquisition(mu, var, gp.f_best)
                kth = float(np.min(ei_sel)) if len(ei_sel) else float("inf")
                rep2.update({"lengthscale": 2.0, "sample": int(len(samp)),
                             "kth_selected_ei": kth, "best_unselected_sample_ei": float(np.max(ei_s)),
                             "topk_beats_sample": bool(np.max(ei_s) <= kth * (1.0 + 1e-5)),
                             "distinct_selected_scores": int(len(np.unique(tx.cpu().numpy()))),
                             # this round's merged selections: decided by the scores (all
                             # distinct), so equal shas across N check the cross-rank merge
                             "selection_sha": selection_sha(ix, dx)})
                parity["score_determined"] = rep2
        if rank == 0:
            legs = [v for v in parity.values() if v]
            parity["all_ok"] = all(v["trials_equal"] and v["digests_equal"] and v["ei_max_rel_err"] <= 1e-5 and
                                   v.get("topk_beats_sample", True) for v in legs)

    # the last timed round's merged selections, as one digest comparable across
    # N (strong scaling: the same at every N; weak: equal to a one-rank run
    # with --m N*m) -- computed outside the timed region
    sel_sha = selection_sha(idx, sdig)
    # device memory per rank: what libuthot holds on the rank's GPU (max over ranks)
    mem = torch.tensor([float(eng.device_bytes())], dtype=torch.float64)
    if world > 1:
        dist.all_reduce(mem, op=dist.ReduceOp.MAX)
    hbm_rank = int(mem.item())
    free_b, total_b = torch.cuda.mem_get_info(eng.device)

    ms_per_step = elapsed * 1000.0 / args.steps
    value = npop / (elapsed / args.steps)   # every candidate of the global pool, all ranks together
    # dominant kernel: the variance GEMM  V = L^-1 K*^T  (fp64 MFMA); at C4 (707
    # features) the K* contraction (2 n d flops per candidate) carries more flops
    var_ms = stages.get("var")
    flops_var = float(m) * n * (n + 1)       # algorithmic: lower-triangular n x n times k* per candidate
    kernel = ("k_gp_var_pp (persistent var contraction L^-1 K*^T, two 4-wave workgroups per CU, "
              "v_mfma_f64_16x16x4_f64)" if args.precision == 64 else
              "k_gp_var_f32 (persistent var contraction L^-1 K*^T, v_mfma_f32_32x32x2_f32)")
    if args.precision == 16:
        kernel = ("k_gp_var_h3 (persistent var contraction L^-1 K*^T, 3 x v_mfma_f32_32x32x16_f16 per product "
                  "on hi/lo fp16 splits; peak = fp16 dense peak / 3)")
    if args.precision == 8:
        kernel = ("k_gp_var_i8 (persistent var contraction L^-1 K*^T over six balanced int8 digit planes per "
                  "operand, %d v_mfma_i32_32x32x32_i8 digit products per multiply-add, exact int32 group sums; "
                  "peak = int8 dense peak / %d)" % (I8_PRODUCTS, I8_PRODUCTS))
    kstar_fp64 = False
    if args.config == "c4" and stages.get("kstar", 0.0) > (var_ms or 0.0):
        # (its stage time includes the hash running beside it on the second stream)
        var_ms = stages["kstar"]
        k64 = kstar_fp64_features(eng, d)
        flops_var = 2.0 * m * n * k64
        kstar_fp64 = True
        kernel = ("k_gp_kstar<double, false, true> (K* = exp(-|x - u|^2 / 2): v_mfma_f64_16x16x4_f64 over the %d "
                  "numeric features + the one-hot codes on v_mfma_i32_16x16x64_i8; its stage shares the chip with "
                  "the round's hash)" % k64)
    if args.prune and prune_stats:
        # a pruned round's dominant kernel is K* (with the mean in its epilogue):
        # its fp64 contraction over the features it contracts in fp64 (the
        # numeric ones in categorical mode; the one-hot blocks' int8 code
        # product beside it is not counted), its "kstar" stage without the wait
        # for the fit ("fit_wait")
        var_ms = stages.get("kstar")
        k64 = kstar_fp64_features(eng, d)
        flops_var = 2.0 * m * n * k64
        if args.prune_pass == 32:
            kernel = ("k_gp_kstar_f32c<%s> (the bound pass: K* with the mean k* . alpha in its epilogue, "
                      "v_mfma_f32_16x16x4f32 over %d features%s, k* by v_exp_f32, every rounding bounded; the "
                      "bound rows in fp64) [pruned round: the variance GEMM runs for the survivors only; peak = "
                      "the f32 MFMA's]" % ("true" if k64 < d else "false", k64,
                                            " + the one-hot codes on v_mfma_i32_16x16x64_i8" if k64 < d else ""))
        else:
            kernel = ("k_gp_kstar<double, true, %s> (K* with the mean k* . alpha in its epilogue, "
                      "v_mfma_f64_16x16x4_f64 over %d fp64 features%s) [pruned round: the variance GEMM runs for "
                      "the survivors only]" % ("true" if k64 < d else "false", k64,
                                               " + the one-hot codes on v_mfma_i32_16x16x64_i8" if k64 < d else ""))
    achieved = flops_var / (var_ms * 1e-3) / 1e12 if var_ms else None
    peak = {64: PEAK_FP64_TFLOPS, 32: PEAK_FP32_TFLOPS, 16: PEAK_FP16_TFLOPS / 3.0,
            8: PEAK_I8_TOPS / I8_PRODUCTS}[args.precision]
    if args.prune and args.prune_pass == 32:
        peak = PEAK_FP32_TFLOPS   # the bound pass's contraction runs on the f32 MFMA
    if kstar_fp64:
        peak = PEAK_FP64_TFLOPS
    # HBM bytes per launch and the rocprof average duration were profiled on the
    # default C2 round (profiles/pmc_summary.json)
    profiled = args.config == "c2" and (m, n, d) == (1 << 20, 1024, 64) and not args.prune
    var_key = {64: "var", 32: "var32", 16: "var16", 8: "var8"}[args.precision]

    def rocprof_of(key, ell_):
        """(HBM bytes per launch, roofline frac at the rocprof duration, source
        label) of a profiled C2 kernel at lengthscale ell_ (records of the ell =
        2 rounds carry the suffix _l2)"""
        if not profiled or ell_ not in (0.2, 2.0):
            return None, None, None
        rec, note = load_pmc(key + profile_suffix(ell_))
        if not rec:
            return None, None, None
        clk = load_clock().get(key + profile_suffix(ell_)) or {}
        dur = clk.get("duration_ms", 0.0) * 1e-3 or (rec.get("avg_ns") or 0.0) * 1e-9
        src = ("profiles/pmc_summary.json[%s] (HBM bytes: %s; duration: %s)" %
               (key + profile_suffix(ell_), rec.get("source") or note.split("source:")[-1].strip(),
                "profiles/clock_summary.json, %s" % clk.get("source", "?") if clk else "--kernel-trace --stats avg"))
        return rec.get("hbm_bytes_per_launch"), (flops_var / dur / 1e12 / peak) if dur > 0 else None, src

    traffic, frac_rocprof, rocprof_src = rocprof_of(var_key, ell)
    i8_info = None
    if args.precision == 8:
        rec, bound_e = eng.gp_i8_stats()   # the last round run: the score-determined parity round when it ran
        _, bound_emu = eng.gp_i8_bounds()
        i8_info = {"recomputed_fp64_last_timed_round": i8_timed[0], "bound_E": i8_timed[1],
                   "bound_Emu_last_round_run": bound_emu,
                   "recomputed_fp64_last_round_run": rec, "bound_E_last_round_run": bound_e, "digit_planes": 6,
                   "products": I8_PRODUCTS, "tolerance": 2.0 ** -20,
                   "note": "variance error per candidate <= E (2 |v| + E) (+ f64 rounding), mean (v . L^-1 y from "
                           "the int8 variance epilogue) error <= Emu; accepted iff those are <= tolerance * var and "
                           "<= tolerance * sigma, else recomputed on the f64 path (gp_i8.hip)"}
    prune_info = None
    if args.prune and prune_stats:
        timed = prune_stats[-args.steps:]
        prune_info = {"bound_rows": timed[-1]["bound_rows"], "bound_pass": args.prune_pass,
                      "survivor_frac": float(np.mean([s["survivors"] / m for s in timed])),
                      "dense_rounds": int(sum(s["dense"] for s in timed)),
                      "dense_equivalent_tflops": float(m) * n * (n + 1) / (elapsed / args.steps) / 1e12,
                      "note": "selection-exact: every pruned candidate's exact score is below the k-th best "
                              "(ut_gp_topk_pruned); value counts all m candidates of a round"}
    if args.config == "c4":
        workload = (f"C4 gcc flags (339 params: 1 + 154 Int, 184 Enum{{on,off,default}}; {d} GP features): GA "
                    f"mutation 0.1 from the best recorded config + hash_config + dedup vs 3,680 recorded configs "
                    f"+ GP-EI n={n} (recorded qor) + top-{k}, {m} candidates per GPU")
        data = ("recorded (samples/gcc-options/matmul-record.csv via tests/golden/gcc_history.npz: history, "
                "GP training configs and qor); proposals synthetic")
    elif args.config == "c3":
        workload = (f"C3 HPL-64 mixed (24 Int, 16 Enum, 8 Bool, 8 Float, 4 LogInt, 4 Pow2; {d} GP features): "
                    f"DE-Alt + hash_config + dedup + GP-EI n={n} + top-{k}, {m} candidates per GPU")
        data = "synthetic (HPL-64 configs from op1_randomize; objective = |features - 0.3|^2; population random-init)"
    else:
        workload = f"C2 R64: DE-Alt + hash_config + dedup + GP-EI n={n} + top-{k}"
        data = "synthetic (Rosenbrock-64 objective on uniform training points; DE population random-init)"
    if args.prune:
        workload += f", EI-bound pruned (first {args.prune} rows of L^-1 k* as the bound)"
    result = {
        "metric": "candidate configs scored/sec (GP-EI + top-k)",
        "value": value,
        "unit": "candidates/s",
        "n_gpus": n_gpus,
        "world": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": args.scaling,
        "vs_baseline": None,
        "dtype": {64: "f64", 32: "f32 (variance L^-1 K*^T on fp32 MFMA; K* contracted in fp64, stored f32; "
                      "fit/mean/EI f64)",
                  16: "f32-tier f16x3 (L^-1 K*^T as hi*hi + hi*lo + lo*hi fp16 MFMA, f32 accumulate; "
                      "K*/fit/EI f64)",
                  8: "f64-tier (int8 Ozaki slices: L^-1 K*^T over 6 balanced 8-bit digit planes, exact int32 "
                     "sums, per-candidate error bound <= 2^-20 relative on the variance, the rest recomputed in "
                     "f64; K*/mean/fit/EI f64)"}[args.precision],
        "data": data,
        "config": {"workload": workload, "candidates_per_gpu": m, "global_pool": npop, "gp_n": n, "dims": d,
                   "k": k, "parallelism": f"dp{world}", "scaling": args.scaling,
                   "exchange": (None if world == 1 else "libuthot RCCL (ut_comm_allgather_topk + HIP merge)"
                                if comm is not None else (exchange_note or "gloo records + HIP merge (rehearsal)"))},
        "parity": parity,
        "selection_sha": sel_sha,
        "hbm_bytes_per_rank": hbm_rank,
        "hbm_device_used_bytes": int(total_b - free_b),
        "stage_ms": stages,
        "kernels": (kernel_table(m, n, d, eng.space_info()[1], args.precision, profile_suffix(ell))
                    if profiled else None),
        "prune": prune_info,
        "i8": i8_info,
        "roofline": {"bound": "mfma", "kernel": kernel,
                     "achieved": achieved, "peak": peak, "unit": "TFLOP/s",
                     "frac": (achieved / peak) if achieved else None, "traffic": traffic,
                     "frac_rocprof": frac_rocprof, "rocprof_source": rocprof_src,
                     "flops_per_launch": flops_var},
        "cpu_baseline": None,
    }
    if sec is not None:
        # the secondary line: the same C2 rounds at ell = 2 (every K* digit plane
        # non-zero, score-determined top-k), timed like the headline
        v2_ms = sec["stages"].get("var")
        a2 = flops_var / (v2_ms * 1e-3) / 1e12 if v2_ms else None
        t2, f2r, s2 = rocprof_of(var_key, 2.0)
        sd = (parity or {}).get("score_determined") or {}
        result["secondary_ell2"] = {
            "lengthscale": 2.0, "rounds": [sec["first_round"], sec["first_round"] + args.steps - 1],
            "value": npop / (sec["elapsed"] / args.steps), "unit": "candidates/s",
            "ms_per_step": sec["elapsed"] * 1000.0 / args.steps, "steps": args.steps,
            "stage_ms": sec["stages"],
            "roofline": {"kernel": kernel, "achieved": a2, "peak": peak, "unit": "TFLOP/s",
                         "frac": (a2 / peak) if a2 else None, "traffic": t2, "frac_rocprof": f2r,
                         "rocprof_source": s2},
            "i8": ({"recomputed_fp64_last_timed_round": sec["i8"][0], "bound_E": sec["i8"][1]}
                   if sec["i8"] else None),
            "kernels": kernel_table(m, n, d, eng.space_info()[1], args.precision, "_l2") if profiled else None,
            "parity": ({"round": sd.get("round"), "all_ok": bool(sd.get("trials_equal") and sd.get("digests_equal")
                                                                 and sd.get("ei_max_rel_err", 1.0) <= 1e-5
                                                                 and sd.get("topk_beats_sample")),
                        "note": "the last timed round of this line is parity.score_determined"} if sd else None),
        }
    if rank == 0 and world == 1 and not args.no_cpu_baseline and args.config == "c2":
        host = host_info()
        result["host"] = host
        try:       # B1: the batch port on this job's host cores (the stronger CPU baseline)
            if args.b1_sample > 0:
                result["cpu_baseline"] = cpu_baseline_b1(args.b1_sample, n, d, k, host["threads"])
        except Exception as ex:  # keep the GPU number even if the baseline fails
            result["cpu_baseline"] = {"error": repr(ex)}
        try:       # the same B1 on every CPU of the job's affinity mask (the box's OMP_NUM_THREADS is 16)
            if args.b1_sample > 0 and host["affinity_cpus"] > host["threads"]:
                # (a 4x larger sample: every thread gets rows to work on)
                result["cpu_baseline_full_affinity"] = cpu_baseline_b1(4 * args.b1_sample, n, d, k,
                                                                       host["affinity_cpus"])
        except Exception as ex:
            result["cpu_baseline_full_affinity"] = {"error": repr(ex)}
        try:       # the reference's per-candidate, single-threaded search loop (api.py:428-446)
            if args.cpu_sample > 0:
                result["cpu_baseline_1thread"] = cpu_baseline(args.cpu_sample, n, d, k)
        except Exception as ex:
            result["cpu_baseline_1thread"] = {"error": repr(ex)}
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.barrier()
        if comm is not None:
            comm.close()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
