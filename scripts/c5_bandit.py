#!/usr/bin/env python
"""C5 (BASELINE.json configs[4]): AUC bandit over GPU DE + PSO + GA + GGA with a
shared GP surrogate on Rosenbrock-64, one process per GPU, per-generation
results broadcast over RCCL.

    python scripts/c5_bandit.py --generations 100                      # 1 GPU
    python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 \\
        --master-addr 127.0.0.1 --master-port 29511 scripts/c5_bandit.py   # 8 GPUs

Rank 0 prints one JSON line: generations, evaluations, best objective, wall
time, scoring rounds (and rounds/s), GP fits of the shared model, candidates
scored per second (all ranks), and the same engine's stand-alone round rate
at the final training-set size (one DE round of `pool` candidates: propose,
hash, dedup, encode, GP-EI, top-k), so the loop's overhead over the kernels
is visible as end_to_end_vs_round.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def rosenbrock64(cfg):
    x = np.array([cfg[i] for i in range(64)], dtype=np.float64) / 500.0   # [-2, 2]
    return float(np.sum(100.0 * (x[1:] - x[:-1] ** 2) ** 2 + (x[:-1] - 1.0) ** 2))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--generations", type=int, default=100)
    ap.add_argument("--parallelism", type=int, default=4)
    ap.add_argument("--n-init", type=int, default=4096, help="initial design = the shared GP's bootstrap set")
    ap.add_argument("--pool", type=int, default=1 << 18, help="candidates per technique round per GPU")
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--population", type=int, default=4096)
    ap.add_argument("--backend", default="nccl")
    ap.add_argument("--precision", type=int, default=None, choices=(64, 32, 16, 8),
                    help="the shared GP's contractions: 8 = the fp64 tier on the int8 MFMA (the default for dense "
                         "rounds, as the bench's), 64 = the fp64 MFMA (the default with --prune, which needs it)")
    ap.add_argument("--prune", type=int, default=0, metavar="ROWS",
                    help="score technique rounds with the selection-exact EI-bound pruning (fp64)")
    ap.add_argument("--warmup-generations", type=int, default=3,
                    help="an untimed short run first (same process): library load, first launches of every "
                         "kernel, allocator growth -- the timed run is the steady-state loop")
    args = ap.parse_args()
    if args.precision is None:
        args.precision = 64 if args.prune else 8

    import torch
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    if world > 1:
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(args.backend)
    from uptune_amd import spaces
    from uptune_amd.tuner import tune_bandit

    if args.warmup_generations > 0:
        tune_bandit(spaces.r64(), rosenbrock64, generations=args.warmup_generations, parallelism=args.parallelism,
                    n_init=min(args.n_init, 512), pool=args.pool, batch=args.batch, population=args.population,
                    seed=2, lengthscale=0.3, device=local, precision=args.precision, prune_rows=args.prune)
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    drv = tune_bandit(spaces.r64(), rosenbrock64, generations=args.generations, parallelism=args.parallelism,
                      n_init=args.n_init, pool=args.pool, batch=args.batch, population=args.population, seed=1,
                      lengthscale=0.3, device=local, precision=args.precision, prune_rows=args.prune)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    techs = drv.root_technique.techniques
    rounds = {t.name: t.round for t in techs}
    scored = sum(t.round * (t.pool * (world if t.sharded else 1) if t.sharded else min(t.pool, t.population))
                 for t in techs)
    # the stand-alone round rate of the same engine at the final training set
    model = techs[0].model
    de = [t for t in techs if t.name == "gpu-de"][0]
    eng = model.engine_for(de)
    acq = eng.acq("ei")
    model.fit(drv)
    rr = []
    for r in range(3):
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        v = eng.propose_de(args.pool, round_=10000 + r, cand_base=0)
        dg = eng.hash_de(v, 0)
        dup = eng.dedup(dg)
        if args.prune:
            eng.gp_topk_pruned(eng.encode(v), args.batch, acq=acq, dup=dup, bound_rows=args.prune)
        else:
            _, _, sc = eng.gp_score(eng.encode(v), acq=acq, dup=dup)
            eng.topk(sc, args.batch, dup=dup)
        torch.cuda.synchronize()
        rr.append(time.perf_counter() - t1)
    round_rate = args.pool / min(rr)
    # the stand-alone rate of the loop's own technique mix: each technique's
    # round (_local_round: propose, hash, dedup, score, local top-k) timed at the
    # final model, weighted by how many rounds the bandit gave it (the DE round
    # above is the cheapest kind; PSO rounds move only the swarm)
    mix_s, mix_c, per_tech = 0.0, 0, {}
    for t in techs:
        if t.round == 0:
            continue
        cands = t.pool if t.sharded else min(t.pool, t.population)
        ts = []
        for _ in range(3):
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            t._local_round()
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t1)
        per_tech[t.name] = {"rounds": t.round, "candidates": cands, "ms": min(ts) * 1e3}
        mix_s += t.round * min(ts)
        mix_c += t.round * cands
    mix_rate = mix_c / mix_s if mix_s else None
    n_train = len(drv.results_query())
    out = {"config": "C5 AUC bandit over GPU DE+PSO+GA+GGA, shared GP, Rosenbrock-64"
                     + (f", EI-bound pruned ({args.prune} rows)" if args.prune else ""), "n_gpus": world,
           "precision": args.precision,
           "generations": drv.generation, "evaluations": len(drv.results) - args.n_init,
           "initial_design": args.n_init, "best": drv.best_result.time if drv.best_result else None,
           "wall_s": wall, "warmup_generations": args.warmup_generations, "technique_rounds": rounds, "rounds_per_s": sum(rounds.values()) / wall,
           "gp_fits": model.fits, "gp_n_final": n_train, "candidates_scored": scored,
           "candidates_scored_per_s": scored / wall,
           # the generation loop alone (wall minus the initial design's draw + evaluation)
           "seed_s": drv.seed_s, "loop_candidates_scored_per_s": scored / (wall - drv.seed_s),
           "round_rate_candidates_per_s": round_rate * (world if world > 1 else 1),
           "end_to_end_vs_round": (scored / wall) / (round_rate * (world if world > 1 else 1)),
           "technique_round_ms": per_tech,
           "mix_round_rate_candidates_per_s": mix_rate * (world if world > 1 else 1) if mix_rate else None,
           "end_to_end_vs_mix": (scored / wall) / (mix_rate * (world if world > 1 else 1)) if mix_rate else None,
           "bandit_uses": dict(drv.root_technique.bandit.use_counts)}
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
