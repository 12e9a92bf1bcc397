#!/usr/bin/env python
"""Host-time profile of the C5 loop (scripts/c5_bandit.py's tune_bandit run)
under cProfile: where the generation loop spends its wall time outside the
device rounds.  Writes the cumulative / own-time tables to gpurun_out/."""
import cProfile
import io
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    prune = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    import torch
    from scripts.c5_bandit import rosenbrock64
    from uptune_amd import spaces
    from uptune_amd.tuner import tune_bandit
    torch.cuda.set_device(0)
    # warm: one short run (library load, kernels, allocator)
    tune_bandit(spaces.r64(), rosenbrock64, generations=5, parallelism=4, n_init=512, pool=1 << 18, batch=8,
                population=4096, seed=1, lengthscale=0.3, prune_rows=prune)
    torch.cuda.synchronize()
    pr = cProfile.Profile()
    t0 = time.perf_counter()
    pr.enable()
    drv = tune_bandit(spaces.r64(), rosenbrock64, generations=100, parallelism=4, n_init=4096, pool=1 << 18,
                      batch=8, population=4096, seed=1, lengthscale=0.3, prune_rows=prune)
    torch.cuda.synchronize()
    pr.disable()
    wall = time.perf_counter() - t0
    os.makedirs("gpurun_out", exist_ok=True)
    for key in ("cumulative", "tottime"):
        s = io.StringIO()
        pstats.Stats(pr, stream=s).sort_stats(key).print_stats(45)
        with open(f"gpurun_out/prof_c5_host_{key}.txt", "w") as f:
            f.write(f"wall {wall:.3f} s, seed {drv.seed_s:.3f} s, best {drv.best_result.time}\n")
            f.write(s.getvalue())
    print(f"wall {wall:.3f} s seed {drv.seed_s:.3f} s best {drv.best_result.time}")


if __name__ == "__main__":
    main()
