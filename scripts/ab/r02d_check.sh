#!/bin/bash
# Round-2 (third session) round trip: GPU tests, smoke, C2 bench (with both CPU
# baselines), C4 bench, then C5 dense and pruned (a warm-up run first: the first
# process on a fresh box pays code-object loading).  Each GPU step has its own
# limit; a failure ends the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
SKIP_C4=1 bash scripts/ab/r02_check.sh || exit $?
timeout -k 10 300 python bench.py --config c4 --steps 5 --warmup 2 > gpurun_out/bench_c4.log 2>&1 || exit 1
tail -1 gpurun_out/bench_c4.log | cut -c1-120
timeout -k 10 200 python scripts/c5_bandit.py --prune 256 > /dev/null 2>&1 || exit 1
timeout -k 10 200 python scripts/c5_bandit.py --prune 256 > gpurun_out/c5_prune.log 2>&1 || exit 1
tail -1 gpurun_out/c5_prune.log | cut -c1-120
timeout -k 10 300 python scripts/c5_bandit.py > gpurun_out/c5_dense.log 2>&1 || exit 1
tail -1 gpurun_out/c5_dense.log | cut -c1-120
