#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --precision 64 > gpurun_out/bench64.log 2>&1 || { echo "bench64 rc=$?"; tail -5 gpurun_out/bench64.log; exit 1; }
tail -1 gpurun_out/bench64.log
timeout -k 10 600 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --precision 32 > gpurun_out/bench32.log 2>&1 || { echo "bench32 rc=$?"; tail -5 gpurun_out/bench32.log; exit 1; }
tail -1 gpurun_out/bench32.log
