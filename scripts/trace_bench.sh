#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/tr
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/tr -o run --output-format csv -- python3 bench.py ${BENCH_ARGS:---steps 3 --warmup 1 --no-cpu-baseline} > gpurun_out/tr/log 2>&1 || { echo "rc=$?"; tail -5 gpurun_out/tr/log; exit 1; }
tail -1 gpurun_out/tr/log
