#!/bin/bash
# round 3: kernel trace of a few rounds (BENCH_ARGS) for a round timeline
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/timeline${TAG}
mkdir -p $OUT
ARGS=${BENCH_ARGS:---precision 16 --steps 3 --warmup 1 --no-cpu-baseline --no-parity}
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT -o run --output-format csv -- python3 bench.py $ARGS > $OUT/bench.log 2>&1
rc=$?; echo "trace rc=$rc"; tail -c 600 $OUT/bench.log; exit $rc
