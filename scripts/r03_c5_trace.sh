#!/bin/bash
# round 3: kernel trace of the C5 pruned loop (device busy vs idle per generation)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/c5trace
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT -o run --output-format csv -- python3 scripts/c5_bandit.py --generations 100 --prune 256 > $OUT/log 2>&1
rc=$?; echo "trace rc=$rc"; tail -c 800 $OUT/log; exit $rc
