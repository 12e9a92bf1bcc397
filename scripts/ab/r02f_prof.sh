#!/bin/bash
# rocprofv3 kernel trace + stats of the C4 bench and of one C5 dense bandit run
# (per-kernel time split of the two workloads other than C2).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/prof
mkdir -p $OUT
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/c4 -o run --output-format csv -- \
  python3 bench.py --config c4 --steps 3 --warmup 1 --no-cpu-baseline > $OUT/c4.log 2>&1 || { echo "c4 rc=$?"; exit 1; }
echo c4 ok; tail -1 $OUT/c4.log | cut -c1-200
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/c5 -o run --output-format csv -- \
  python3 scripts/c5_bandit.py > $OUT/c5.log 2>&1 || { echo "c5 rc=$?"; exit 1; }
echo c5 ok; tail -1 $OUT/c5.log | cut -c1-200
find $OUT -name "*stats*.csv"
