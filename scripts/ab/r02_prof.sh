#!/bin/bash
# rocprofv3 kernel trace + stats of the default C2 bench (one pass), then HBM
# byte counters in separate passes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/prof
mkdir -p $OUT
ARGS=${BENCH_ARGS:---steps 4 --warmup 1 --no-cpu-baseline}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- \
  python3 bench.py $ARGS > $OUT/trace.log 2>&1 || { echo "trace rc=$?"; exit 1; }
echo trace ok; tail -1 $OUT/trace.log | cut -c1-300
[ -n "$NO_PMC" ] && exit 0
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch -o run --output-format csv -- \
  python3 bench.py $ARGS > $OUT/pmc_fetch.log 2>&1 || { echo "fetch rc=$?"; exit 1; }
echo fetch ok
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_write -o run --output-format csv -- \
  python3 bench.py $ARGS > $OUT/pmc_write.log 2>&1 || { echo "write rc=$?"; exit 1; }
echo write ok
find $OUT -name "*stats*.csv" -o -name "*counter*.csv" | head -20
