#!/bin/bash
# rocprofv3 kernel trace of the default C2 bench with every kernel launch
# serialised (AMD_SERIALIZE_KERNEL=3): per-kernel standalone durations, no
# side-stream overlap inflating them.  EXTRA_ENV (e.g. UT_VAR_KERNEL=1) and
# TAG name a second configuration.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp AMD_SERIALIZE_KERNEL=3
OUT=gpurun_out/prof_serial${TAG:+_$TAG}
mkdir -p $OUT
ARGS=${BENCH_ARGS:---steps 4 --warmup 1 --no-cpu-baseline}
[ -n "$EXTRA_ENV" ] && export $EXTRA_ENV
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- \
  python3 bench.py $ARGS > $OUT/trace.log 2>&1 || { echo "trace rc=$?"; exit 1; }
echo trace ok; tail -1 $OUT/trace.log | cut -c1-300
python3 - "$OUT/trace/run_kernel_stats.csv" <<'PY'
import csv, sys
for r in list(csv.DictReader(open(sys.argv[1])))[:14]:
    print(f"{r['Name'][:58]:58s} {r['Calls']:>4} {float(r['AverageNs'])/1e3:9.1f} us")
PY
