#!/bin/bash
# rocprofv3 kernel trace + stats of the C5 bandit loop (ARGS, e.g. --prune 256)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/prof_c5${TAG:+_$TAG}
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- \
  python3 scripts/c5_bandit.py $ARGS > $OUT/trace.log 2>&1 || { echo "trace rc=$?"; exit 1; }
tail -1 $OUT/trace.log | cut -c1-400
python3 - "$OUT/trace/run_kernel_stats.csv" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
tot = sum(float(r['TotalDurationNs']) for r in rows)
print(f"total kernel time {tot/1e6:.1f} ms")
for r in rows[:16]:
    print(f"{r['Name'][:58]:58s} {r['Calls']:>6} {float(r['TotalDurationNs'])/1e6:9.1f} ms total")
PY
