#!/bin/bash
# round 6: FETCH_SIZE calibration of k_de's access widths (fetch_calib.hip)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r06_fetchcal; mkdir -p $O
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $O/f -o run --output-format csv -- ./scripts/exp/fetch_calib > $O/log 2>&1 || { echo failed; tail $O/log; exit 1; }
cat $O/log | tail -1
python3 - <<PY
import csv
from collections import defaultdict
acc=defaultdict(list)
for r in csv.DictReader(open('$O/f/run_counter_collection.csv')):
    if r['Counter_Name']=='FETCH_SIZE': acc[r['Kernel_Name'][:40]].append(float(r['Counter_Value'])*1024)
for k,v in acc.items(): print(k, ['%.3f GB' % (x/1e9) for x in v])
PY
