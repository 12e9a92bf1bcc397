#!/bin/bash
# round 3: how much of the C3 rounds the per-round GP refit costs (n = 4096):
# the bench with a refit every round against the same with the fit done once
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/fitcost
mkdir -p $O
for spec in "p --prune 256" "h --precision 16"; do set -- $spec; tag=$1; shift
  for prog in bench.py scripts/exp/bench_fit_once.py; do
    timeout -k 10 300 python $prog --config c3 $* --steps 5 --warmup 2 --no-cpu-baseline --no-parity > $O/x.log 2>&1 || { echo "$tag $prog rc=$?"; tail -5 $O/x.log; exit 1; }
    python3 -c "import json; d=json.loads([l for l in open('$O/x.log') if l.startswith('{')][-1]); print('$tag $prog', round(d['ms_per_step'],2), {k: round(v,2) for k,v in d['stage_ms'].items()})"
  done
done
