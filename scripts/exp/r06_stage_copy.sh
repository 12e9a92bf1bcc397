#!/bin/bash
# round 6: C4 and C3 rounds with the fit's training rows staged by 8 threads
# (gp.hip stage_copy): the "between" stage (device idle between rounds)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r06_stage_copy; mkdir -p $O
for cfg in c4 c3; do
  f=$O/$cfg.log
  timeout -k 10 300 python bench.py --config $cfg --steps 5 --warmup 2 --no-cpu-baseline --no-secondary --no-parity \
    > $f 2>&1 || { tail -20 $f; exit 1; }
  python -c "
import json; l=[x for x in open('$f') if x.startswith('{')][-1]; j=json.loads(l)
print('$cfg', round(j['ms_per_step'],3), {k: round(v,2) for k,v in j['stage_ms'].items()})"
done
