#!/bin/bash
# round 6 A/B (knob removed after it: held rounds 18.5-18.7 vs 16.9-17.1 ms at ell 0.2, 21.0-21.4 vs 19.8-20.1 at ell 2):
# the C2 round's hash held until the refit is done (UT_HASH_HOLD=1)
# against the default (precision-8 rounds do not hold), at ell = 0.2 and 2
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r06_hashhold; mkdir -p $O
for rep in 1 2; do
for ell in 0.2 2; do
for v in 0 1; do
  UT_HASH_HOLD=$v timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-secondary --ell $ell \
    > $O/h${v}_l${ell}_$rep.log 2>&1 || { tail -20 $O/h${v}_l${ell}_$rep.log; exit 1; }
  python -c "
import json; l=[x for x in open('$O/h${v}_l${ell}_$rep.log') if x.startswith('{')][-1]; j=json.loads(l)
print('hold=$v ell=$ell rep $rep', round(j['ms_per_step'],3), j['parity'].get('all_ok'), {k: round(v,2) for k,v in j['stage_ms'].items()})"
done
done
done
