#!/bin/bash
# (not kept: 16.49-16.54 / 19.48-19.75 ms against 16.19-16.30 / 19.16-19.31; the knob was removed -- profiles/r06_kq_ab.txt)
# round 6 A/B: with the int8 K*, only the outer hash (one-shot workgroups) held
# until the refit is done (UTX_HOLD_OUTER=1); the inner digests run at once
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r06_holdouter; mkdir -p $O
for rep in 1 2; do
for v in 1 0; do
for ell in 0.2 2; do
  f=$O/h${v}_l${ell}_$rep.log
  if [ $v = 1 ]; then export UTX_HOLD_OUTER=1; else unset UTX_HOLD_OUTER; fi
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline \
    --no-secondary --no-parity --ell $ell > $f 2>&1 || { tail -20 $f; exit 1; }
  python -c "
import json; l=[x for x in open('$f') if x.startswith('{')][-1]; j=json.loads(l)
print('holdouter=$v ell=$ell rep $rep', round(j['ms_per_step'],3), {k: round(v,2) for k,v in j['stage_ms'].items()})"
done
done
done
