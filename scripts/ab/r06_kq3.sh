#!/bin/bash
# (not kept; the UTX_* knobs were removed after the measurement -- profiles/r06_kq_ab.txt)
# round 6 A/B (3): with the int8 K*, the round's hash held until the refit is
# done (UTX_HOLD8=1) against not held, and the fp64-MFMA K* (UT_KSTAR_Q=0)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r06_kq3; mkdir -p $O
for rep in 1 2; do
for v in "q1 h0" "q1 h1" "q0 h0"; do
set -- $v
for ell in 0.2 2; do
  f=$O/$1$2_l${ell}_$rep.log
  if [ $2 = h1 ]; then export UTX_HOLD8=1; else unset UTX_HOLD8; fi
  UT_KSTAR_Q=${1#q} timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline \
    --no-secondary --no-parity --ell $ell > $f 2>&1 || { tail -20 $f; exit 1; }
  python -c "
import json; l=[x for x in open('$f') if x.startswith('{')][-1]; j=json.loads(l)
print('$1 $2 ell=$ell rep $rep', round(j['ms_per_step'],3), {k: round(v,2) for k,v in j['stage_ms'].items()})"
done
done
done
