#!/bin/bash
# (not kept; the UTX_* knobs were removed after the measurement -- profiles/r06_kq_ab.txt)
# round 6 A/B (5): with the int8 K*, the hash's grids one-shot (one pass per
# workgroup, UT_HASH_WG_PER_CU=64: workgroups retire and free their slots)
# with and without the fit stream at the greatest priority (UTX_FIT_PRIO)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r06_kq5; mkdir -p $O
for v in "0 -1" "0 64" "1 64" "1 16"; do
set -- $v
for ell in 0.2 2; do
  f=$O/p$1_w$2_l${ell}.log
  UTX_FIT_PRIO=$1 UT_HASH_WG_PER_CU=$2 timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline \
    --no-secondary --no-parity --ell $ell > $f 2>&1 || { tail -20 $f; exit 1; }
  python -c "
import json; l=[x for x in open('$f') if x.startswith('{')][-1]; j=json.loads(l)
print('prio=$1 wg=$2 ell=$ell', round(j['ms_per_step'],3), {k: round(v,2) for k,v in j['stage_ms'].items()})"
done
done
