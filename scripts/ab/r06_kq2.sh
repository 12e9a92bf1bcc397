#!/bin/bash
# (not kept; the UTX_* knobs were removed after the measurement -- profiles/r06_kq_ab.txt)
# round 6 A/B (2): with the int8 K* (gp_kq.hip) the variance GEMM waits for the
# refit (var_wait): the fit stream at the greatest priority (UTX_FIT_PRIO=1),
# the hash capped at 4 workgroups per CU (UT_HASH_WG_PER_CU=4), both, neither
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r06_kq2; mkdir -p $O
for cfgv in "0 -1" "1 -1" "0 4" "1 4"; do
set -- $cfgv
for ell in 0.2 2; do
  f=$O/p$1_c$2_l${ell}.log
  UTX_FIT_PRIO=$1 UT_HASH_WG_PER_CU=$2 timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline \
    --no-secondary --no-parity --ell $ell > $f 2>&1 || { tail -20 $f; exit 1; }
  python -c "
import json; l=[x for x in open('$f') if x.startswith('{')][-1]; j=json.loads(l)
print('prio=$1 cap=$2 ell=$ell', round(j['ms_per_step'],3), {k: round(v,2) for k,v in j['stage_ms'].items()})"
done
done
