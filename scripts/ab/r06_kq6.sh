#!/bin/bash
# round 6 A/B (6): with the int8 K* (the refit now gates the variance GEMM),
# the staged fit issued at ut_gp_fit_async (UT_FIT_DEFER=0: it starts beside the
# previous round's top-k) against after the proposal (1)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r06_kq6; mkdir -p $O
for rep in 1 2; do
for v in 0 1; do
for ell in 0.2 2; do
  f=$O/d${v}_l${ell}_$rep.log
  UT_FIT_DEFER=$v timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline \
    --no-secondary --no-parity --ell $ell > $f 2>&1 || { tail -20 $f; exit 1; }
  python -c "
import json; l=[x for x in open('$f') if x.startswith('{')][-1]; j=json.loads(l)
print('defer=$v ell=$ell rep $rep', round(j['ms_per_step'],3), {k: round(v,2) for k,v in j['stage_ms'].items()})"
done
done
done
