#!/bin/bash
# round 6 A/B (4): with the int8 K* the variance GEMM waits ~1.7 ms for the
# refit (var_wait): the refit's fused Cholesky update (UT_CHOL_FUSE=1, fewer
# launches in its chain) against the default (fused from 2048 rows only)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r06_kq4; mkdir -p $O
for rep in 1 2; do
for v in 1 -1; do
for ell in 0.2 2; do
  f=$O/f${v}_l${ell}_$rep.log
  UT_CHOL_FUSE=$v timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline \
    --no-secondary --no-parity --ell $ell > $f 2>&1 || { tail -20 $f; exit 1; }
  python -c "
import json; l=[x for x in open('$f') if x.startswith('{')][-1]; j=json.loads(l)
print('fuse=$v ell=$ell rep $rep', round(j['ms_per_step'],3), {k: round(v,2) for k,v in j['stage_ms'].items()})"
done
done
done
