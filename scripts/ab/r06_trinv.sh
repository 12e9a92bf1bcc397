#!/bin/bash
# round 6 A/B: the refit gates the C2 variance GEMM (var_wait); its largest
# L^-1 level (512 x 512, 16 workgroups of 128 x 128 on k_trinv_big) against
# 64 x 64 tiles (k_trinv_level, 64 workgroups: UT_TRINV_BIG=0)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r06_trinv; mkdir -p $O
for rep in 1 2; do
for v in 0 1; do
for ell in 0.2 2; do
  f=$O/t${v}_l${ell}_$rep.log
  UT_TRINV_BIG=$v timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline \
    --no-secondary --no-parity --ell $ell > $f 2>&1 || { tail -20 $f; exit 1; }
  python -c "
import json; l=[x for x in open('$f') if x.startswith('{')][-1]; j=json.loads(l)
print('trinv_big=$v ell=$ell rep $rep', round(j['ms_per_step'],3), {k: round(v,2) for k,v in j['stage_ms'].items()})"
done
done
done
