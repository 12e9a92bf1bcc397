#!/bin/bash
# round 6 A/B: the C2 round's hash grids capped at 1 / 2 / 3 workgroups per CU
# (UT_HASH_WG_PER_CU; -1 = the default, uncapped at n = 1024) now that the
# int8 variance GEMM starts when K* ends
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r06_hashcap; mkdir -p $O
for v in -1 1 2 3; do
for ell in 0.2 2; do
  f=$O/c${v}_l${ell}.log
  UT_HASH_WG_PER_CU=$v timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-secondary \
    --no-parity --ell $ell > $f 2>&1 || { tail -20 $f; exit 1; }
  python -c "
import json; l=[x for x in open('$f') if x.startswith('{')][-1]; j=json.loads(l)
print('cap=$v ell=$ell', round(j['ms_per_step'],3), {k: round(v,2) for k,v in j['stage_ms'].items()})"
done
done
