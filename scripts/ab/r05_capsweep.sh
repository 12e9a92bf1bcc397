#!/bin/bash
# round 5: the hash grid cap while the refit runs (UT_HASH_WG_PER_CU; -1 = the
# default rule: 4 per CU while an n >= 2048 fit is in flight), C3 pruned line
# after the f32 bound pass.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r05_capsweep; mkdir -p $O
for rep in 1 2; do
for cap in -1 2 1 8; do
  UT_HASH_WG_PER_CU=$cap timeout -k 10 300 python bench.py --config c3 --prune 256 --steps 5 --warmup 2 \
    --no-cpu-baseline --no-parity > $O/c3p_${cap}_$rep.log 2>&1 || { tail -20 $O/c3p_${cap}_$rep.log; exit 1; }
  python -c "
import json; l=[x for x in open('$O/c3p_${cap}_$rep.log') if x.startswith('{')][-1]; j=json.loads(l)
print('cap $cap rep $rep', round(j['ms_per_step'],3), {k: round(v,2) for k,v in j['stage_ms'].items()})"
done
done
