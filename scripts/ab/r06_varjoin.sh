#!/bin/bash
# (the UTX_* knobs were removed after the measurement: the i8 variance GEMM no longer joins the hash;
#  K* after the hash and the encode launched first were not kept -- profiles/r06_sched_ab.txt)
# round 6 A/B: the C2 round's variance GEMM waiting for the side stream's hash
# + dedup (UTX_VAR_JOIN=1, as before) or starting when K* and the fit are done
# (0; the finalize still joins the dup mask), at ell 0.2 and 2
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r06_varjoin; mkdir -p $O
for rep in 1 2; do
for v in 1 0; do
for ell in 0.2 2; do
  UTX_VAR_JOIN=$v timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-secondary --no-parity \
    --ell $ell > $O/j${v}_l${ell}_$rep.log 2>&1 || { tail -20 $O/j${v}_l${ell}_$rep.log; exit 1; }
  python -c "
import json; l=[x for x in open('$O/j${v}_l${ell}_$rep.log') if x.startswith('{')][-1]; j=json.loads(l)
st=j['stage_ms']
print('join=$v ell=$ell rep $rep', round(j['ms_per_step'],3), {k: round(v,2) for k,v in st.items()})"
done
done
done
