#!/bin/bash
# (the UTX_* knobs were removed after the measurement: the i8 variance GEMM no longer joins the hash;
#  K* after the hash and the encode launched first were not kept -- profiles/r06_sched_ab.txt)
# round 6 A/B (2): UTX_VAR_JOIN on the C3 dense f64-tier and C4 lines
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r06_varjoin2; mkdir -p $O
for v in 1 0; do
for cfg in c4 c3; do
  UTX_VAR_JOIN=$v timeout -k 10 300 python bench.py --config $cfg --steps 5 --warmup 2 --no-cpu-baseline --no-secondary \
    --no-parity > $O/j${v}_$cfg.log 2>&1 || { tail -20 $O/j${v}_$cfg.log; exit 1; }
  python -c "
import json; l=[x for x in open('$O/j${v}_$cfg.log') if x.startswith('{')][-1]; j=json.loads(l)
st=j['stage_ms']
print('join=$v $cfg', j['dtype'][:12], round(j['ms_per_step'],3), {k: round(v,2) for k,v in st.items()})"
done
done
