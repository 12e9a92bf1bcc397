#!/bin/bash
# (the UTX_* knobs were removed after the measurement: the i8 variance GEMM no longer joins the hash;
#  K* after the hash and the encode launched first were not kept -- profiles/r06_sched_ab.txt)
# round 6 A/B: C2 round schedule -- the variance GEMM's join on the hash
# (UTX_VAR_JOIN) x the encode launched before the hash (UTX_ENCODE_FIRST)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r06_sched; mkdir -p $O
for rep in 1 2; do
for cfgv in "1 0" "0 0" "0 1" "1 1"; do
set -- $cfgv
for ell in 0.2 2; do
  f=$O/j$1_e$2_l${ell}_$rep.log
  UTX_VAR_JOIN=$1 UTX_ENCODE_FIRST=$2 timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline \
    --no-secondary --no-parity --ell $ell > $f 2>&1 || { tail -20 $f; exit 1; }
  python -c "
import json; l=[x for x in open('$f') if x.startswith('{')][-1]; j=json.loads(l)
st=j['stage_ms']
print('join=$1 encfirst=$2 ell=$ell rep $rep', round(j['ms_per_step'],3), {k: round(v,2) for k,v in st.items()})"
done
done
done
