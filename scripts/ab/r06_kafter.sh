#!/bin/bash
# (the UTX_* knobs were removed after the measurement: the i8 variance GEMM no longer joins the hash;
#  K* after the hash and the encode launched first were not kept -- profiles/r06_sched_ab.txt)
# round 6 A/B: K* after the hash + dedup (UTX_KSTAR_AFTER_HASH=1: the hash runs
# beside encode only, K* and the variance GEMM alone) against K* beside the hash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r06_kafter; mkdir -p $O
for rep in 1 2; do
for v in 0 1; do
for ell in 0.2 2; do
  UTX_KSTAR_AFTER_HASH=$v timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-secondary \
    --no-parity --ell $ell > $O/k${v}_l${ell}_$rep.log 2>&1 || { tail -20 $O/k${v}_l${ell}_$rep.log; exit 1; }
  python -c "
import json; l=[x for x in open('$O/k${v}_l${ell}_$rep.log') if x.startswith('{')][-1]; j=json.loads(l)
st=j['stage_ms']
print('kafter=$v ell=$ell rep $rep', round(j['ms_per_step'],3), {k: round(v,2) for k,v in st.items()})"
done
done
done
for v in 0 1; do
for cfg in c4 c3; do
  UTX_KSTAR_AFTER_HASH=$v timeout -k 10 300 python bench.py --config $cfg --steps 5 --warmup 2 --no-cpu-baseline \
    --no-secondary --no-parity > $O/k${v}_$cfg.log 2>&1 || { tail -20 $O/k${v}_$cfg.log; exit 1; }
  python -c "
import json; l=[x for x in open('$O/k${v}_$cfg.log') if x.startswith('{')][-1]; j=json.loads(l)
st=j['stage_ms']
print('kafter=$v $cfg', round(j['ms_per_step'],3), {k: round(v,2) for k,v in st.items()})"
done
done
