#!/bin/bash
# round 6 A/B: the staged fit issued after the round's proposal (UT_FIT_DEFER=1,
# the default) against issued inside ut_gp_fit_async (UT_FIT_DEFER=0), C2 at
# ell 0.2 and 2; then the GPU tests on the default
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r06_fitdefer; mkdir -p $O
for rep in 1 2; do
for v in 0 1; do
for ell in 0.2 2; do
  UT_FIT_DEFER=$v timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-secondary --no-parity \
    --ell $ell > $O/d${v}_l${ell}_$rep.log 2>&1 || { tail -20 $O/d${v}_l${ell}_$rep.log; exit 1; }
  python -c "
import json; l=[x for x in open('$O/d${v}_l${ell}_$rep.log') if x.startswith('{')][-1]; j=json.loads(l)
st=j['stage_ms']; main=sum(st[k] for k in ('propose','encode','fit_wait','kstar','var','finalize','recompute','topk') if k in st)
print('defer=$v ell=$ell rep $rep', round(j['ms_per_step'],3), 'main-stream stages', round(main,3), {k: round(v,2) for k,v in st.items()})"
done
done
done
