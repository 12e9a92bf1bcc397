#!/bin/bash
# round 6: the C2 round's per-stage device times including "outputs" (the
# selections' gather) and "between" (last mark of a round -> first of the next)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r06_between; mkdir -p $O
for v in 1 0; do
  UT_FIT_DEFER=$v timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-secondary --no-parity \
    > $O/d$v.log 2>&1 || { tail -20 $O/d$v.log; exit 1; }
  python -c "
import json; l=[x for x in open('$O/d$v.log') if x.startswith('{')][-1]; j=json.loads(l)
st=j['stage_ms']; main=sum(st[k] for k in ('propose','encode','fit_wait','kstar','var','finalize','recompute','topk','outputs','between') if k in st)
print('defer=$v', round(j['ms_per_step'],3), 'main-stream stages', round(main,3), {k: round(v,3) for k,v in st.items()})"
done
