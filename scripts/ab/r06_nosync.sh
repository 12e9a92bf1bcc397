#!/bin/bash
# round 6 A/B: the precision-8 round without its mid-round host sync
# (UTX_I8_NOSYNC=1 skipped the recompute: a measurement of the host gap only; the knob
# was removed after it: 16.67 ms without the sync against 16.74-16.98 with it)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r06_nosync; mkdir -p $O
for rep in 1 2 3; do
for v in 0 1; do
  if [ $v = 1 ]; then export UTX_I8_NOSYNC=1; else unset UTX_I8_NOSYNC; fi
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-secondary --no-parity \
    > $O/s${v}_$rep.log 2>&1 || { tail -20 $O/s${v}_$rep.log; exit 1; }
  python -c "
import json; l=[x for x in open('$O/s${v}_$rep.log') if x.startswith('{')][-1]; j=json.loads(l)
st=j['stage_ms']; main=sum(st[k] for k in ('propose','encode','fit_wait','kstar','var','finalize','recompute','topk') if k in st)
print('nosync=$v rep $rep', round(j['ms_per_step'],3), 'main-stream stages', round(main,3), {k: round(v,2) for k,v in st.items()})"
done
done
