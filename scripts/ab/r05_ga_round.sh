#!/bin/bash
# round 5: the fused GA scoring round (ut_score_round_ga) -- C4 GPU tests, then
# the C4 line (hash + dedup now beside the GP on a second stream).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r05_ga_round; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_c4.py \
  > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for rep in 1 2; do
  timeout -k 10 400 python bench.py --config c4 --steps 5 --warmup 2 --no-cpu-baseline > $O/c4_$rep.log 2>&1 \
    || { tail -20 $O/c4_$rep.log; exit 1; }
  python -c "
import json; l=[x for x in open('$O/c4_$rep.log') if x.startswith('{')][-1]; j=json.loads(l)
print('c4 rep $rep', round(j['ms_per_step'],3), round(j['value']/1e6,2), j['parity'].get('all_ok'), {k: round(v,2) for k,v in j['stage_ms'].items()})"
done
