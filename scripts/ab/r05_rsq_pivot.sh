#!/bin/bash
# round 5: Cholesky pivots by v_rsq_f64 + Newton -- the fit / GP GPU tests, then
# the C3 pruned and C2 lines (fit_wait).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r05_rsq; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_i8.py tests/test_gpu_fullsize.py -k "gp or fit or chol or i8 or full" \
  > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for rep in 1 2; do
  timeout -k 10 300 python bench.py --config c3 --prune 256 --steps 5 --warmup 2 --no-cpu-baseline \
    > $O/c3p_$rep.log 2>&1 || { tail -20 $O/c3p_$rep.log; exit 1; }
  timeout -k 10 300 python bench.py --no-cpu-baseline > $O/c2_$rep.log 2>&1 || { tail -20 $O/c2_$rep.log; exit 1; }
  for f in c3p c2; do python -c "
import json; l=[x for x in open('$O/${f}_$rep.log') if x.startswith('{')][-1]; j=json.loads(l)
print('$f rep $rep', round(j['ms_per_step'],3), round(j['value']/1e6,2), j['parity'].get('all_ok'), {k: round(v,2) for k,v in j['stage_ms'].items()})"; done
done
