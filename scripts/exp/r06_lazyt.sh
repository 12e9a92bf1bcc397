#!/bin/bash
# round 6: precision-8 refits without (L^-1)^T / alpha on the fit chain
# (gp_ensure_linvt): the GP tests that reach the recompute and append paths,
# then C2 at ell 0.2 and 2
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r06_lazyt; mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 150 --timeout-method thread -m gpu tests/test_gpu_i8.py \
  tests/test_gpu_parity.py tests/test_gpu_fit_staging.py tests/test_gpu_kstar_q.py > $O/tests.log 2>&1 \
  || { grep -E "FAILED|Error" $O/tests.log | head; tail -5 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for rep in 1 2; do
for ell in 0.2 2; do
  f=$O/l${ell}_$rep.log
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-secondary --no-parity --ell $ell \
    > $f 2>&1 || { tail -20 $f; exit 1; }
  python -c "
import json; l=[x for x in open('$f') if x.startswith('{')][-1]; j=json.loads(l)
print('ell=$ell rep $rep', round(j['ms_per_step'],3), {k: round(v,2) for k,v in j['stage_ms'].items()})"
done
done
