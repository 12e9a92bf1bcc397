#!/bin/bash
# round 5: pruned DE rounds encode straight into the K* operands (no feature
# matrix, no prep pass) -- the pruned tests, then the C3 pruned line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r05_prune_encode; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_c5.py -k "prune or round" > $O/pytest.log 2>&1 \
  || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for rep in 1 2; do
  timeout -k 10 300 python bench.py --config c3 --prune 256 --steps 5 --warmup 2 --no-cpu-baseline \
    > $O/c3p_$rep.log 2>&1 || { tail -20 $O/c3p_$rep.log; exit 1; }
  python -c "
import json; l=[x for x in open('$O/c3p_$rep.log') if x.startswith('{')][-1]; j=json.loads(l)
print('c3p rep $rep', round(j['ms_per_step'],3), round(j['value']/1e6,2), j['parity'].get('all_ok'), j['prune']['survivor_frac'], {k: round(v,2) for k,v in j['stage_ms'].items()})"
done
