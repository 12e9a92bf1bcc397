#!/bin/bash
# round 5 A/B: the GA round's hash + dedup forked after propose (0) or after
# K* (1: beside the int8 variance GEMM), C4 line alternating; the C4 tests with 1.
# (the UTX_GA_FORK knob was removed after this A/B; fork 0 kept)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r05_ga_fork; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_c4.py -k "separate" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for rep in 1 2; do
for f in 0 1; do
  UTX_GA_FORK=$f timeout -k 10 400 python bench.py --config c4 --steps 5 --warmup 2 --no-cpu-baseline \
    > $O/c4_f${f}_$rep.log 2>&1 || { tail -20 $O/c4_f${f}_$rep.log; exit 1; }
  python -c "
import json; l=[x for x in open('$O/c4_f${f}_$rep.log') if x.startswith('{')][-1]; j=json.loads(l)
print('fork $f rep $rep', round(j['ms_per_step'],3), round(j['value']/1e6,2), j['parity'].get('all_ok'), {k: round(v,2) for k,v in j['stage_ms'].items()})"
done
done
