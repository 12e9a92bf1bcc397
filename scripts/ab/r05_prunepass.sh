#!/bin/bash
# round 5: the pruned round's bound pass in f32 (default) against fp64: GPU
# pruned tests, then the C3 pruned line with each pass, alternating.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r05_prunepass; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py -k "pruned" > $O/pytest_parity.log 2>&1 || { tail -30 $O/pytest_parity.log; exit 1; }
tail -2 $O/pytest_parity.log
for rep in 1 2; do
for p in 32 64; do
  timeout -k 10 300 python bench.py --config c3 --prune 256 --prune-pass $p --steps 5 --warmup 2 --no-cpu-baseline \
    > $O/c3p_${p}_$rep.log 2>&1 || { tail -20 $O/c3p_${p}_$rep.log; exit 1; }
  python -c "
import json; l=[x for x in open('$O/c3p_${p}_$rep.log') if x.startswith('{')][-1]; j=json.loads(l)
print('pass $p rep $rep', round(j['ms_per_step'],3), j['parity'].get('all_ok'), j['prune']['survivor_frac'], {k: round(v,2) for k,v in j['stage_ms'].items()})"
done
done
