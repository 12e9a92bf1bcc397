#!/bin/bash
# round 5: the f32-contraction bound pass (prune pass 32, the default) -- every
# pruned GPU test, then the C3 pruned line with each pass and the C5 pruned loop.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r05_prunepass2; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_c5.py -k "prune" > $O/pytest.log 2>&1 \
  || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for rep in 1 2; do
for p in 32 64; do
  timeout -k 10 300 python bench.py --config c3 --prune 256 --prune-pass $p --steps 5 --warmup 2 --no-cpu-baseline \
    > $O/c3p_${p}_$rep.log 2>&1 || { tail -20 $O/c3p_${p}_$rep.log; exit 1; }
  python -c "
import json; l=[x for x in open('$O/c3p_${p}_$rep.log') if x.startswith('{')][-1]; j=json.loads(l)
print('pass $p rep $rep', round(j['ms_per_step'],3), j['parity'].get('all_ok'), j['prune']['survivor_frac'], round(j['roofline']['frac'],3), {k: round(v,2) for k,v in j['stage_ms'].items()})"
done
done
timeout -k 10 300 python scripts/c5_bandit.py --generations 100 --prune 256 > $O/c5_prune.log 2>&1 || { tail -20 $O/c5_prune.log; exit 1; }
tail -c 400 $O/c5_prune.log
