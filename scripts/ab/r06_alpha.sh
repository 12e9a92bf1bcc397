#!/bin/bash
# (not kept: the one-workgroup solve took fit_wait 6.8 -> 13.4-13.6 ms at C3 pruned (n 4096, beside the hash);
#  the change is scripts/ab/r06_alpha_solve.patch -- profiles/r06_alpha_ab.txt)
# round 6: fp64 refits solve for alpha before L^-1 (k_alpha_solve; the pruned
# K* waits for alpha only) -- tests, then C3 pruned and the C5 pruned loop with
# UT_ALPHA_SOLVE=1 (default) / 0
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r06_alpha; mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 150 --timeout-method thread -m gpu tests/test_gpu_alpha_solve.py \
  tests/test_gpu_parity.py tests/test_gpu_fullsize.py > $O/tests.log 2>&1 \
  || { grep -E "FAILED|Error" $O/tests.log | head; tail -5 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for rep in 1 2; do
for v in 1 0; do
  f=$O/c3p_a${v}_$rep.log
  UT_ALPHA_SOLVE=$v timeout -k 10 300 python bench.py --config c3 --prune 256 --steps 5 --warmup 2 --no-cpu-baseline \
    > $f 2>&1 || { tail -20 $f; exit 1; }
  python -c "
import json; l=[x for x in open('$f') if x.startswith('{')][-1]; j=json.loads(l)
print('c3prune alpha_solve=$v rep $rep', round(j['ms_per_step'],3), j['parity']['all_ok'], {k: round(v,2) for k,v in j['stage_ms'].items()})"
done
done
for v in 1 0; do
  f=$O/c5p_a$v.log
  UT_ALPHA_SOLVE=$v timeout -k 10 300 python scripts/c5_bandit.py --prune 256 > $f 2>&1 || { tail -20 $f; exit 1; }
  python -c "
import json; l=[x for x in open('$f') if x.startswith('{')][-1]; j=json.loads(l)
print('c5prune alpha_solve=$v', round(j['wall_s'],4), round(j['candidates_scored_per_s']/1e6,2), j['best'], j['evaluations'])"
done
