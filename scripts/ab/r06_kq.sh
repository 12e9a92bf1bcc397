#!/bin/bash
# round 6: precision-8 K* as the distance contraction on the int8 MFMA
# (gp_kq.hip, UT_KSTAR_Q=1) against k_gp_kstar<int8_t> on the fp64 MFMA (0):
# the GPU tests first, then C2 at ell 0.2 and 2
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r06_kq; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 150 --timeout-method thread -m gpu tests/ > $O/tests.log 2>&1 \
  || { echo tests failed; grep -E "FAILED|Error" $O/tests.log | head -20; tail -5 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for rep in 1 2; do
for v in 1 0; do
for ell in 0.2 2; do
  f=$O/q${v}_l${ell}_$rep.log
  UT_KSTAR_Q=$v timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-secondary \
    --ell $ell > $f 2>&1 || { tail -20 $f; exit 1; }
  python -c "
import json; l=[x for x in open('$f') if x.startswith('{')][-1]; j=json.loads(l)
print('kq=$v ell=$ell rep $rep', round(j['ms_per_step'],3), j['parity']['all_ok'], j['i8']['recomputed_fp64_last_timed_round'], {k: round(v,2) for k,v in j['stage_ms'].items()})"
done
done
done
