#!/bin/bash
# (not kept: the fused k_de ran 0.97 against 0.71 ms and the C2 round 16.72-16.79 against 16.57 ms;
#  the change is kept as scripts/ab/r06_deenc_fused.patch against dc9c427 -- profiles/r06_deenc_ab.txt)
# round 6 A/B: k_de writing the K* operands itself (UT_DE_ENCODE=1, the
# default) against the separate k_encode_scaled pass (0), C2 at ell 0.2 and 2;
# then the two test files of the round's changes
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r06_deenc; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_de_encode.py \
  > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for rep in 1 2; do
for v in 1 0; do
for ell in 0.2 2; do
  f=$O/e${v}_l${ell}_$rep.log
  UT_DE_ENCODE=$v timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-secondary \
    --no-parity --ell $ell > $f 2>&1 || { tail -20 $f; exit 1; }
  python -c "
import json; l=[x for x in open('$f') if x.startswith('{')][-1]; j=json.loads(l)
print('deenc=$v ell=$ell rep $rep', round(j['ms_per_step'],3), {k: round(v,2) for k,v in j['stage_ms'].items()})"
done
done
done
