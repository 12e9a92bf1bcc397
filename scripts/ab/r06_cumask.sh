#!/bin/bash
# (not kept; the UTX_* knobs were removed after the measurement -- profiles/r06_kq_ab.txt)
# round 6 A/B: with the int8 K*, the side stream (hash + dedup) kept off N CUs
# (UTX_HASH_CUMASK=N; UTX_CUMASK_STRIDE: spread over the chip) so that the
# refit's chain of small kernels finishes beside the hash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r06_cumask; mkdir -p $O
for v in "0 0" "8 0" "16 0" "32 0" "16 1" "32 1"; do
set -- $v
for ell in 0.2 2; do
  f=$O/m$1_s$2_l${ell}.log
  if [ $2 = 1 ]; then export UTX_CUMASK_STRIDE=1; else unset UTX_CUMASK_STRIDE; fi
  UTX_HASH_CUMASK=$1 timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline \
    --no-secondary --no-parity --ell $ell > $f 2>&1 || { tail -20 $f; exit 1; }
  python -c "
import json; l=[x for x in open('$f') if x.startswith('{')][-1]; j=json.loads(l)
print('mask=$1 stride=$2 ell=$ell', round(j['ms_per_step'],3), {k: round(v,2) for k,v in j['stage_ms'].items()})"
done
done
