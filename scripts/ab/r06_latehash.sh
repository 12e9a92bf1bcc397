#!/bin/bash
# (not kept; the knobs were removed after it -- profiles/r06_latehash_ab.txt)
# round 6 A/B: the C2 round's hash started when K* ends, beside the int8
# variance GEMM (UTX_HASH_AFTER_KSTAR=1; the int8 MFMA co-issues with integer
# VALU work, the f64 K* does not), x the variance GEMM at 1 or 2 workgroups
# per CU (UTX_VAR_WG: at 2 its 256 VGPRs x 2 waves and 2 x 79 KB of LDS leave
# no room on a CU for the hash's waves)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r06_latehash; mkdir -p $O
for rep in 1; do
for cfgv in "0 2" "1 2" "1 1" "0 1"; do
set -- $cfgv
for ell in 0.2 2; do
  f=$O/h$1_w$2_l${ell}_$rep.log
  UTX_HASH_AFTER_KSTAR=$1 UTX_VAR_WG=$2 timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline \
    --no-secondary --ell $ell > $f 2>&1 || { tail -20 $f; exit 1; }
  python -c "
import json; l=[x for x in open('$f') if x.startswith('{')][-1]; j=json.loads(l)
print('late=$1 wg=$2 ell=$ell rep $rep', round(j['ms_per_step'],3), j['parity']['all_ok'], {k: round(v,2) for k,v in j['stage_ms'].items()})"
done
done
done
