#!/bin/bash
# round 5 A/B: the precision-8 variance GEMM beside the side stream's hash
# (UTX_NOJOIN=1: no wait for the dup mask before k_gp_var_i8) and with one
# workgroup per CU (UTX_VARWG=1), C2 bench lines.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r05_varjoin; mkdir -p $O
for cfg in "0 2" "1 2" "0 1" "1 1" "0 2" "1 2"; do
  set -- $cfg
  UTX_NOJOIN=$1 UTX_VARWG=$2 timeout -k 10 200 python bench.py --no-cpu-baseline --no-parity > $O/j$1_w$2.log 2>&1 || exit 1
  python -c "
import json; l=[x for x in open('$O/j$1_w$2.log') if x.startswith('{')][-1]; j=json.loads(l)
print('nojoin=$1 wg=$2', round(j['ms_per_step'],3), {k: round(v,2) for k,v in j['stage_ms'].items()})"
done
