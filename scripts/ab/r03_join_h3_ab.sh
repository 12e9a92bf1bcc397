#!/bin/bash
# round 3: does the f16x3 round gain from letting the hash spill into the
# variance GEMM (UT_JOIN_BEFORE_VAR=0; fp16 MFMA beside integer VALU) -- C2 and
# C3 f16x3 lines, each schedule twice, one process each
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/joinab
mkdir -p $O
for cfg in "c2 --steps 20 --warmup 3" "c3 --config c3 --steps 5 --warmup 2"; do
  set -- $cfg; tag=$1; shift
  for rep in 1 2; do
    for j in 1 0; do
      UT_JOIN_BEFORE_VAR=$j timeout -k 10 300 python bench.py $* --precision 16 --no-cpu-baseline --no-parity > $O/${tag}_j${j}_$rep.log 2>&1 || { echo "$tag j$j rc=$?"; tail -5 $O/${tag}_j${j}_$rep.log; exit 1; }
      python3 -c "import json,sys; d=json.loads([l for l in open('$O/${tag}_j${j}_$rep.log') if l.startswith('{')][-1]); print('$tag join=$j rep $rep', round(d['ms_per_step'],2), 'ms', round(d['value']/1e6,2), 'M/s')"
    done
  done
done
