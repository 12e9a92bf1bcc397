#!/bin/bash
# round 4: kernel timeline of the C2 round (where the 25.9 ms go beyond the
# main stream's stages) and of the C3 pruned round
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r04v; mkdir -p $O
export TMPDIR=/tmp
for cfg in c2 c3p; do
  A="--steps 3 --warmup 1 --no-cpu-baseline --no-parity"
  [ $cfg = c3p ] && A="--config c3 --prune 256 $A"
  timeout -k 10 300 rocprofv3 --kernel-trace -d $O/tr_$cfg -o run --output-format csv -- python3 bench.py $A > $O/$cfg.log 2>&1 || exit $?
  f=$(find $O/tr_$cfg -name "*kernel_trace.csv" | head -1)
  cp $f $O/${cfg}_kernel_trace.csv && rm -rf $O/tr_$cfg
  python scripts/exp/timeline.py $O/${cfg}_kernel_trace.csv --span 30 --top 400 > $O/${cfg}_timeline.txt
done
