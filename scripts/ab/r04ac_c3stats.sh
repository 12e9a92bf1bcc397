#!/bin/bash
# round 4 head: rocprofv3 kernel stats of the C3 pruned and f16x3 rounds
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r04ac; mkdir -p $O
export TMPDIR=/tmp
for cfg in c3p c3h; do
  A="--config c3 --steps 3 --warmup 1 --no-cpu-baseline --no-parity"
  [ $cfg = c3p ] && A="$A --prune 256" || A="$A --precision 16"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/p_$cfg -o run --output-format csv -- python3 bench.py $A > $O/$cfg.log 2>&1 || exit $?
  cp $(find $O/p_$cfg -name "*kernel_stats.csv" | head -1) $O/${cfg}_kernel_stats.csv
  f=$(find $O/p_$cfg -name "*kernel_trace.csv" | head -1)
  python scripts/exp/timeline.py $f --span 45 --top 500 > $O/${cfg}_timeline.txt
  rm -rf $O/p_$cfg
done
