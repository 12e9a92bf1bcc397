#!/bin/bash
# round 4: kernel stats of the categorical-K* C3 / C4 rounds, the fp64 dense C3
# line, and the C5 loop (dense, pruned, host profile)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r04e; mkdir -p $O
run() { local t=$1 name=$2; shift 2; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?;
        echo "$name rc=$rc"; tail -1 $O/$name.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc; }
for cfg in "--config c3 --precision 16" "--config c3 --prune 256" "--config c4"; do
  tag=$(echo $cfg | tr -d ' -')
  run 400 tr_$tag rocprofv3 --kernel-trace --stats -d $O/tr_$tag -o run --output-format csv -- \
    python3 bench.py $cfg --steps 3 --warmup 1 --no-cpu-baseline --no-parity
done
run 600 c3_f64 python bench.py --config c3 --steps 3 --warmup 1 --no-cpu-baseline
run 300 c5_prune python scripts/c5_bandit.py --prune 256
run 300 c5_dense python scripts/c5_bandit.py
run 300 c5_host python scripts/prof_c5_host.py 256
