#!/bin/bash
# round 4: early alpha + parent-relative K* together -- the GPU suite, the C5
# history with the relative K* on / off (and dense), C3 pruned / f16x3 with
# early alpha on / off, C2, a kernel trace of the C5 pruned loop
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r04j; mkdir -p $O
run() { local t=$1 name=$2; shift 2; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?;
        echo "$name rc=$rc"; tail -1 $O/$name.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc; }
run 900 pytest python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
for r in 1 0; do UT_KSTAR_REL=$r run 300 c5_rel$r python scripts/c5_bandit.py --prune 256; done
run 300 c5_dense python scripts/c5_bandit.py
for cfg in "--config c3 --prune 256" "--config c3 --precision 16"; do
  tag=$(echo $cfg | tr -d ' -')
  for ea in 1 0; do
    UT_EARLY_ALPHA=$ea run 400 ${tag}_ea$ea python bench.py $cfg --steps 3 --warmup 1 --no-cpu-baseline
  done
done
run 300 c2 python bench.py --steps 10 --warmup 3 --no-cpu-baseline
run 300 c5_trace rocprofv3 --kernel-trace --stats -d $O/c5_trace -o run --output-format csv -- python3 scripts/c5_bandit.py --prune 256
