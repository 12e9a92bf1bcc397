#!/bin/bash
# round 4: alpha / beta by triangular solves right after the Cholesky
# (UT_EARLY_ALPHA=1) -- tests, then C3 pruned / f16x3 A/B, C2, C5 pruned
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r04f; mkdir -p $O
run() { local t=$1 name=$2; shift 2; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?;
        echo "$name rc=$rc"; tail -1 $O/$name.log | cut -c1-250; [ $rc -eq 0 ] || exit $rc; }
run 300 pytest_ea python -u -m pytest tests/test_gpu_parity.py -m gpu -q --timeout 120 --timeout-method thread -k "early_alpha or chol or fit_append or prune or golden or precision"
run 900 pytest python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
for cfg in "--config c3 --prune 256" "--config c3 --precision 16"; do
  tag=$(echo $cfg | tr -d ' -')
  for ea in 1 0; do
    UT_EARLY_ALPHA=$ea run 400 ${tag}_ea$ea python bench.py $cfg --steps 3 --warmup 1 --no-cpu-baseline
  done
done
run 300 c2 python bench.py --steps 10 --warmup 3 --no-cpu-baseline
run 300 c5_prune python scripts/c5_bandit.py --prune 256
