#!/bin/bash
# round 4: the pruned round's K* operand prep before the wait for the whole fit
# (it needs only 1/ell) -- pruned parity tests, C3 pruned, C5 pruned
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r04ad; mkdir -p $O
run() { local t=$1 name=$2; shift 2; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?;
        echo "$name rc=$rc"; tail -1 $O/$name.log | cut -c1-120; [ $rc -eq 0 ] || exit $rc; }
run 600 pytest python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "prune or topk" tests/test_gpu_fullsize.py tests/test_gpu_c5.py
run 300 c3p python bench.py --config c3 --prune 256 --steps 5 --warmup 2 --no-cpu-baseline
run 300 c5p python scripts/c5_bandit.py --generations 100 --prune 256
run 300 c3p_2 python bench.py --config c3 --prune 256 --steps 5 --warmup 2 --no-cpu-baseline --no-parity
