#!/bin/bash
# round 4: defaults UT_FIT_SETPRIO=1 + the auto hash cap vs both off
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r04u; mkdir -p $O
run() { local t=$1 name=$2; shift 2; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?;
        echo "$name rc=$rc"; tail -1 $O/$name.log | cut -c1-120; [ $rc -eq 0 ] || exit $rc; }
run 400 pytest python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py \
  -k "capped or trinv or chol or hash_de" tests/test_gpu_fullsize.py
B="--steps 3 --warmup 1 --no-cpu-baseline --no-parity"
run 300 c3p python bench.py --config c3 --prune 256 $B
run 300 c3h python bench.py --config c3 --precision 16 $B
run 300 c2 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-parity
run 300 c4 python bench.py --config c4 $B
run 300 c5p python scripts/c5_bandit.py --generations 100 --prune 256
export UT_FIT_SETPRIO=0 UT_HASH_WG_PER_CU=0
run 300 c3p_off python bench.py --config c3 --prune 256 $B
run 300 c3h_off python bench.py --config c3 --precision 16 $B
run 300 c5p_off python scripts/c5_bandit.py --generations 100 --prune 256
