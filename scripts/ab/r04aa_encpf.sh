#!/bin/bash
# round 4: the encoders' value columns loaded 8 params ahead -- parity, then C4 /
# C3 / C2 lines (the encode stage)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r04aa; mkdir -p $O
run() { local t=$1 name=$2; shift 2; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?;
        echo "$name rc=$rc"; tail -1 $O/$name.log | cut -c1-120; [ $rc -eq 0 ] || exit $rc; }
run 600 pytest python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_c4.py tests/test_gpu_fullsize.py
B="--steps 3 --warmup 1 --no-cpu-baseline"
run 300 c4 python bench.py --config c4 $B
run 300 c3h python bench.py --config c3 --precision 16 $B
run 300 c3p python bench.py --config c3 --prune 256 $B
run 300 c2 python bench.py --steps 10 --warmup 3 --no-cpu-baseline
