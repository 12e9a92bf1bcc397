#!/bin/bash
# round 4: the coalesced categorical encoders (tests, C4 / C3 lines), then the
# fit wait of C3 rounds: fit stream priority, the pruned round's hash held for
# the fit, the f16x3 round's hash held for the fit
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r04m; mkdir -p $O
run() { local t=$1 name=$2; shift 2; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?;
        echo "$name rc=$rc"; tail -1 $O/$name.log | cut -c1-120; [ $rc -eq 0 ] || exit $rc; }
run 600 pytest python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_c4.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 300 --timeout-method thread -k "categorical or c4 or c3 or prune or gp_"
run 400 c4 python bench.py --config c4 --steps 3 --warmup 1 --no-cpu-baseline
B="python bench.py --config c3 --prune 256 --steps 3 --warmup 1 --no-cpu-baseline --no-parity"
run 300 c3p_base $B
UT_FIT_PRIORITY=1 run 300 c3p_prio $B
UT_HASH_HOLD_PRUNED=2 run 300 c3p_hold2 $B
UT_HASH_HOLD_PRUNED=1 run 300 c3p_hold1 $B
UT_FIT_PRIORITY=1 UT_HASH_HOLD_PRUNED=2 run 300 c3p_both $B
H="python bench.py --config c3 --precision 16 --steps 3 --warmup 1 --no-cpu-baseline --no-parity"
run 300 c3h_base $H
UT_FIT_PRIORITY=1 run 300 c3h_prio $H
UT_HASH_HOLD_LOWPREC=1 run 300 c3h_hold $H
C="python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-parity"
run 300 c2_base $C
UT_FIT_PRIORITY=1 run 300 c2_prio $C
