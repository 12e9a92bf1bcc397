#!/bin/bash
# round 3 validation + artifacts on the committed tree: every GPU test, smoke,
# the default bench line (N = 1), the 2-rank rehearsal, then the rocprofv3
# passes of the C2 round (kernel trace + stats, FETCH_SIZE, WRITE_SIZE, clock /
# MFMA busy).  Each GPU step has its own time limit; a failure ends the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/final
mkdir -p $O
run() { local t=$1 name=$2; shift 2; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?;
        echo "$name rc=$rc"; tail -c 400 $O/$name.log; echo; [ $rc -eq 0 ] || exit $rc; }
run 1100 pytest_gpu python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider
run 300 smoke python -c "import __graft_entry__ as g; g.smoke()"
run 400 bench_c2 python bench.py
[ -n "$SKIP_PROF" ] && exit 0
BENCH_ARGS="--steps 5 --warmup 2 --no-cpu-baseline --no-parity" bash scripts/profile.sh > $O/profile.log 2>&1 || { echo "profile failed"; tail -5 $O/profile.log; exit 1; }
echo profile ok
BENCH_ARGS="--steps 5 --warmup 2 --no-cpu-baseline --no-parity" bash scripts/pmc_clock.sh > $O/clock.log 2>&1 || { echo "clock failed"; tail -5 $O/clock.log; exit 1; }
echo clock ok
