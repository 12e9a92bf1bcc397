#!/bin/bash
# Round-2 GPU round trip: parity tests, smoke, default C2 bench (with both CPU
# baselines), C4 bench.  Every GPU step has its own limit; a fault / abort /
# timeout ends the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
stop_if_fatal() { case "$1" in 0|1) ;; *) echo "fatal rc=$1 ($2)"; exit "$1";; esac; }
if [ -z "$SKIP_TESTS" ]; then
KARGS=()
[ -n "$PYTEST_K" ] && KARGS=(-k "$PYTEST_K")
timeout -k 10 ${PYTEST_TIMEOUT:-900} python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread -p no:cacheprovider "${KARGS[@]}" \
  > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|error" gpurun_out/pytest_gpu.log | tail -3; stop_if_fatal $rc pytest
[ $rc -ne 0 ] && { tail -60 gpurun_out/pytest_gpu.log; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/smoke.log; stop_if_fatal $rc smoke
fi
timeout -k 10 600 python bench.py ${BENCH_ARGS:---steps 10 --warmup 3} > gpurun_out/bench_c2.log 2>&1
rc=$?; echo "bench c2 rc=$rc"; tail -1 gpurun_out/bench_c2.log; stop_if_fatal $rc bench
[ -n "$SKIP_C4" ] && exit 0
timeout -k 10 600 python bench.py --config c4 --steps 5 --warmup 2 > gpurun_out/bench_c4.log 2>&1
rc=$?; echo "bench c4 rc=$rc"; tail -1 gpurun_out/bench_c4.log
exit $rc
