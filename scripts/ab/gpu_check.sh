#!/bin/bash
# GPU round trip: parity tests, smoke, short bench.  Every GPU step has its
# own time limit; a fault / abort / timeout ends the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
stop_if_fatal() { case "$1" in 0|1) ;; *) echo "fatal rc=$1 ($2)"; exit "$1";; esac; }
timeout -k 10 ${PYTEST_TIMEOUT:-900} python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider ${PYTEST_ARGS} \
  > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -30 gpurun_out/pytest_gpu.log; stop_if_fatal $rc pytest
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -5 gpurun_out/smoke.log; stop_if_fatal $rc smoke
[ -n "$SKIP_BENCH" ] && exit 0
timeout -k 10 ${BENCH_TIMEOUT:-600} python bench.py ${BENCH_ARGS:---steps 5 --warmup 2 --cpu-sample 32768} \
  > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -5 gpurun_out/bench.log
exit $rc
