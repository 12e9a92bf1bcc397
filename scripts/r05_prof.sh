#!/bin/bash
# round 5: rocprofv3 record of the default C2 round (precision 8): kernel trace +
# stats, FETCH_SIZE and WRITE_SIZE passes, then the clock / MFMA-busy pass.
# Processed on the host by scripts/pmc_summary.py and scripts/clock_summary.py.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r05}
export PROF_OUT=gpurun_out/${TAG}_prof
export BENCH_ARGS=${BENCH_ARGS:---steps 3 --warmup 1 --no-cpu-baseline --no-parity}
bash scripts/profile.sh || exit 1
PROF_OUT=gpurun_out/${TAG}_clk bash scripts/pmc_clock.sh || exit 1
