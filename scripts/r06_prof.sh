#!/bin/bash
# round 6: rocprofv3 record of the default C2 round (precision 8) at the
# headline's ell = 0.2 and at the secondary line's ell = 2:
# per lengthscale a kernel trace + stats pass, FETCH_SIZE and WRITE_SIZE passes,
# and the clock / MFMA-busy pass (dispatches serialized: each kernel alone).
# Processed on the host:
#   python scripts/pmc_summary.py  gpurun_out/${TAG}_l02 ${TAG}_l02
#   python scripts/pmc_summary.py  gpurun_out/${TAG}_l2  ${TAG}_l2 _l2
#   python scripts/clock_summary.py gpurun_out/${TAG}_l02/clk ${TAG}_l02
#   python scripts/clock_summary.py gpurun_out/${TAG}_l2/clk  ${TAG}_l2 _l2
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r06}
for ELL in ${ELLS:-0.2 2}; do
  S=$([ "$ELL" = "0.2" ] && echo l02 || echo l2)
  export PROF_OUT=gpurun_out/${TAG}_${S}
  export BENCH_ARGS="--steps 3 --warmup 1 --no-cpu-baseline --no-parity --no-secondary --ell $ELL ${EXTRA_ARGS}"
  bash scripts/profile.sh || exit 1
  PROF_OUT=gpurun_out/${TAG}_${S}/clk bash scripts/pmc_clock.sh || exit 1
done
