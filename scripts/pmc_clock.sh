#!/bin/bash
# effective clock + MFMA busy per kernel (MI355X_MICROARCH.md 'DVFS give-back'):
# clock = GRBM_GUI_ACTIVE / 8 / duration; MFMA util = SQ_VALU_MFMA_BUSY_CYCLES / (cycles * CUs)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${PROF_OUT:-gpurun_out/clk}
mkdir -p $OUT
ARGS=${BENCH_ARGS:---steps 3 --warmup 1 --no-cpu-baseline}
timeout -k 10 600 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES -d $OUT -o run --output-format csv -- \
  python3 bench.py $ARGS > $OUT/log 2>&1 || { echo "pmc rc=$?"; tail -5 $OUT/log; exit 1; }
echo clk ok
