#!/bin/bash
# K* (precision 8) alone: kernel trace + stats, then the stall counters
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
OUT=${PROF_OUT:-gpurun_out/kq}
mkdir -p $OUT/tr $OUT/st
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/tr -o run --output-format csv -- python3 scripts/exp/kstar_micro.py c2_i8_mu > $OUT/tr/log 2>&1 || { echo "trace rc=$?"; exit 1; }
timeout -k 10 -s KILL 300 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
  SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES -d $OUT/st -o run --output-format csv -- \
  python3 scripts/exp/kstar_micro.py c2_i8_mu > $OUT/st/log 2>&1 || { echo "pmc rc=$?"; exit 1; }
echo kq ok
