#!/bin/bash
# where a kernel's waves spend their cycles (MI355X_MICROARCH.md, rocprofv3 PMC
# slots): SQ_WAIT_ANY = parked on s_waitcnt / barrier, SQ_WAIT_INST_ANY = issue
# stall (MFMA dependency / pipe busy; SQ_WAIT_INST_LDS its LDS share),
# SQ_ACTIVE_INST_ANY = issuing; the three add to SQ_WAVE_CYCLES.  One pass of
# 8 SQ counters.  Summarised by scripts/stall_summary.py.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${PROF_OUT:-gpurun_out/stall}
mkdir -p $OUT
ARGS=${BENCH_ARGS:---steps 3 --warmup 1 --no-cpu-baseline --no-parity}
timeout -k 10 -s KILL 300 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
  SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES -d $OUT -o run --output-format csv -- \
  python3 bench.py $ARGS > $OUT/log 2>&1 || { echo "pmc rc=$?"; tail -5 $OUT/log; exit 1; }
echo stall ok
