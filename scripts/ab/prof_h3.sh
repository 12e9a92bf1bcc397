#!/bin/bash
# rocprofv3 of the f16x3 (precision 16) C2 round: kernel trace + stats, HBM
# bytes (FETCH_SIZE / WRITE_SIZE, separate passes), clock + MFMA busy, LDS bank
# conflicts.  Every pass is its own run with its own time limit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/prof_h3
mkdir -p $OUT
ARGS=${BENCH_ARGS:---precision 16 --steps 3 --warmup 1 --no-cpu-baseline}
pass() { local name=$1; shift; timeout -k 10 300 rocprofv3 "$@" -d $OUT/$name -o run --output-format csv -- \
  python3 bench.py $ARGS > $OUT/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
pass trace --kernel-trace --stats
pass pmc_fetch --pmc FETCH_SIZE
pass pmc_write --pmc WRITE_SIZE
pass clk --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES
pass lds --kernel-trace --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS
tail -1 $OUT/trace.log
