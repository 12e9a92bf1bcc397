#!/bin/bash
# round 3: where the wave cycles of the f16x3 variance kernel (and the fp64
# one) go -- SQ wave-state counters, instruction mix, L2 hit rate -- on the
# C2 round (BENCH_ARGS picks the precision).  One rocprofv3 run per pass.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/prof_waves${TAG}
mkdir -p $OUT
ARGS=${BENCH_ARGS:---precision 16 --steps 3 --warmup 1 --no-cpu-baseline --no-parity}
timeout -k 10 60 rocprofv3 --list-avail > $OUT/avail.txt 2>&1; echo "list rc=$?"
pass() { local name=$1; shift; timeout -s KILL 120 rocprofv3 "$@" -d $OUT/$name -o run --output-format csv -- \
  python3 bench.py $ARGS > $OUT/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
pass states --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM
pass insts --kernel-trace --pmc SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_VALU SQ_INSTS_SALU SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_SMEM SQ_VALU_MFMA_BUSY_CYCLES
pass l2 --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE
exit 0
