#!/bin/bash
# hash kernel: per-space timing + instruction counters (separate passes)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/hashpmc
mkdir -p $OUT
timeout -k 10 300 python scripts/microbench.py hash > $OUT/micro.json 2> $OUT/micro.err || { echo "micro rc=$?"; tail -5 $OUT/micro.err; exit 1; }
cat $OUT/micro.json
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU -d $OUT/p1 -o run --output-format csv -- python3 scripts/microbench.py hash > $OUT/p1.log 2>&1 || { echo "p1 rc=$?"; tail -5 $OUT/p1.log; exit 1; }
echo p1 ok
