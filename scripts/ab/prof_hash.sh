#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/phash
timeout -k 10 300 python3 scripts/microbench.py hash > gpurun_out/phash/micro.json 2>&1 || exit 1
cat gpurun_out/phash/micro.json
timeout -k 10 600 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -d gpurun_out/phash/pmc -o run --output-format csv -- python3 scripts/microbench.py hash > gpurun_out/phash/pmc.log 2>&1 || { echo "pmc rc=$?"; tail -20 gpurun_out/phash/pmc.log; exit 1; }
echo pmc ok
