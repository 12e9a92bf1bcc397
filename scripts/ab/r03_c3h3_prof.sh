#!/bin/bash
# round 3: the C3 f16x3 round's kernels -- a kernel trace (concurrent streams as
# they run) and a counter pass (dispatches serialized: standalone durations,
# clock, MFMA busy)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/c3p
mkdir -p $O
ARGS="--config c3 --precision 16 --steps 3 --warmup 1 --no-cpu-baseline --no-parity"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 bench.py $ARGS > $O/trace.log 2>&1 || { echo "trace rc=$?"; tail -5 $O/trace.log; exit 1; }
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES -d $O/pmc -o run --output-format csv -- python3 bench.py $ARGS > $O/pmc.log 2>&1 || { echo "pmc rc=$?"; tail -5 $O/pmc.log; exit 1; }
python3 scripts/exp/pmc_by_kernel.py $O/pmc | sort -t= -k2 | awk '{print}' | grep -v "n=  0" | sort -k3 -n -r -t' ' | head -40
find $O/trace -name "*kernel_stats.csv" | head -1 | xargs -I{} sh -c 'cut -c1-160 {} | head -20'
