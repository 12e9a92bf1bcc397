#!/bin/bash
# round 3: kernel trace + stats and a clock / MFMA-busy counter pass of the
# secondary lines (C3 pruned fp64, C4), each under its own time limit
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for spec in "c3p --config c3 --prune 256" "c4 --config c4"; do
  set -- $spec; tag=$1; shift
  O=gpurun_out/sec_$tag
  mkdir -p $O
  ARGS="$* --steps 3 --warmup 1 --no-cpu-baseline --no-parity"
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 bench.py $ARGS > $O/trace.log 2>&1 || { echo "$tag trace rc=$?"; tail -5 $O/trace.log; exit 1; }
  timeout -s KILL 400 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES -d $O/pmc -o run --output-format csv -- python3 bench.py $ARGS > $O/pmc.log 2>&1 || { echo "$tag pmc rc=$?"; tail -5 $O/pmc.log; exit 1; }
  echo "$tag ok"
done
