#!/bin/bash
# h3_probe at C3 and C2, then one counter pass (clock, MFMA busy) at C3
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/h3p
mkdir -p $O
timeout -k 10 150 scripts/exp/h3_probe 4096 2097152 3 > $O/c3.log 2>&1; rc=$?; cat $O/c3.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 60 scripts/exp/h3_probe 1024 1048576 10 > $O/c2.log 2>&1; rc=$?; cat $O/c2.log; [ $rc -eq 0 ] || exit $rc
[ -n "$NO_PMC" ] && exit 0
timeout -s KILL 200 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES -d $O/pmc -o run --output-format csv -- scripts/exp/h3_probe 4096 2097152 1 > $O/pmc.log 2>&1; rc=$?
[ $rc -eq 0 ] || { echo "pmc rc=$rc"; tail -5 $O/pmc.log; exit $rc; }
python3 scripts/exp/pmc_by_kernel.py $O/pmc
