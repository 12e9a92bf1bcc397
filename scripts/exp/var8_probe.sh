#!/bin/bash
# round 6: var8_probe timing (random digits and zero low planes), then one
# FETCH_SIZE pass and one clock / MFMA-busy pass over the random-digit run
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r06_var8p}; mkdir -p $O
timeout -k 10 120 ./scripts/exp/var8_probe 1024 1048576 5 0 > $O/rand.log 2>&1 || { cat $O/rand.log; exit 1; }
timeout -k 10 120 ./scripts/exp/var8_probe 1024 1048576 5 1 > $O/zero.log 2>&1 || { cat $O/zero.log; exit 1; }
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $O/fetch -o run --output-format csv -- ./scripts/exp/var8_probe 1024 1048576 1 0 > $O/fetch.log 2>&1 || { echo fetch failed; exit 1; }
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES -d $O/clk -o run --output-format csv -- ./scripts/exp/var8_probe 1024 1048576 1 0 > $O/clk.log 2>&1 || { echo clk failed; exit 1; }
cat $O/rand.log $O/zero.log
