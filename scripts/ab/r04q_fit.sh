#!/bin/bash
# round 4: the GP fit's chain at n = 4096 standalone (latency by n, and the
# kernel trace of those fits), then the hash-grid cap A/B of r04p
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r04q; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python scripts/microbench.py fit > $O/fit.log 2>&1 || exit $?
tail -3 $O/fit.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o fit -- python scripts/microbench.py fit > $O/fit_prof.log 2>&1 || exit $?
find $O/prof -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $O/fit_kernel_stats.csv
find $O/prof -name "*kernel_trace.csv" | head -1 | xargs -I{} cp {} $O/fit_kernel_trace.csv
rm -rf $O/prof
bash scripts/ab/r04p_hashcap.sh
