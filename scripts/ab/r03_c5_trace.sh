#!/bin/bash
# round 3: kernel trace of the C5 pruned loop (where the device time of a
# generation goes: the fit's kernels, the scoring round, the gaps between)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/c5trace
mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- \
  python3 scripts/c5_bandit.py --prune 256 > $O/trace.log 2>&1 || { echo "trace rc=$?"; tail -5 $O/trace.log; exit 1; }
tail -1 $O/trace.log
echo c5 trace ok
