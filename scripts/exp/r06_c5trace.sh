#!/bin/bash
# round 6: HIP API + kernel trace of a short C5 pruned loop (where does the
# host block inside torch.maximum / torch.where?)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r06_c5trace; mkdir -p $O
timeout -k 10 300 rocprofv3 --hip-runtime-trace --kernel-trace -d $O/t -o run --output-format csv -- \
  python scripts/c5_bandit.py --prune 256 --generations 20 --warmup-generations 0 > $O/log 2>&1 || { tail -20 $O/log; exit 1; }
echo ok
