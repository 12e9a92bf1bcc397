#!/bin/bash
# round 6: var8_probe timing only (random digits, then zero low planes)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${TAG:-r06_var8pt}; mkdir -p $O
timeout -k 10 120 ./scripts/exp/var8_probe 1024 1048576 7 0 > $O/rand.log 2>&1 || { cat $O/rand.log; exit 1; }
timeout -k 10 120 ./scripts/exp/var8_probe 1024 1048576 7 1 > $O/zero.log 2>&1 || { cat $O/zero.log; exit 1; }
cat $O/rand.log $O/zero.log
