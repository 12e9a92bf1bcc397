#!/bin/bash
# round 3: kernel timeline of the C3 f16x3 round (where the hash runs beside
# K* and the variance GEMM, and what the finalize waits for)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/c3h3tl
mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace -d $O -o run --output-format csv -- \
  python3 bench.py --config c3 --precision 16 --steps 2 --warmup 1 --no-cpu-baseline --no-parity > $O/log 2>&1 || { echo "rc=$?"; tail -5 $O/log; exit 1; }
echo ok
