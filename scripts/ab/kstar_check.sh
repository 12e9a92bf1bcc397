#!/bin/bash
# K* change check: GP parity tests, then rocprofv3 kernel stats of the C2 round
# and the C3 pruned round (each GPU step under its own limit; stop on failure)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 150 --timeout-method thread -p no:cacheprovider -k "gp or prune or score or h3 or topk" > gpurun_out/kstar_tests.log 2>&1
rc=$?; tail -2 gpurun_out/kstar_tests.log; [ $rc -ne 0 ] && { tail -40 gpurun_out/kstar_tests.log; exit $rc; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/kc2 -o run -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/kc2.log 2>&1 || exit 1
tail -1 gpurun_out/kc2.log | cut -c1-150
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/kc3 -o run -- python bench.py --config c3 --prune 128 --steps 5 --warmup 2 > gpurun_out/kc3.log 2>&1 || exit 1
tail -1 gpurun_out/kc3.log | cut -c1-150
for d in kc2 kc3; do f=$(find gpurun_out/$d -name "*kernel_stats.csv" | head -1); echo "== $d"; grep -E "kstar|k_de|var_pp" "$f" | cut -d, -f1-4 | cut -c1-60,200-400; done
