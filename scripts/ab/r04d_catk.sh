#!/bin/bash
# round 4: the categorical K* -- its parity tests, then the C3 / C4 lines with
# it on and off (UT_CAT_KSTAR)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r04d; mkdir -p $O
run() { local t=$1 name=$2; shift 2; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?;
        echo "$name rc=$rc"; tail -1 $O/$name.log | cut -c1-250; [ $rc -eq 0 ] || exit $rc; }
run 300 pytest_cat python -u -m pytest tests/test_gpu_parity.py -m gpu -q --timeout 120 --timeout-method thread -k "categorical"
run 900 pytest python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
for cfg in "--config c3 --precision 16" "--config c3 --prune 256" "--config c4"; do
  tag=$(echo $cfg | tr -d ' -')
  for on in 1 0; do
    UT_CAT_KSTAR=$on run 400 ${tag}_cat$on python bench.py $cfg --steps 3 --warmup 1 --no-cpu-baseline
  done
done
# per-rank device memory at N > 1 (gloo rehearsal on one GPU): weak N = 2 at
# the full C2 m (population 2M), strong N = 8 over the C2 pool (128k per rank)
UT_DIST_BACKEND=gloo run 400 mem_weak2 python bench.py --gpus 2 --steps 2 --warmup 1 --no-cpu-baseline --no-parity
UT_DIST_BACKEND=gloo run 400 mem_strong8 python bench.py --gpus 8 --scaling strong --steps 2 --warmup 1 --no-cpu-baseline --no-parity
