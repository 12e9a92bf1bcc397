#!/bin/bash
# round 4: k_trinv_big (L^-1 levels >= 256 rows on 128 x 128 tiles) -- parity,
# the fit's latency by n (UT_TRINV_BIG 0 / 1), its kernel trace, C3 / C2 rounds
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r04r; mkdir -p $O
export TMPDIR=/tmp
run() { local t=$1 name=$2; shift 2; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?;
        echo "$name rc=$rc"; tail -1 $O/$name.log | cut -c1-160; [ $rc -eq 0 ] || exit $rc; }
run 400 pytest python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py \
  -k "trinv or chol or fit or gp_score" tests/test_gpu_fullsize.py
UT_TRINV_BIG=0 run 300 fit_old python scripts/microbench.py fit
UT_TRINV_BIG=1 run 300 fit_new python scripts/microbench.py fit
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o fit -- python scripts/microbench.py fit > $O/fit_prof.log 2>&1 || exit $?
find $O/prof -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $O/fit_kernel_stats.csv
rm -rf $O/prof
B="--steps 3 --warmup 1 --no-cpu-baseline --no-parity"
for v in 1 0; do
  UT_TRINV_BIG=$v run 300 c3p_big$v python bench.py --config c3 --prune 256 $B
  UT_TRINV_BIG=$v run 300 c3h_big$v python bench.py --config c3 --precision 16 $B
  UT_TRINV_BIG=$v run 300 c2_big$v python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-parity
done
