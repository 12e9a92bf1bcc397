#!/bin/bash
# round 4: validation + artifacts on the committed tree -- every GPU test,
# smoke, the default bench line (N = 1), the secondary bench lines (C2 / C3
# f16x3, C3 pruned, C3 fp64 dense, C4), the C5 loop dense and pruned, the N > 1
# footprint rehearsals (gloo, one GPU), then the rocprofv3 passes of the C2
# round (kernel trace + stats, FETCH_SIZE, WRITE_SIZE, clock / MFMA busy).
# Each GPU step has its own time limit; a failure ends the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=${FINAL_OUT:-gpurun_out/final4}
mkdir -p $O
run() { local t=$1 name=$2; shift 2; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?;
        echo "$name rc=$rc"; tail -c 300 $O/$name.log; echo; [ $rc -eq 0 ] || exit $rc; }
[ -n "$SKIP_TESTS" ] || {
run 1100 pytest_gpu python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider
run 300 smoke python -c "import __graft_entry__ as g; g.smoke()"
}
run 400 bench_c2 python bench.py
[ -n "$SKIP_LINES" ] || {
run 300 bench_c2_h3 python bench.py --precision 16 --no-cpu-baseline
run 400 bench_c3_h3 python bench.py --config c3 --precision 16 --steps 5 --warmup 2 --no-cpu-baseline
run 400 bench_c3_prune python bench.py --config c3 --prune 256 --steps 5 --warmup 2 --no-cpu-baseline
run 600 bench_c3_f64 python bench.py --config c3 --steps 3 --warmup 1 --no-cpu-baseline
run 400 bench_c4 python bench.py --config c4 --steps 5 --warmup 2 --no-cpu-baseline
run 300 c5_dense python scripts/c5_bandit.py --generations 100
run 300 c5_prune python scripts/c5_bandit.py --generations 100 --prune 256
}
[ -n "$SKIP_MEM" ] || {
UT_DIST_BACKEND=gloo run 400 mem_strong8_c2 python bench.py --gpus 8 --scaling strong --steps 2 --warmup 1 --no-cpu-baseline --no-parity
UT_DIST_BACKEND=gloo run 600 mem_strong8_c3 python bench.py --config c3 --precision 16 --gpus 8 --scaling strong --steps 2 --warmup 1 --no-cpu-baseline --no-parity
}
[ -n "$SKIP_PROF" ] && exit 0
PROF_OUT=$O/prof BENCH_ARGS="--steps 5 --warmup 2 --no-cpu-baseline --no-parity" bash scripts/profile.sh > $O/profile.log 2>&1 || { echo "profile failed"; tail -5 $O/profile.log; exit 1; }
echo profile ok
PROF_OUT=$O/clk BENCH_ARGS="--steps 5 --warmup 2 --no-cpu-baseline --no-parity" bash scripts/pmc_clock.sh > $O/clock.log 2>&1 || { echo "clock failed"; tail -5 $O/clock.log; exit 1; }
echo clock ok
