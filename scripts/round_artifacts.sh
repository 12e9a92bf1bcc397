#!/bin/bash
# Everything the round's profiles/ are regenerated from, one GPU call:
# rocprofv3 stats + HBM counters + clocks on the C2 bench, the bench lines of
# every config / precision, the C5 bandit run and the kernel microbenchmarks.
# Each GPU step has its own time limit; the first failure ends the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/art
mkdir -p $O
run() { local t=$1 name=$2; shift 2; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?;
        echo "$name rc=$rc"; tail -1 $O/$name.log; [ $rc -eq 0 ] || exit $rc; }
bash scripts/profile.sh > $O/profile.log 2>&1 || { echo "profile failed"; tail -5 $O/profile.log; exit 1; }
echo profile ok
bash scripts/pmc_clock.sh > $O/clock.log 2>&1 || { echo "clock failed"; tail -5 $O/clock.log; exit 1; }
echo clock ok
run 400 bench_c2_f64 python bench.py --steps 10 --warmup 3
run 300 bench_c2_f32 python bench.py --steps 10 --warmup 3 --precision 32 --no-cpu-baseline
run 400 bench_c3_f64 python bench.py --config c3 --steps 3 --warmup 1 --no-cpu-baseline
run 400 bench_c3_f32 python bench.py --config c3 --steps 3 --warmup 1 --precision 32 --no-cpu-baseline
run 400 bench_c4_f64 python bench.py --config c4 --steps 3 --warmup 1 --no-cpu-baseline
run 300 c5_bandit python scripts/c5_bandit.py --generations 100
run 300 microbench python scripts/microbench.py all
