#!/bin/bash
# round 4: k_gp_var_pp item order A/B (UT_VAR_SCHED 0 = strip-major, 1 = paired row
# tiles in XCD groups), GP parity tests first, then HBM bytes + clock of the var kernel
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r04c; mkdir -p $O
run() { local t=$1 name=$2; shift 2; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?;
        echo "$name rc=$rc"; tail -1 $O/$name.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc; }
UT_VAR_SCHED=1 run 600 pytest python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 300 --timeout-method thread -k "gp or var or prune or score or round or c3"
for i in 1 2; do for s in 0 1; do
  UT_VAR_SCHED=$s run 300 c2_s${s}_$i python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-parity
done; done
for s in 0 1; do
  UT_VAR_SCHED=$s PROF_OUT=$O/clk_s$s bash scripts/pmc_clock.sh > $O/clk_s$s.log 2>&1 || { echo clk fail; exit 1; }
  UT_VAR_SCHED=$s timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $O/fetch_s$s -o run --output-format csv -- \
    python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-parity > $O/fetch_s$s.log 2>&1 || { echo fetch fail; exit 1; }
  echo "prof s$s ok"
done
