#!/bin/bash
# round 3: the f16x3 K* epilogue with the split scale folded into the exp table
# and the lo plane taken in f32 -- parity, the C2 / C3 f16x3 lines, and the
# rocprofv3 passes of the C2 f16x3 round (for the var16 / kstar16 records)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/h3k
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 150 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for spec in "c2 10" "c3 5"; do set -- $spec
  timeout -k 10 300 python bench.py --config $1 --precision 16 --steps $2 --warmup 2 --no-cpu-baseline > $O/bench_$1.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "bench $1 rc=$rc"; tail -5 $O/bench_$1.log; exit $rc; }
  tail -1 $O/bench_$1.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$1 p16', round(d['ms_per_step'],2), 'ms', round(d['value']/1e6,2), 'M/s', {k: round(v,2) for k,v in d['stage_ms'].items()}, 'parity', (d.get('parity') or {}).get('all_ok'))"
done
PROF_OUT=gpurun_out/prof16 BENCH_ARGS="--precision 16 --steps 5 --warmup 2 --no-cpu-baseline --no-parity" bash scripts/profile.sh > $O/profile.log 2>&1 || { echo "profile failed"; tail -5 $O/profile.log; exit 1; }
PROF_OUT=gpurun_out/clk16 BENCH_ARGS="--precision 16 --steps 5 --warmup 2 --no-cpu-baseline --no-parity" bash scripts/pmc_clock.sh > $O/clock.log 2>&1 || { echo "clock failed"; tail -5 $O/clock.log; exit 1; }
echo prof ok
