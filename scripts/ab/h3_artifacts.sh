#!/bin/bash
# f16x3 round artifacts: full GPU parity suite, rocprofv3 passes (scripts/ab/prof_h3.sh),
# bench lines C2 / C3 at precision 16.  First failure ends the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/h3art; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
bash scripts/ab/prof_h3.sh || exit 1
for cfg in c2 c3; do
  st=10; [ $cfg = c3 ] && st=3
  timeout -k 10 300 python bench.py --config $cfg --precision 16 --steps $st --warmup 2 --no-cpu-baseline > $O/bench_${cfg}_h3.log 2>&1
  rc=$?; echo "bench $cfg rc=$rc"; tail -1 $O/bench_${cfg}_h3.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc
done
