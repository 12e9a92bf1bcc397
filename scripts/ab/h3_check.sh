#!/bin/bash
# f16x3 variance path: parity tests, then C2 / C3 bench lines at precision 16 (and 32 beside it)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/h3
O=gpurun_out/h3
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "gp_vs_oracle or f16x3" -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -25 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for cfg in ${H3_CONFIGS:-c2 c3}; do
  for p in ${H3_PRECS:-16 32}; do
    st=10; [ $cfg = c3 ] && st=3
    timeout -k 10 300 python bench.py --config $cfg --precision $p --steps $st --warmup 1 --no-cpu-baseline > $O/bench_${cfg}_$p.log 2>&1
    rc=$?; echo "bench $cfg $p rc=$rc"; tail -1 $O/bench_${cfg}_$p.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], {k: round(v,2) for k,v in d['stage_ms'].items()}, d['roofline']['achieved'], d['roofline']['frac'])"
    [ $rc -eq 0 ] || exit $rc
  done
done
