#!/bin/bash
# round 3: the blocked f16x3 variance kernel -- parity (every test_gpu_parity
# case, the f16x3 ones included), then the C2 / C3 f16x3 bench lines and the
# C2 fp64 line (stage "var" = the kernel's HIP-event time)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/h3c
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for spec in "c2 16 10" "c3 16 3" "c2 64 10"; do
  set -- $spec
  timeout -k 10 300 python bench.py --config $1 --precision $2 --steps $3 --warmup 2 --no-cpu-baseline > $O/bench_$1_$2.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "bench $spec rc=$rc"; tail -5 $O/bench_$1_$2.log; exit $rc; }
  tail -1 $O/bench_$1_$2.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$1 p$2', round(d['ms_per_step'],2), 'ms/round', round(d['value']/1e6,2), 'M/s', {k: round(v,2) for k,v in d['stage_ms'].items()}, 'frac', round(d['roofline']['frac'],3), 'parity', (d.get('parity') or {}).get('all_ok'))"
done
