#!/bin/bash
# h3 ring-shape comparison: parity of the default ring, then C2 / C3 bench lines per ring
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/h3ring; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "gp_vs_oracle" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for ring in 16x6 32x3; do for cfg in c2 c3; do
  st=10; [ $cfg = c3 ] && st=3
  UT_H3_RING=$ring timeout -k 10 300 python bench.py --config $cfg --precision 16 --steps $st --warmup 1 --no-cpu-baseline > $O/b_${ring}_$cfg.log 2>&1
  rc=$?; echo "ring $ring $cfg rc=$rc"; [ $rc -eq 0 ] || exit $rc
  tail -1 $O/b_${ring}_$cfg.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['value']/1e6,2), round(d['ms_per_step'],2), {k: round(v,2) for k,v in d['stage_ms'].items()}, round(d['roofline']['frac'],3))"
done; done
