#!/bin/bash
# (historical: UT_H3_KERNEL and these variants were removed in round 3, when the
# blocked 256 x 256-tile kernel replaced them; see DESIGN.md "Round 3: the f16x3 variance kernel")
# round 3: f16x3 variance kernel A/B (UT_H3_KERNEL = 0: one 8-wave workgroup
# per CU on 128 x 256 tiles; 1 / 2: two 4-wave workgroups per CU on 128 x 128
# tiles, BK 32 x 2 slots / BK 16 x 4 slots): parity at each, then the C2 / C3
# f16x3 bench lines (stage "var" = the kernel's HIP-event time).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/h3ab
O=gpurun_out/h3ab
for L in ${H3_VARIANTS:-1 2 0}; do
  UT_H3_KERNEL=$L timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "gp_vs_oracle and 16 or f16x3 or fit_append" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_$L.log 2>&1
  rc=$?; echo "pytest L=$L rc=$rc"; tail -2 $O/pytest_$L.log; [ $rc -eq 0 ] || exit $rc
done
for cfg in c2 c3; do
  for L in ${H3_VARIANTS:-1 2 0} ${H3_VARIANTS:-1 2 0}; do
    st=10; [ $cfg = c3 ] && st=3
    UT_H3_KERNEL=$L timeout -k 10 300 python bench.py --config $cfg --precision 16 --steps $st --warmup 2 --no-cpu-baseline --no-parity > $O/bench_${cfg}_$L.log 2>&1
    rc=$?; [ $rc -eq 0 ] || { echo "bench $cfg L=$L rc=$rc"; tail -5 $O/bench_${cfg}_$L.log; exit $rc; }
    tail -1 $O/bench_${cfg}_$L.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$cfg L=$L', round(d['ms_per_step'],2), 'ms/round', {k: round(v,2) for k,v in d['stage_ms'].items()}, 'frac', round(d['roofline']['frac'],3))"
  done
done
