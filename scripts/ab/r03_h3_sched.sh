#!/bin/bash
# round 3: low-precision dense rounds with the hash enqueued after K* and the
# variance GEMM beside it (UT_HASH_AFTER_KSTAR=1) vs the default schedule (0);
# parity of the round under the new schedule first.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/h3sched
O=gpurun_out/h3sched
UT_HASH_AFTER_KSTAR=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "score_round or f16x3 or gp_vs_oracle" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for cfg in c2 c3; do
  for p in 16 32; do
    for L in 0 1 0 1; do
      st=10; [ $cfg = c3 ] && st=3
      [ $cfg = c3 ] && [ $p = 32 ] && continue
      UT_HASH_AFTER_KSTAR=$L timeout -k 10 300 python bench.py --config $cfg --precision $p --steps $st --warmup 2 --no-cpu-baseline --no-parity > $O/bench_${cfg}_${p}_$L.log 2>&1
      rc=$?; [ $rc -eq 0 ] || { echo "bench $cfg L=$L rc=$rc"; tail -5 $O/bench_${cfg}_${p}_$L.log; exit $rc; }
      tail -1 $O/bench_${cfg}_${p}_$L.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$cfg p$p late=$L', round(d['ms_per_step'],2), 'ms/round', {k: round(v,2) for k,v in d['stage_ms'].items()})"
    done
  done
done
