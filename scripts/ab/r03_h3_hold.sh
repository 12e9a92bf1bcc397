#!/bin/bash
# round 3: fp32 / f16x3 dense rounds with the hash held for the in-flight fit
# (UT_HASH_HOLD_LOWPREC=1) vs not (0), C3 and C2.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/h3hold
O=gpurun_out/h3hold
for cfg in c3 c2; do
  for p in 16 32; do
    for L in 0 1 0 1; do
      st=10; [ $cfg = c3 ] && st=3
      UT_HASH_HOLD_LOWPREC=$L timeout -k 10 300 python bench.py --config $cfg --precision $p --steps $st --warmup 2 --no-cpu-baseline --no-parity > $O/bench_${cfg}_${p}_$L.log 2>&1
      rc=$?; [ $rc -eq 0 ] || { echo "bench $cfg L=$L rc=$rc"; tail -5 $O/bench_${cfg}_${p}_$L.log; exit $rc; }
      tail -1 $O/bench_${cfg}_${p}_$L.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$cfg p$p hold=$L', round(d['ms_per_step'],2), 'ms/round', {k: round(v,2) for k,v in d['stage_ms'].items()})"
    done
    [ $cfg = c3 ] && [ $p = 16 ] && continue
  done
done
