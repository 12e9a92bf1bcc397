#!/bin/bash
# round 3: low-precision dense rounds with the hash forked at the round start
# and K* waiting for it (UT_HASH_JOIN_KSTAR=1, with UT_HASH_AFTER_KSTAR=0 at
# n >= 2048), against the default schedule: C2 / C3 f16x3 rounds
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/hj
for rep in 1 2; do
  for env in "" "UT_HASH_JOIN_KSTAR=1 UT_HASH_AFTER_KSTAR=0"; do
    for spec in "c2 10" "c3 3"; do set -- $spec
      env $env timeout -k 10 300 python bench.py --config $1 --precision 16 --steps $2 --warmup 2 --no-cpu-baseline > gpurun_out/hj/bk.log 2>&1 || { tail -5 gpurun_out/hj/bk.log; exit 1; }
      tail -1 gpurun_out/hj/bk.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('[$env] $1', round(d['ms_per_step'],2), d.get('parity',{}).get('all_ok'), {k: round(v,2) for k,v in d['stage_ms'].items() if k in ('kstar','hash','var','finalize')})"
    done
  done
done
