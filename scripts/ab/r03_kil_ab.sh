#!/bin/bash
# round 3: K* with the next stage's loads spread over the current stage's k4
# sub-steps (UT_KSTAR_IL=1 build) against the in-tree library: K* alone
# (kstar_micro), then the C2, C3 pruned and C3 f16x3 rounds (stage times)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/kil
for L in uptune_amd/libuthot.so scripts/exp/lib/libuthot_kil.so uptune_amd/libuthot.so scripts/exp/lib/libuthot_kil.so; do
  echo "== $L"
  UTHOT_LIB=$PWD/$L timeout -k 10 200 python scripts/exp/kstar_micro.py > gpurun_out/kil/micro.log 2>&1 || { tail -5 gpurun_out/kil/micro.log; exit 1; }
  tail -1 gpurun_out/kil/micro.log
  for spec in "c2 64 0 10" "c3 64 256 5" "c3 16 0 3"; do set -- $spec
    UTHOT_LIB=$PWD/$L timeout -k 10 300 python bench.py --config $1 --precision $2 --prune $3 --steps $4 --warmup 2 --no-cpu-baseline > gpurun_out/kil/bk.log 2>&1 || { tail -5 gpurun_out/kil/bk.log; exit 1; }
    tail -1 gpurun_out/kil/bk.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$1 p$2 prune$3', round(d['ms_per_step'],2), d.get('parity',{}).get('all_ok'), {k: round(v,2) for k,v in d['stage_ms'].items()})"
  done
done
