#!/bin/bash
# round 3: K* store forms (UT_KSTAR_ST, scripts/exp/lib variants) -- kstar_micro
# (K* alone, HIP-event stage time) then the C2 round, per library build
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/kab
for L in uptune_amd/libuthot.so scripts/exp/lib/libuthot_*.so; do
  echo "== $L"
  UTHOT_LIB=$PWD/$L timeout -k 10 200 python scripts/exp/kstar_micro.py > gpurun_out/kab/micro.log 2>&1 || { tail -5 gpurun_out/kab/micro.log; exit 1; }
  tail -1 gpurun_out/kab/micro.log
  UTHOT_LIB=$PWD/$L timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/kab/bk.log 2>&1 || { tail -5 gpurun_out/kab/bk.log; exit 1; }
  tail -1 gpurun_out/kab/bk.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['ms_per_step'],3), d.get('parity',{}).get('all_ok'), {k: round(v,2) for k,v in d['stage_ms'].items()})"
done
