#!/bin/bash
# K* A/B: the in-tree library vs gpurun_tmp variants (kstar_micro + C2 round)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
for L in uptune_amd/libuthot.so gpurun_tmp/libuthot_*.so; do
  echo "== $L"
  UTHOT_LIB=$PWD/$L timeout -k 10 200 python scripts/exp/kstar_micro.py 2>&1 | tail -1 || exit 1
  UTHOT_LIB=$PWD/$L timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bk.log 2>&1 || exit 1
  tail -1 gpurun_out/bk.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['ms_per_step'],3), {k: round(v,2) for k,v in d['stage_ms'].items()})"
done
