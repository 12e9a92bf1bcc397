#!/bin/bash
# round 3: fp64 variance tickets row-tile-major in groups of G strips per XCD
# (UT_VAR_GROUP builds) against the in-tree library: the C2 and C3 dense rounds
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/vg
for L in uptune_amd/libuthot.so scripts/exp/lib/libuthot_vg4.so scripts/exp/lib/libuthot_vg8.so uptune_amd/libuthot.so scripts/exp/lib/libuthot_vg4.so scripts/exp/lib/libuthot_vg8.so; do
  for spec in "c2 10"; do set -- $spec
    UTHOT_LIB=$PWD/$L timeout -k 10 300 python bench.py --config $1 --steps $2 --warmup 2 --no-cpu-baseline > gpurun_out/vg/bk.log 2>&1 || { tail -5 gpurun_out/vg/bk.log; exit 1; }
    tail -1 gpurun_out/vg/bk.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$L $1', round(d['ms_per_step'],2), d.get('parity',{}).get('all_ok'), {k: round(v,2) for k,v in d['stage_ms'].items() if k in ('kstar','hash','var')})"
  done
done
