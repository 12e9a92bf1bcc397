#!/bin/bash
# round 3: s_setprio 1 for waves 4-7 of the f16x3 variance kernel (UT_H3_PRIO=1
# build) against the in-tree library: the C2 / C3 f16x3 rounds (stage "var")
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/h3p
for L in uptune_amd/libuthot.so scripts/exp/lib/libuthot_prio.so uptune_amd/libuthot.so scripts/exp/lib/libuthot_prio.so; do
  for spec in "c2 10" "c3 3"; do set -- $spec
    UTHOT_LIB=$PWD/$L timeout -k 10 300 python bench.py --config $1 --precision 16 --steps $2 --warmup 2 --no-cpu-baseline --no-parity > gpurun_out/h3p/bk.log 2>&1 || { tail -5 gpurun_out/h3p/bk.log; exit 1; }
    tail -1 gpurun_out/h3p/bk.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$L $1', round(d['ms_per_step'],2), {k: round(v,2) for k,v in d['stage_ms'].items() if k in ('kstar','hash','var')})"
  done
done
