#!/bin/bash
# round 3: the per-round refit in the C3 rounds (n = 4096) against the hash
# beside it: default schedule; the side stream (hash + dedup) CU-masked so a
# few CUs per XCD stay free for the fit's chain (UT_SIDE_CU_MASK=1); pruned
# rounds' hash held until the fit is done (UT_HASH_HOLD_PRUNED=1); C2 as the
# control for the mask
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/fitsched
mkdir -p $O
one() { local tag=$1 envs=$2; shift 2
  env $envs timeout -k 10 300 python bench.py "$@" --no-cpu-baseline --no-parity > $O/x.log 2>&1 || { echo "$tag rc=$?"; tail -5 $O/x.log; exit 1; }
  python3 -c "import json; d=json.loads([l for l in open('$O/x.log') if l.startswith('{')][-1]); print('$tag', '$envs', round(d['ms_per_step'],2), {k: round(v,2) for k,v in d['stage_ms'].items() if k in ('hash','kstar','var','dedup')})"
}
for rep in 1 2; do
  for e in "X=0" "UT_CHOL_FUSE=1" "UT_SIDE_CU_MASK=1" "UT_HASH_HOLD_PRUNED=1" "UT_CHOL_FUSE=1 UT_SIDE_CU_MASK=1"; do
    one c3p "$e" --config c3 --prune 256 --steps 5 --warmup 2
  done
  for e in "X=0" "UT_CHOL_FUSE=1" "UT_SIDE_CU_MASK=1"; do
    one c3h "$e" --config c3 --precision 16 --steps 5 --warmup 2
    one c2 "$e" --steps 20 --warmup 3
  done
done
