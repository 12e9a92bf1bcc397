#!/bin/bash
# round 4: GA children's hash (ut_hash_parent) held until an in-flight fit is
# done (UT_HASH_PARENT_AFTER_FIT=1) vs beside it -- C4, C5
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r04z; mkdir -p $O
run() { local t=$1 name=$2; shift 2; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?;
        echo "$name rc=$rc"; tail -1 $O/$name.log | cut -c1-120; [ $rc -eq 0 ] || exit $rc; }
B="--steps 3 --warmup 1 --no-cpu-baseline --no-parity"
for v in 1 0; do
  UT_HASH_PARENT_AFTER_FIT=$v run 300 c4_hold$v python bench.py --config c4 $B
  UT_HASH_PARENT_AFTER_FIT=$v run 300 c5p_hold$v python scripts/c5_bandit.py --generations 100 --prune 256
  UT_HASH_PARENT_AFTER_FIT=$v run 300 c5d_hold$v python scripts/c5_bandit.py --generations 100
done
