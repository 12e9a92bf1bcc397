#!/bin/bash
# round 4: f16x3 dense rounds with the hash enqueued after K* (UT_HASH_AFTER_KSTAR=1)
# now that the fit's waves run at s_setprio 3
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r04ab; mkdir -p $O
run() { local t=$1 name=$2; shift 2; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?;
        echo "$name rc=$rc"; tail -1 $O/$name.log | cut -c1-120; [ $rc -eq 0 ] || exit $rc; }
A="--precision 16 --steps 10 --warmup 3 --no-cpu-baseline --no-parity"
B="--config c3 --precision 16 --steps 3 --warmup 1 --no-cpu-baseline --no-parity"
for v in 0 1; do
  UT_HASH_AFTER_KSTAR=$v run 300 c2h3_late$v python bench.py $A
  UT_HASH_AFTER_KSTAR=$v run 300 c3h_late$v python bench.py $B
done
UT_HASH_AFTER_KSTAR=1 UT_HASH_WG_PER_CU=0 run 300 c2h3_late1_nocap python bench.py $A
