#!/bin/bash
# round 4: C2 schedule -- the hash beside the variance GEMM (UT_JOIN_BEFORE_VAR=0)
# and/or beside the fit (UT_HASH_AFTER_FIT), fp64 and f16x3
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r04w; mkdir -p $O
run() { local t=$1 name=$2; shift 2; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?;
        echo "$name rc=$rc"; tail -1 $O/$name.log | cut -c1-120; [ $rc -eq 0 ] || exit $rc; }
A="--steps 10 --warmup 3 --no-cpu-baseline --no-parity"
for j in 1 0; do for h in 2 1 0; do
  UT_JOIN_BEFORE_VAR=$j UT_HASH_AFTER_FIT=$h run 300 c2_j${j}_h$h python bench.py $A
done; done
for j in 1 0; do UT_JOIN_BEFORE_VAR=$j run 300 c2h3_j$j python bench.py --precision 16 $A; done
