#!/bin/bash
# round 4: fit waves at s_setprio 3 + hash grids capped at N workgroups per CU
# (UT_FIT_SETPRIO=1, UT_HASH_WG_PER_CU=N): C3 pruned / f16x3 / C2 / C4
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r04t; mkdir -p $O
run() { local t=$1 name=$2; shift 2; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?;
        echo "$name rc=$rc"; tail -1 $O/$name.log | cut -c1-120; [ $rc -eq 0 ] || exit $rc; }
B="--steps 3 --warmup 1 --no-cpu-baseline --no-parity"
export UT_FIT_SETPRIO=1
for n in 2 3 5 6 8; do
  UT_HASH_WG_PER_CU=$n run 300 c3p_cap$n python bench.py --config c3 --prune 256 $B
done
for n in 0 3 4 6; do
  UT_HASH_WG_PER_CU=$n run 300 c3h_cap$n python bench.py --config c3 --precision 16 $B
done
for n in 0 4 6; do
  UT_HASH_WG_PER_CU=$n run 300 c2_cap$n python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-parity
done
for n in 0 4; do
  UT_HASH_WG_PER_CU=$n run 300 c4_cap$n python bench.py --config c4 $B
done
