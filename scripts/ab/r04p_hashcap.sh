#!/bin/bash
# round 4: the fit's chain beside the hash -- the hash grids capped at N
# workgroups per CU (UT_HASH_WG_PER_CU), C3 pruned / f16x3 rounds and C2
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r04p; mkdir -p $O
run() { local t=$1 name=$2; shift 2; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?;
        echo "$name rc=$rc"; tail -1 $O/$name.log | cut -c1-100; [ $rc -eq 0 ] || exit $rc; }
B="python bench.py --config c3 --prune 256 --steps 3 --warmup 1 --no-cpu-baseline --no-parity"
H="python bench.py --config c3 --precision 16 --steps 3 --warmup 1 --no-cpu-baseline --no-parity"
for n in 0 6 4 2; do
  UT_HASH_WG_PER_CU=$n run 300 c3p_cap$n $B
  UT_HASH_WG_PER_CU=$n run 300 c3h_cap$n $H
done
for n in 0 4; do UT_HASH_WG_PER_CU=$n run 300 c2_cap$n python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-parity; done
