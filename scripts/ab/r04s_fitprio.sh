#!/bin/bash
# round 4: the fit chain beside the hash -- fit waves at s_setprio 3
# (UT_FIT_SETPRIO), with and without the hash-grid cap (UT_HASH_WG_PER_CU);
# C3 pruned / f16x3, C2; then the fit's kernel stats standalone
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r04s; mkdir -p $O
export TMPDIR=/tmp
run() { local t=$1 name=$2; shift 2; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?;
        echo "$name rc=$rc"; tail -1 $O/$name.log | cut -c1-120; [ $rc -eq 0 ] || exit $rc; }
B="--steps 3 --warmup 1 --no-cpu-baseline --no-parity"
for v in 1 0; do
  UT_FIT_SETPRIO=$v run 300 c3p_prio$v python bench.py --config c3 --prune 256 $B
  UT_FIT_SETPRIO=$v run 300 c3h_prio$v python bench.py --config c3 --precision 16 $B
done
UT_FIT_SETPRIO=1 UT_HASH_WG_PER_CU=4 run 300 c3p_prio1_cap4 python bench.py --config c3 --prune 256 $B
UT_FIT_SETPRIO=0 UT_HASH_WG_PER_CU=4 run 300 c3p_prio0_cap4 python bench.py --config c3 --prune 256 $B
UT_FIT_SETPRIO=1 UT_FIT_PRIORITY=1 run 300 c3p_prio1_sprio python bench.py --config c3 --prune 256 $B
for v in 1 0; do
  UT_FIT_SETPRIO=$v run 300 c2_prio$v python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-parity
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o fit --output-format csv -- python scripts/microbench.py fit > $O/fit_prof.log 2>&1 || exit $?
find $O/prof -name "*kernel_stats.csv" -exec cp {} $O/fit_kernel_stats.csv \;
rm -rf $O/prof
