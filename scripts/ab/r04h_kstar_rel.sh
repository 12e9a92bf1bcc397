#!/bin/bash
# round 4: parent-relative K* for pruned GA / GGA rounds (ut_gp_topk_pruned_ref)
# -- parity tests, the C5 pruned loop with it on / off, kernel stats of the loop
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r04h; mkdir -p $O
run() { local t=$1 name=$2; shift 2; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?;
        echo "$name rc=$rc"; tail -1 $O/$name.log | cut -c1-250; [ $rc -eq 0 ] || exit $rc; }
run 300 pytest_rel python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_c5.py -m gpu -q --timeout 200 --timeout-method thread -k "parent_relative or pruned"
for i in 1 2; do for r in 1 0; do
  UT_KSTAR_REL=$r run 300 c5_rel${r}_$i python scripts/c5_bandit.py --prune 256
done; done
run 300 c5_trace rocprofv3 --kernel-trace --stats -d $O/c5_trace -o run --output-format csv -- python3 scripts/c5_bandit.py --prune 256
