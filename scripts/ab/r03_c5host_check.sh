#!/bin/bash
# round 3, C5 host path (one host copy per round's selections, features from
# the round's encoding, growable training-row buffers, GP buffers with
# headroom): every GPU test, the C5 loop dense and pruned, its kernel trace.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=${CHECK_OUT:-gpurun_out/c5host}
mkdir -p $O
run() { local t=$1 name=$2; shift 2; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?;
        echo "$name rc=$rc"; tail -c 400 $O/$name.log; echo; [ $rc -eq 0 ] || exit $rc; }
[ -n "$SKIP_TESTS" ] || run 1100 pytest_gpu python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider
run 300 c5_dense python scripts/c5_bandit.py --generations 100
run 300 c5_prune python scripts/c5_bandit.py --generations 100 --prune 256
run 300 c5_prune2 python scripts/c5_bandit.py --generations 100 --prune 256
bash scripts/ab/r03_c5_trace.sh
