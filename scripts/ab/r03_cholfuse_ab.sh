#!/bin/bash
# round 3: the refit with the next diagonal block factored inside the trailing
# update (UT_CHOL_FUSE=1): every GPU test under it, the fit alone, then the C3
# lines and C2 with / without it; then the hash-beside-fit schedule knobs
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/cholfuse
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_default.log 2>&1
rc=$?; echo "pytest (default) rc=$rc"; tail -3 $O/pytest_default.log; [ $rc -eq 0 ] || exit $rc
UT_CHOL_FUSE=1 timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; echo "pytest (fused) rc=$rc"; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for f in 0 1; do
  UT_CHOL_FUSE=$f timeout -k 10 300 python scripts/exp/fit_alone.py > $O/fa.log 2>&1 || { echo "fit_alone rc=$?"; tail -5 $O/fa.log; exit 1; }
  echo "fuse=$f"; cat $O/fa.log | grep "n="
done
bash scripts/ab/r03_fitsched_ab.sh
