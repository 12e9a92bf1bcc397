#!/bin/bash
# round 3: small-m ut_hash (inner digests of every (param, candidate) first)
# against the head library, then every GPU test on the new one
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/hsmall
mkdir -p $O
for L in scripts/exp/lib/libuthot_head.so uptune_amd/libuthot.so; do
  echo "== $L"
  UTHOT_LIB=$PWD/$L timeout -k 10 300 python scripts/exp/hash_small_m.py > $O/hs.log 2>&1 || { echo "rc=$?"; tail -5 $O/hs.log; exit 1; }
  grep "m=2" $O/hs.log
done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/c5_bandit.py --generations 100 --prune 256 > $O/c5p.log 2>&1 || { echo "c5 rc=$?"; exit 1; }
tail -c 700 $O/c5p.log
