#!/bin/bash
# round 3: the C5 loop end to end (dense and pruned) after the host-path work,
# the technique / C5 GPU tests, and the host profile of the pruned loop.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_c5.py tests/test_gpu_c5_oracle.py tests/test_gpu_technique.py tests/test_gpu_refbinding.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/r03_c5_tests.log 2>&1
rc=$?; echo "c5 tests rc=$rc"; tail -8 gpurun_out/r03_c5_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/c5_bandit.py --generations 100 > gpurun_out/r03_c5_dense.log 2>&1
rc=$?; echo "c5 dense rc=$rc"; tail -c 1500 gpurun_out/r03_c5_dense.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/c5_bandit.py --generations 100 --prune 256 > gpurun_out/r03_c5_prune.log 2>&1
rc=$?; echo "c5 prune rc=$rc"; tail -c 1500 gpurun_out/r03_c5_prune.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/prof_c5_host.py 256 > gpurun_out/r03_prof_c5.log 2>&1
rc=$?; echo "prof rc=$rc"; tail -3 gpurun_out/r03_prof_c5.log
exit $rc
