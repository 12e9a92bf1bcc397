#!/bin/bash
# round 6 first GPU call: the changed tests, the bench line with the ell = 2
# secondary, then the precision-8 profile passes at both lengthscales
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
timeout -k 10 400 python -u -m pytest -x -v --timeout 150 --timeout-method thread -m gpu tests/test_gpu_rccl.py tests/test_gpu_i8.py \
  "tests/test_gpu_parity.py::test_pruned_entry_points_share_one_categorical_fit" > gpurun_out/r06a_tests.log 2>&1 || { echo tests failed; tail -30 gpurun_out/r06a_tests.log; exit 1; }
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r06a_bench.log 2>&1 || { echo bench failed; tail -20 gpurun_out/r06a_bench.log; exit 1; }
TAG=r06a bash scripts/r06_prof.sh
