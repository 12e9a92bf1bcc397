#!/bin/bash
# round 3: the multi-GPU exchange on the device -- comm/merge tests, the RCCL
# path at world 1, rank-invariant bench rounds, the spawned 2-rank bench
# (gloo rehearsal on one GPU), then the default N=1 bench with its parity block.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_dist.py tests/test_gpu_rccl.py tests/test_gpu_fullsize.py "tests/test_gpu_parity.py::test_gp_score_values_equals_score_of_encoded" -x -v -s --timeout 300 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/r03_dist_tests.log 2>&1
rc=$?; echo "dist tests rc=$rc"; tail -15 gpurun_out/r03_dist_tests.log; [ $rc -eq 0 ] || exit $rc
UT_DIST_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --m 65536 --steps 3 --warmup 1 --no-cpu-baseline \
  > gpurun_out/r03_bench_2rank_gloo.log 2>&1
rc=$?; echo "bench 2-rank rc=$rc"; tail -c 3000 gpurun_out/r03_bench_2rank_gloo.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --steps 10 --warmup 3 > gpurun_out/r03_bench_c2.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -c 4000 gpurun_out/r03_bench_c2.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/prof_c5_host.py 256 > gpurun_out/r03_prof_c5.log 2>&1
rc=$?; echo "prof rc=$rc"; tail -3 gpurun_out/r03_prof_c5.log
exit $rc
