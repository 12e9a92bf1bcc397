cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/prof
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_c4.py -k "ga or c4 or parent or score_values or gp" > gpurun_out/ga_tests.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/ga_tests.log; exit 1; }
tail -2 gpurun_out/ga_tests.log
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/c4ga -o run --output-format csv -- \
  python3 bench.py --config c4 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/prof/c4ga.log 2>&1 || { echo "c4 rc=$?"; exit 1; }
grep '"metric"' gpurun_out/prof/c4ga.log | cut -c1-220
grep -E "k_ga|prep_cand|encode" gpurun_out/prof/c4ga/run_kernel_stats.csv | cut -c1-200
timeout -k 10 300 python bench.py --config c4 --steps 5 --warmup 2 > gpurun_out/bench_c4.log 2>&1 || { echo "c4 bench rc=$?"; exit 1; }
tail -1 gpurun_out/bench_c4.log | cut -c1-220
