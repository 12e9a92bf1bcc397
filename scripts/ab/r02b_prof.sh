#!/bin/bash
# Round-2 (second session) artefacts: rocprofv3 stats + HBM counters of the
# default C2 round, per-kernel clock / MFMA busy, and the secondary bench
# lines (C3 dense + pruned, C4, f16x3).  Every GPU step has its own limit and
# a failure ends the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
set -e
bash scripts/ab/r02_prof.sh
bash scripts/pmc_clock.sh
python3 scripts/clock_summary.py gpurun_out/clk > gpurun_out/clock.json
if [ -z "$NO_BENCH" ]; then
  timeout -k 10 600 python bench.py --config c3 --steps 3 --warmup 1 > gpurun_out/bench_c3_f64.log 2>&1
  tail -1 gpurun_out/bench_c3_f64.log | cut -c1-200
  timeout -k 10 300 python bench.py --config c3 --prune 256 --steps 5 --warmup 2 > gpurun_out/bench_c3_prune.log 2>&1
  tail -1 gpurun_out/bench_c3_prune.log | cut -c1-200
  timeout -k 10 300 python bench.py --config c4 --steps 5 --warmup 2 > gpurun_out/bench_c4.log 2>&1
  tail -1 gpurun_out/bench_c4.log | cut -c1-200
  timeout -k 10 300 python bench.py --precision 16 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench_c2_h3.log 2>&1
  tail -1 gpurun_out/bench_c2_h3.log | cut -c1-200
fi
