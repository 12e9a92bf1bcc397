#!/bin/bash
# round 6: where the ~0.65 ms per C2 round between the main-stream stages and
# the wall goes -- cProfile of the bench loop (host time per call) and a HIP
# API + kernel trace of a short run
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r06_gap; mkdir -p $O
timeout -k 10 300 python -m cProfile -o $O/bench.prof bench.py --steps 200 --warmup 5 --no-cpu-baseline --no-secondary \
  --no-parity > $O/prof_bench.log 2>&1 || { tail -20 $O/prof_bench.log; exit 1; }
python - <<PY > $O/prof_top.txt
import pstats
p = pstats.Stats('$O/bench.prof'); p.sort_stats('tottime').print_stats(40)
PY
echo cprofile ok
timeout -k 10 300 rocprofv3 --hip-runtime-trace --kernel-trace -d $O/tr -o run --output-format csv -- \
  python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-secondary --no-parity > $O/trace.log 2>&1 || { tail -20 $O/trace.log; exit 1; }
echo trace ok
