#!/bin/bash
# round 6: host profile of the C5 pruned loop (cProfile, tottime)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r06_c5prof; mkdir -p $O
timeout -k 10 300 python -m cProfile -o $O/c5.prof scripts/c5_bandit.py --prune 256 > $O/c5.log 2>&1 || { tail -20 $O/c5.log; exit 1; }
python - <<PY > $O/top.txt
import pstats
p = pstats.Stats('$O/c5.prof'); p.sort_stats('tottime').print_stats(35)
PY
tail -1 $O/c5.log | cut -c1-300
