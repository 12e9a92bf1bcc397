#!/bin/bash
# round 5 A/B: precision-8 variance GEMM with / without the wait for the side
# stream's dup mask before it (UTX_NOJOIN), C2 / C3 / C4 lines, alternating.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r05_varjoin2; mkdir -p $O
for rep in 1 2; do
for j in 0 1; do
  UTX_NOJOIN=$j timeout -k 10 200 python bench.py --no-cpu-baseline --no-parity > $O/c2_j${j}_$rep.log 2>&1 || exit 1
  UTX_NOJOIN=$j timeout -k 10 300 python bench.py --config c3 --steps 3 --warmup 1 --no-cpu-baseline --no-parity > $O/c3_j${j}_$rep.log 2>&1 || exit 1
  UTX_NOJOIN=$j timeout -k 10 300 python bench.py --config c4 --steps 4 --warmup 1 --no-cpu-baseline --no-parity > $O/c4_j${j}_$rep.log 2>&1 || exit 1
  for c in c2 c3 c4; do python -c "
import json; l=[x for x in open('$O/${c}_j${j}_$rep.log') if x.startswith('{')][-1]; j=json.loads(l)
print('$c nojoin=$j rep $rep', round(j['ms_per_step'],3), {k: round(v,2) for k,v in j['stage_ms'].items()})"; done
done
done
