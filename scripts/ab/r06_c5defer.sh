#!/bin/bash
# round 6 A/B: the C5 loop (dense precision 8 and pruned fp64) with the staged
# fit issued after each round's proposal (UT_FIT_DEFER=1) or inside
# ut_gp_fit_async (0); the evaluated history must not change
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r06_c5defer; mkdir -p $O
for rep in 1 2; do
for v in 1 0; do
  UT_FIT_DEFER=$v timeout -k 10 240 python scripts/c5_bandit.py > $O/dense_d${v}_$rep.log 2>&1 || { tail -20 $O/dense_d${v}_$rep.log; exit 1; }
  UT_FIT_DEFER=$v timeout -k 10 240 python scripts/c5_bandit.py --prune 256 > $O/prune_d${v}_$rep.log 2>&1 || { tail -20 $O/prune_d${v}_$rep.log; exit 1; }
  for k in dense prune; do python -c "
import json; l=[x for x in open('$O/${k}_d${v}_$rep.log') if x.startswith('{')][-1]; j=json.loads(l)
print('$k defer=$v rep $rep', 'wall', round(j['wall_s'],4), 'M/s', round(j['candidates_scored_per_s']/1e6,3), 'vs_round', round(j['end_to_end_vs_round'],3), 'best', j['best'], 'evals', j['evaluations'])"; done
done
done
