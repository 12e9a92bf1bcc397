#!/bin/bash
# round 3: the C5 pruned loop with / without selections joining the dedup set at round time
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/noteab
mkdir -p $O
for rep in 1 2 3; do for v in on off; do
  timeout -k 10 300 python scripts/exp/c5_note_ab.py $v > $O/$v.log 2>&1 || { echo "$v rc=$?"; tail -5 $O/$v.log; exit 1; }
  python3 -c "import json; d=json.loads([l for l in open('$O/$v.log') if l.startswith('{')][-1]); print('$v', d['best'], round(d['wall_s'],3), round(d['seed_s'],3), round(d['end_to_end_vs_round'],3))"
done; done
