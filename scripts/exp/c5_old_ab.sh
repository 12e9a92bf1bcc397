cd "${GRAFT_REPO_ROOT:-.}"
R=$PWD
for rep in 1 2 3; do
  (cd scripts/exp/old169 && timeout -k 10 200 python scripts/c5_bandit.py --generations 100 --prune 256 > $R/gpurun_out/c5old.log 2>&1) || { tail -5 gpurun_out/c5old.log; exit 1; }
  tail -1 gpurun_out/c5old.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('old169', round(d['wall_s'],3), d['best'], round(d['end_to_end_vs_round'],3))"
  timeout -k 10 200 python scripts/c5_bandit.py --generations 100 --prune 256 > gpurun_out/c5new.log 2>&1 || { tail -5 gpurun_out/c5new.log; exit 1; }
  tail -1 gpurun_out/c5new.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('new', round(d['wall_s'],3), d['best'], round(d['end_to_end_vs_round'],3), round(d['end_to_end_vs_mix'],3))"
done
