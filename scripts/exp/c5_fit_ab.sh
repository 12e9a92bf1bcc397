cd "${GRAFT_REPO_ROOT:-.}"
for rep in 1 2; do
for cfg in "1 1" "0 1" "1 0"; do set -- $cfg
UT_FIT_FIRST=$1 UT_JOIN_FIT=$2 timeout -k 10 200 python scripts/c5_bandit.py --generations 100 --prune 256 > gpurun_out/c5ab.log 2>&1 || { tail -5 gpurun_out/c5ab.log; exit 1; }
tail -1 gpurun_out/c5ab.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('fit_first=$1 join=$2', round(d['wall_s'],3), d['best'], round(d['end_to_end_vs_mix'],3), {k: round(v['ms'],2) for k,v in d['technique_round_ms'].items()})"
done; done
