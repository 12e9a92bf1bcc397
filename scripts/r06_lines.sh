#!/bin/bash
# round 6: the secondary bench lines and the C5 loop on the round's tree
# (precision-8 mean from the variance epilogue), one time limit per step
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=${LINES_OUT:-gpurun_out/r06_lines}; mkdir -p $O
run() { local t=$1 name=$2; shift 2; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?;
        echo "$name rc=$rc"; [ $rc -eq 0 ] || { tail -20 $O/$name.log; exit $rc; }
        python - "$O/$name.log" <<'PY'
import json, sys
ls = [x for x in open(sys.argv[1]) if x.startswith('{')]
if ls:
    j = json.loads(ls[-1])
    if 'ms_per_step' in j:
        print('  ', round(j['value'] / 1e6, 2), 'M/s', round(j['ms_per_step'], 2), 'ms parity', (j.get('parity') or {}).get('all_ok'),
              'frac', round((j.get('roofline') or {}).get('frac') or 0, 3))
    else:
        print('  ', {k: v for k, v in j.items() if not isinstance(v, (dict, list))})
else:
    print('  ', open(sys.argv[1]).read()[-300:])
PY
}
run 300 bench_c2_h3 python bench.py --precision 16 --no-cpu-baseline --no-secondary
run 400 bench_c3_i8 python bench.py --config c3 --steps 3 --warmup 1 --no-cpu-baseline
run 400 bench_c3_prune python bench.py --config c3 --prune 256 --steps 5 --warmup 2 --no-cpu-baseline
run 400 bench_c4 python bench.py --config c4 --steps 5 --warmup 2 --no-cpu-baseline
run 300 c5_dense python scripts/c5_bandit.py --generations 100
run 300 c5_prune python scripts/c5_bandit.py --generations 100 --prune 256
