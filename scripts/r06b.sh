#!/bin/bash
# round 6: the precision-8 mean from the int8 variance epilogue (K* no longer
# waits for the whole fit): every GPU test, smoke, then the bench line
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-r06b}; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 150 --timeout-method thread -m gpu tests/ > $O/tests.log 2>&1 || { echo tests failed; grep -E "FAILED|Error" $O/tests.log | head -20; tail -5 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1 || { echo bench failed; tail -20 $O/bench.log; exit 1; }
python - <<PY
import json
l=[x for x in open('$O/bench.log') if x.startswith('{')][-1]; d=json.loads(l)
print('headline', round(d['value']/1e6,2), 'M/s', round(d['ms_per_step'],3), 'ms', d['parity']['all_ok'], {k: round(v,2) for k,v in d['stage_ms'].items()}, 'frac', round(d['roofline']['frac'],3))
s=d.get('secondary_ell2') or {}
print('ell2', round(s.get('value',0)/1e6,2), 'M/s', round(s.get('ms_per_step',0),3), 'ms', (s.get('parity') or {}).get('all_ok'), {k: round(v,2) for k,v in (s.get('stage_ms') or {}).items()}, 'frac', round(s['roofline']['frac'],3), s.get('i8'))
print(d['i8'])
PY
