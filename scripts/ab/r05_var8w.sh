#!/bin/bash
# round 5 A/B: k_gp_var_i8w (one 8-wave workgroup per CU, 128 x 128 tiles,
# 3-stage ring) against k_gp_var_i8 (UTX_VAR8W=1 / 0): the i8 tests with the
# new kernel, then C2 and C3 f64-tier lines alternating.
# (k_gp_var_i8w and the UTX_VAR8W knob were removed after this A/B: slower at C2, 2% faster at C3)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r05_var8w; mkdir -p $O
UTX_VAR8W=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_i8.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for rep in 1 2; do
for v in 0 1; do
  UTX_VAR8W=$v timeout -k 10 300 python bench.py --no-cpu-baseline > $O/c2_w${v}_$rep.log 2>&1 || { tail -20 $O/c2_w${v}_$rep.log; exit 1; }
  python -c "
import json; l=[x for x in open('$O/c2_w${v}_$rep.log') if x.startswith('{')][-1]; j=json.loads(l)
print('c2 w$v rep $rep', round(j['ms_per_step'],3), j['parity'].get('all_ok'), round(j['roofline']['frac'],3), {k: round(v,2) for k,v in j['stage_ms'].items()})"
done
done
for v in 0 1; do
  UTX_VAR8W=$v timeout -k 10 400 python bench.py --config c3 --steps 3 --warmup 1 --no-cpu-baseline > $O/c3_w$v.log 2>&1 || { tail -20 $O/c3_w$v.log; exit 1; }
  python -c "
import json; l=[x for x in open('$O/c3_w$v.log') if x.startswith('{')][-1]; j=json.loads(l)
print('c3 w$v', round(j['ms_per_step'],3), j['parity'].get('all_ok'), round(j['roofline']['frac'],3), round(j['stage_ms']['var'],2))"
done
