#!/bin/bash
# round 3: K* items handed out statically (round-robin per XCD group, no
# ticket atomic; UT_KSTAR_STATIC=1 build) against the in-tree library
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/kst
UTHOT_LIB=$PWD/scripts/exp/lib/libuthot_static.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 150 --timeout-method thread -p no:cacheprovider > gpurun_out/kst/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/kst/pytest.log; [ $rc -eq 0 ] || exit $rc
for L in uptune_amd/libuthot.so scripts/exp/lib/libuthot_static.so uptune_amd/libuthot.so scripts/exp/lib/libuthot_static.so; do
  echo "== $L"
  UTHOT_LIB=$PWD/$L timeout -k 10 200 python scripts/exp/kstar_micro.py > gpurun_out/kst/micro.log 2>&1 || { tail -5 gpurun_out/kst/micro.log; exit 1; }
  tail -1 gpurun_out/kst/micro.log
  for spec in "c2 64 0 10" "c3 64 256 5" "c3 16 0 3"; do set -- $spec
    UTHOT_LIB=$PWD/$L timeout -k 10 300 python bench.py --config $1 --precision $2 --prune $3 --steps $4 --warmup 2 --no-cpu-baseline --no-parity > gpurun_out/kst/bk.log 2>&1 || { tail -5 gpurun_out/kst/bk.log; exit 1; }
    tail -1 gpurun_out/kst/bk.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$1 p$2 prune$3', round(d['ms_per_step'],2), {k: round(v,2) for k,v in d['stage_ms'].items() if k in ('kstar','hash','var')})"
  done
done
