#!/bin/bash
# round 3: K*'s exp with the 1.5 * 2^52 shifter instead of rint + cvt
# (UT_EXP_MAGIC=1 build) -- parity, then K* alone and the C2 / C3-pruned rounds
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/mag
UTHOT_LIB=$PWD/scripts/exp/lib/libuthot_magic.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 150 --timeout-method thread -p no:cacheprovider > gpurun_out/mag/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/mag/pytest.log; [ $rc -eq 0 ] || exit $rc
for L in uptune_amd/libuthot.so scripts/exp/lib/libuthot_magic.so uptune_amd/libuthot.so scripts/exp/lib/libuthot_magic.so; do
  echo "== $L"
  UTHOT_LIB=$PWD/$L timeout -k 10 200 python scripts/exp/kstar_micro.py > gpurun_out/mag/micro.log 2>&1 || { tail -5 gpurun_out/mag/micro.log; exit 1; }
  tail -1 gpurun_out/mag/micro.log
  for spec in "c2 0 10" "c3 256 5"; do set -- $spec
    UTHOT_LIB=$PWD/$L timeout -k 10 300 python bench.py --config $1 --prune $2 --steps $3 --warmup 2 --no-cpu-baseline > gpurun_out/mag/bk.log 2>&1 || { tail -5 gpurun_out/mag/bk.log; exit 1; }
    tail -1 gpurun_out/mag/bk.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$1 prune$2', round(d['ms_per_step'],2), d.get('parity',{}).get('all_ok'), {k: round(v,2) for k,v in d['stage_ms'].items() if k in ('kstar','hash','var')})"
  done
done
