#!/bin/bash
# round 3: K* feature padding to a multiple of 4 (the f64 MFMA's k) instead of
# 16, against the round-3 head library: K* alone (C2 d = 64: no partial stage;
# C3 d = 119 -> 120 instead of 128), the K* / pruned / f16x3 parity tests, then
# the C3 pruned and f16x3 lines and C4 with each library, twice
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/dpad
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
for L in scripts/exp/lib/libuthot_head.so uptune_amd/libuthot.so; do
  UTHOT_LIB=$PWD/$L timeout -k 10 300 python scripts/exp/kstar_micro.py > $O/km.log 2>&1 || { echo "kstar_micro rc=$?"; tail -5 $O/km.log; exit 1; }
  echo "$L kstar: $(tail -c 600 $O/km.log)"
  for spec in "c3p --config c3 --prune 256" "c3h --config c3 --precision 16" "c4 --config c4"; do set -- $spec; tag=$1; shift
    UTHOT_LIB=$PWD/$L timeout -k 10 300 python bench.py $* --steps 5 --warmup 2 --no-cpu-baseline --no-parity > $O/bk.log 2>&1 || { echo "$tag rc=$?"; tail -5 $O/bk.log; exit 1; }
    python3 -c "import json; d=json.loads([l for l in open('$O/bk.log') if l.startswith('{')][-1]); print('$L $tag', round(d['ms_per_step'],2), {k: round(v,2) for k,v in d['stage_ms'].items() if k in ('kstar','hash','var')})"
  done
done
done
