#!/bin/bash
# round 4: which change moves the C5 pruned history -- the pruned-equals-dense
# C5 test and the C5 pruned loop under UT_KSTAR_REL x UT_EARLY_ALPHA
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r04i; mkdir -p $O
for cfg in "0 1" "1 0" "0 0" "1 1"; do
  set -- $cfg
  UT_KSTAR_REL=$1 UT_EARLY_ALPHA=$2 timeout -k 10 300 python -u -m pytest tests/test_gpu_c5.py -m gpu -q --timeout 200 --timeout-method thread -k "pruned_scoring_equals_dense" > $O/t_rel$1_ea$2.log 2>&1
  rc=$?; echo "test rel=$1 ea=$2 rc=$rc $(tail -1 $O/t_rel$1_ea$2.log)"; [ $rc -le 1 ] || exit $rc
  UT_KSTAR_REL=$1 UT_EARLY_ALPHA=$2 timeout -k 10 300 python scripts/c5_bandit.py --prune 256 > $O/c5_rel$1_ea$2.log 2>&1
  rc=$?; echo "c5 rel=$1 ea=$2 rc=$rc"; [ $rc -eq 0 ] || exit $rc
  tail -1 $O/c5_rel$1_ea$2.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['best'], d['wall_s'], d['end_to_end_vs_round'], d['technique_round_ms'])"
done
timeout -k 10 300 python scripts/c5_bandit.py > $O/c5_dense.log 2>&1; echo "dense rc=$?"
tail -1 $O/c5_dense.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['best'], d['wall_s'])"
