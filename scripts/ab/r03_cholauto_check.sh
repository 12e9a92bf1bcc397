#!/bin/bash
# round 3: the refit's fused update + diagonal block on from 2048 padded rows
# (default): every GPU test, then C2, C3 pruned, C3 f16x3 and the C5 pruned loop
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/cholauto
mkdir -p $O
run() { local t=$1 name=$2; shift 2; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?;
        echo "$name rc=$rc"; tail -c 300 $O/$name.log; echo; [ $rc -eq 0 ] || exit $rc; }
run 900 pytest_gpu python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider
run 300 smoke python -c "import __graft_entry__ as g; g.smoke()"
run 400 bench_c2 python bench.py
run 400 bench_c3_prune python bench.py --config c3 --prune 256 --steps 5 --warmup 2 --no-cpu-baseline
run 400 bench_c3_h3 python bench.py --config c3 --precision 16 --steps 5 --warmup 2 --no-cpu-baseline
run 300 c5_prune python scripts/c5_bandit.py --generations 100 --prune 256
