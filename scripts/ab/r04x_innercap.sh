#!/bin/bash
# round 4: the inner-digest kernel capped beside fits of >= 1024 padded rows
# (C2 f16x3), the outer hash beside fits of >= 2048 (C3); vs no cap
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r04x; mkdir -p $O
run() { local t=$1 name=$2; shift 2; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?;
        echo "$name rc=$rc"; tail -1 $O/$name.log | cut -c1-120; [ $rc -eq 0 ] || exit $rc; }
A="--steps 10 --warmup 3 --no-cpu-baseline --no-parity"
B="--steps 3 --warmup 1 --no-cpu-baseline --no-parity"
run 300 c2h3 python bench.py --precision 16 $A
UT_HASH_WG_PER_CU=0 run 300 c2h3_off python bench.py --precision 16 $A
run 300 c2 python bench.py $A
run 300 c3p python bench.py --config c3 --prune 256 $B
run 300 c3h python bench.py --config c3 --precision 16 $B
run 300 c5p python scripts/c5_bandit.py --generations 100 --prune 256
run 300 c5d python scripts/c5_bandit.py --generations 100
