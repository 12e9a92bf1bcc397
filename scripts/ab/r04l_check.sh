#!/bin/bash
# round 4: K* exponent in 2^(1/256) units -- GPU suite, bench lines, and the
# f16x3 C3 round with the hash forked before K* (UT_HASH_AFTER_KSTAR=0)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r04l; mkdir -p $O
run() { local t=$1 name=$2; shift 2; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?;
        echo "$name rc=$rc"; tail -1 $O/$name.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc; }
run 900 pytest python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
run 300 c2a python bench.py --steps 10 --warmup 3 --no-cpu-baseline
run 300 c2b python bench.py --steps 10 --warmup 3 --no-cpu-baseline
run 400 c3p python bench.py --config c3 --prune 256 --steps 3 --warmup 1 --no-cpu-baseline
run 400 c3h python bench.py --config c3 --precision 16 --steps 3 --warmup 1 --no-cpu-baseline
UT_HASH_AFTER_KSTAR=0 run 400 c3h_early_hash python bench.py --config c3 --precision 16 --steps 3 --warmup 1 --no-cpu-baseline
run 400 c4 python bench.py --config c4 --steps 3 --warmup 1 --no-cpu-baseline
run 300 c5p python scripts/c5_bandit.py --prune 256
run 300 c5d python scripts/c5_bandit.py
