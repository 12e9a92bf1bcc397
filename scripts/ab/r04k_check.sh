#!/bin/bash
# round 4: K* epilogue without per-element branches -- GPU suite, then every
# bench line (C2 x2, C3 pruned, C3 f16x3, C4, C5 pruned / dense) and kernel stats
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r04k; mkdir -p $O
run() { local t=$1 name=$2; shift 2; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?;
        echo "$name rc=$rc"; tail -1 $O/$name.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc; }
run 900 pytest python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
run 300 c2a python bench.py --steps 10 --warmup 3 --no-cpu-baseline
run 300 c2b python bench.py --steps 10 --warmup 3 --no-cpu-baseline
run 400 c3p python bench.py --config c3 --prune 256 --steps 3 --warmup 1 --no-cpu-baseline
run 400 c3h python bench.py --config c3 --precision 16 --steps 3 --warmup 1 --no-cpu-baseline
run 400 c4 python bench.py --config c4 --steps 3 --warmup 1 --no-cpu-baseline
run 300 c5p python scripts/c5_bandit.py --prune 256
run 300 c5d python scripts/c5_bandit.py
run 300 tr_c2 rocprofv3 --kernel-trace --stats -d $O/tr_c2 -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-parity
run 400 tr_c3p rocprofv3 --kernel-trace --stats -d $O/tr_c3p -o run --output-format csv -- python3 bench.py --config c3 --prune 256 --steps 2 --warmup 1 --no-cpu-baseline --no-parity
