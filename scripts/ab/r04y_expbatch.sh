#!/bin/bash
# round 4: the K* epilogue's exp table reads issued 4 at a time
# (sf2_exp2t_nonpos_n) and the diagonal blocks' inverse inside the Cholesky
# column loop (UT_CHOL_MERGED) -- parity, the fit alone, then every line
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r04y; mkdir -p $O
run() { local t=$1 name=$2; shift 2; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?;
        echo "$name rc=$rc"; tail -1 $O/$name.log | cut -c1-120; [ $rc -eq 0 ] || exit $rc; }
run 600 pytest python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_c4.py
UT_CHOL_MERGED=0 run 300 fit_sep python scripts/microbench.py fit
UT_CHOL_MERGED=1 run 300 fit_merged python scripts/microbench.py fit
A="--steps 10 --warmup 3 --no-cpu-baseline"
B="--steps 3 --warmup 1 --no-cpu-baseline"
run 300 c2 python bench.py $A
run 300 c2h3 python bench.py --precision 16 $A
run 300 c3p python bench.py --config c3 --prune 256 $B
run 300 c3h python bench.py --config c3 --precision 16 $B
run 300 c4 python bench.py --config c4 $B
run 300 c5p python scripts/c5_bandit.py --generations 100 --prune 256
UT_CHOL_MERGED=0 run 300 c3p_sep python bench.py --config c3 --prune 256 $B
