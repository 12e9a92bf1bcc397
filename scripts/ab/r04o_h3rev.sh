#!/bin/bash
# round 4: k_gp_var_h3 with the pair's short tile in descending k (UT_H3_REV):
# f16x3 tests, C3 / C2 f16x3 rounds on / off, FETCH and clock of the kernel
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r04o; mkdir -p $O
run() { local t=$1 name=$2; shift 2; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?;
        echo "$name rc=$rc"; tail -1 $O/$name.log | cut -c1-120; [ $rc -eq 0 ] || exit $rc; }
run 400 pytest python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 300 --timeout-method thread -k "16 or h3 or precision or c3"
H="python bench.py --config c3 --precision 16 --steps 3 --warmup 1 --no-cpu-baseline --no-parity"
for i in 1 2; do for r in 1 0; do UT_H3_REV=$r run 300 c3h_rev${r}_$i $H; done; done
for r in 1 0; do UT_H3_REV=$r run 300 c2h_rev$r python bench.py --precision 16 --steps 10 --warmup 3 --no-cpu-baseline --no-parity; done
for r in 1 0; do
  UT_H3_REV=$r timeout -s KILL 150 rocprofv3 --kernel-trace --pmc FETCH_SIZE GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES -d $O/pmc_rev$r -o run --output-format csv -- python3 bench.py --config c3 --precision 16 --steps 2 --warmup 1 --no-cpu-baseline --no-parity > $O/pmc_rev$r.log 2>&1
  rc=$?; echo "pmc rev$r rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
