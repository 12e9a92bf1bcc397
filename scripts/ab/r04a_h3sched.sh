#!/bin/bash
# round 4: GPU tests touched by the h3 schedule / fit test, the C2 headline,
# and the k_gp_var_h3 item order A/B (UT_H3_SCHED 0 = strip-major, 1 = paired groups)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r04b; mkdir -p $O
run() { local t=$1 name=$2; shift 2; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?;
        echo "$name rc=$rc"; tail -1 $O/$name.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc; }
run 600 pytest python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_rccl.py tests/test_gpu_refbinding.py tests/test_gpu_technique.py -m gpu -x -q --timeout 120 --timeout-method thread
run 300 bench_c2 python bench.py --steps 20 --warmup 5
for s in 0 1; do
  UT_H3_SCHED=$s run 300 c3h3_s$s python bench.py --config c3 --precision 16 --steps 3 --warmup 1 --no-cpu-baseline --no-parity
  UT_H3_SCHED=$s run 300 c2h3_s$s python bench.py --precision 16 --steps 10 --warmup 3 --no-cpu-baseline --no-parity
done
UT_H3_SCHED=0 run 300 c3h3_s0b python bench.py --config c3 --precision 16 --steps 3 --warmup 1 --no-cpu-baseline --no-parity
UT_H3_SCHED=1 run 300 c3h3_s1b python bench.py --config c3 --precision 16 --steps 3 --warmup 1 --no-cpu-baseline --no-parity
