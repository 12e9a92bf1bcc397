#!/bin/bash
# round 3: K* with the next item's first stage prefetched ahead of the epilogue
# stores (UT_KSTAR_PF=1 build in scripts/exp/lib) -- parity, then the K* A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/kpf
UTHOT_LIB=$PWD/scripts/exp/lib/libuthot_kpf.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -x -q --timeout 150 --timeout-method thread -p no:cacheprovider > gpurun_out/kpf/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/kpf/pytest.log; [ $rc -eq 0 ] || exit $rc
bash scripts/ab/r03_kstar_ab.sh
