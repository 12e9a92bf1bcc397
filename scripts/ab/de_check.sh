cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_c5_oracle.py -x -q --timeout 150 --timeout-method thread -p no:cacheprovider -k "de or DE or c5 or hpl or perm" > gpurun_out/de_tests.log 2>&1
rc=$?; tail -3 gpurun_out/de_tests.log; [ $rc -ne 0 ] && { tail -40 gpurun_out/de_tests.log; exit $rc; }
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/b_aos.log 2>&1 || exit 1
UT_DE_AOS=0 timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/b_soa.log 2>&1 || exit 1
for f in b_aos b_soa; do python -c "import json;d=json.loads(open('gpurun_out/$f.log').read().strip().splitlines()[-1]);print('$f',round(d['value']/1e6,2),round(d['ms_per_step'],3),{k:round(v,3) for k,v in d['stage_ms'].items()})"; done
