cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 python scripts/microbench.py hash > gpurun_out/mh_new.json 2>&1 || exit 1
UTHOT_LIB=$PWD/gpurun_tmp/libuthot_h3w.so timeout -k 10 200 python scripts/microbench.py hash > gpurun_out/mh_old.json 2>&1 || exit 1
python - <<'PY'
import json
for f in ("mh_new", "mh_old"):
    s = open(f"gpurun_out/{f}.json").read(); d = json.loads(s[s.index("{"):])["hash"]
    print(f, {k: round(v["ms"], 3) for k, v in d.items()})
PY
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_history.py tests/test_gpu_c4.py -x -q --timeout 150 --timeout-method thread -p no:cacheprovider -k "hash or de or DE or digest or c4 or ga or pso or perm or history" 2>&1 | tail -2
