#!/bin/bash
# round 6 A/B: the C2 round with and without the library's per-stage event
# marks (ut_set_timing) -- do the ~15 timed events per round cost wall time?
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r06_marks; mkdir -p $O
for rep in 1 2; do
for v in on off; do
  timeout -k 10 200 python - $v > $O/m_${v}_$rep.log 2>&1 <<'PY' || { tail -20 $O/m_${v}_$rep.log; exit 1; }
import runpy, sys
if sys.argv[1] == "off":
    import uptune_amd.engine as e
    e.BatchEngine.set_timing = lambda self, on: None
sys.argv = ["bench.py", "--steps", "40", "--warmup", "5", "--no-cpu-baseline", "--no-secondary", "--no-parity"]
runpy.run_path("bench.py", run_name="__main__")
PY
  python -c "
import json; l=[x for x in open('$O/m_${v}_$rep.log') if x.startswith('{')][-1]; j=json.loads(l)
print('marks=$v rep $rep', round(j['ms_per_step'],3))"
done
done
