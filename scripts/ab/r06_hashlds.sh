#!/bin/bash
# (not kept: var_wait 0 but the hash 10-18 ms and the rounds 19.7-22.8 ms; the knob was removed -- profiles/r06_kq_ab.txt)
# round 6 A/B: the round's hash kernels reserving unused dynamic LDS
# (UTX_HASH_LDS bytes) so that at most 3 / 2 of their workgroups sit on a CU
# and the refit's kernels find VGPRs beside them (the variance GEMM waits
# ~1.6 ms for the refit, var_wait)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r06_hashlds; mkdir -p $O
for v in 0 45056 57344 0; do
for ell in 0.2 2; do
  f=$O/p${v}_l${ell}.log
  UTX_HASH_LDS=$v timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline \
    --no-secondary --no-parity --ell $ell > $f 2>&1 || { tail -20 $f; exit 1; }
  python -c "
import json; l=[x for x in open('$f') if x.startswith('{')][-1]; j=json.loads(l)
print('lds=$v ell=$ell', round(j['ms_per_step'],3), {k: round(v,2) for k,v in j['stage_ms'].items()})"
done
done
