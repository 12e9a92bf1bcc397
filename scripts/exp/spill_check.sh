#!/bin/bash
# VGPR spills / scratch of every kernel in the library's HIP sources (host
# only: hipcc -Rpass-analysis); prints the kernels that spill
cd "$(dirname "$0")/../.."
for f in uptune_amd/csrc/*.hip; do
  /opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -std=c++17 -ffp-contract=off -Iuptune_amd/csrc -Iinclude -c "$f" \
    -o /tmp/spill_check.o -Rpass-analysis=kernel-resource-usage 2>&1 | sed 's/ \[-Rpass-analysis=kernel-resource-usage\]//' |
    awk -v F="$f" '/Function Name:/ {fn=$NF} /VGPRs Spill:/ {n=$NF; if (n+0 > 0) print F, fn, "spill", n}'
done
