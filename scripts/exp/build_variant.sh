#!/bin/bash
# build a variant of libuthot.so with extra defines for propose.hip:
#   scripts/exp/build_variant.sh NAME -DFOO=1 ...  ->  gpurun_tmp/libuthot_NAME.so
set -e
cd "$(dirname "$0")/../.."
name=$1; shift
mkdir -p gpurun_tmp/obj_$name
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -Wno-unused-result "$@" \
  -c uptune_amd/csrc/propose.hip -o gpurun_tmp/obj_$name/propose.o
objs=$(ls uptune_amd/_build/*.o | grep -v propose.o)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $objs gpurun_tmp/obj_$name/propose.o -o gpurun_tmp/libuthot_$name.so
