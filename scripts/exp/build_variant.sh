#!/bin/bash
# build a variant of libuthot.so with extra defines for propose.hip:
#   scripts/exp/build_variant.sh NAME -DFOO=1 ...  ->  gpurun_tmp/libuthot_NAME.so
# SRC (default uptune_amd/csrc/propose.hip) is the translation unit rebuilt;
# it may be a copy elsewhere (e.g. an older revision) that includes the csrc headers
set -e
cd "$(dirname "$0")/../.."
name=$1; shift
mkdir -p gpurun_tmp/obj_$name
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -Wno-unused-result "$@" \
  -I uptune_amd/csrc -c ${SRC:-uptune_amd/csrc/propose.hip} -o gpurun_tmp/obj_$name/$(basename ${SRC:-propose.hip} .hip).o
base=$(basename ${SRC:-propose.hip} .hip); base=${base%_old}
objs=$(ls uptune_amd/_build/*.o | grep -v "/$base.o")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $objs gpurun_tmp/obj_$name/*.o -o gpurun_tmp/libuthot_$name.so
