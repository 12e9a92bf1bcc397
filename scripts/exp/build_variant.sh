#!/bin/bash
# build a variant of libuthot.so with extra defines for one translation unit:
#   scripts/exp/build_variant.sh NAME -DFOO=1 ...  ->  scripts/exp/lib/libuthot_NAME.so
# SRC (default uptune_amd/csrc/propose.hip) is the translation unit rebuilt;
# it may be a copy elsewhere (e.g. an older revision) that includes the csrc headers
set -e
cd "$(dirname "$0")/../.."
name=$1; shift
mkdir -p scripts/exp/lib/obj_$name
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -Wno-unused-result "$@" \
  -I uptune_amd/csrc -c ${SRC:-uptune_amd/csrc/propose.hip} -o scripts/exp/lib/obj_$name/$(basename ${SRC:-propose.hip} .hip).o
base=$(basename ${SRC:-propose.hip} .hip); base=${base%_old}
objs=$(ls uptune_amd/_build/*.o | grep -v "/$base.o")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $objs scripts/exp/lib/obj_$name/*.o -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib -o scripts/exp/lib/libuthot_$name.so
rm -rf scripts/exp/lib/obj_$name
