#!/bin/bash
# build a variant of libuthot.so with extra defines for some translation units:
#   SRC="uptune_amd/csrc/a.hip uptune_amd/csrc/b.hip" scripts/exp/build_variant.sh NAME -DFOO=1 ...
#   ->  scripts/exp/lib/libuthot_NAME.so
# SRC (default uptune_amd/csrc/propose.hip) lists the translation units rebuilt;
# one may be a copy elsewhere (e.g. an older revision, name ending _old) that
# includes the csrc headers
set -e
cd "$(dirname "$0")/../.."
name=$1; shift
mkdir -p scripts/exp/lib/obj_$name
skip=""
for src in ${SRC:-uptune_amd/csrc/propose.hip}; do
  base=$(basename $src .hip)
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -Wno-unused-result "$@" \
    -I uptune_amd/csrc -c $src -o scripts/exp/lib/obj_$name/$base.o
  skip="$skip /${base%_old}.o"
done
objs=$(for o in uptune_amd/_build/*.o; do keep=1; for s in $skip; do case "$o" in *$s) keep=0;; esac; done; [ $keep = 1 ] && echo $o; done)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $objs scripts/exp/lib/obj_$name/*.o -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib -o scripts/exp/lib/libuthot_$name.so
rm -rf scripts/exp/lib/obj_$name
