#!/bin/bash
# A variant of libprgpu.so with one source recompiled under extra flags (tuning experiments):
#   tools/probe/build_variant.sh <name> <source.hip> <flags...>  ->  tools/probe/lib<name>.so
# load it with PRGPU_LIB=tools/probe/lib<name>.so
set -e
cd "$(dirname "$0")/../.."
name=$1; src=$2; shift 2
objs=""
for o in build/obj/*.o; do
  b=$(basename "$o" .o)
  if [ "$b" = "$(basename "$src")" ]; then
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -pthread -ffp-contract=off -fno-fast-math \
      -Wno-unused-function -Wno-unused-variable "$@" -c -o /tmp/variant_$name.o proovread_amd/csrc/$(basename "$src")
    objs="$objs /tmp/variant_$name.o"
  else
    objs="$objs $o"
  fi
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -pthread -o tools/probe/lib$name.so $objs -lz -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
