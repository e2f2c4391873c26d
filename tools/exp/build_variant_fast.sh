#!/bin/bash
# Like build_variant.sh, but recompiles only <file> (e.g. flow_hash.hip) with the variant's flags and
# links it with the other objects of the in-tree build (build/obj, from halo_amd/build.py).
# usage: tools/exp/build_variant_fast.sh <name> <file> [-DMACRO=1 ...]   (tools only)
set -e
cd "$(dirname "$0")/../.."
name=$1; file=$2; shift 2
C=halo_amd/csrc
O=build/obj
mkdir -p build/var
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -fvisibility=hidden -Wall "$@" -Iinclude -I$C \
  -c $C/$file -o build/var/$name.$file.o
objs=""
for o in $O/*.o; do
  [ "$(basename $o)" = "$file.o" ] || objs="$objs $o"
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -fPIC -shared $objs build/var/$name.$file.o -o tools/exp/libhalo_rx_$name.so
