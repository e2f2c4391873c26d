#!/bin/bash
# Build an experimental libhalo_rx.so variant into tools/exp/libhalo_rx_<name>.so (tools only).
# usage: tools/exp/build_variant.sh <name> [-DMACRO=1 ...]
set -e
cd "$(dirname "$0")/../.."
name=$1; shift
C=halo_amd/csrc
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -fvisibility=hidden "$@" -Iinclude -I$C \
  $C/*.hip $C/*.cc \
  -o tools/exp/libhalo_rx_$name.so
