#!/bin/bash
# Build libhalo_rx.so as of git revision <rev> into tools/exp/libhalo_rx_<name>.so (tools only).
# usage: tools/exp/build_rev.sh <rev> <name> [-DMACRO=1 ...]
set -e
cd "$(dirname "$0")/../.."
rev=$1; name=$2; shift 2
tmp=$(mktemp -d /tmp/halo_rev.XXXXXX)
git archive "$rev" halo_amd/csrc include | tar -x -C "$tmp"
C=$tmp/halo_amd/csrc
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -fvisibility=hidden "$@" -I$tmp/include -I$C \
  $C/*.hip $C/*.cc -o tools/exp/libhalo_rx_$name.so
rm -rf "$tmp"
