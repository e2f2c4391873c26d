#!/bin/bash
# Run one command with tools/exp/libhalo_rx_<v>.so swapped in as the in-tree library, then restore
# it (tools only). usage: with_variant.sh <v> <command...>
cd "${GRAFT_REPO_ROOT:-.}"
v=$1; shift
cp halo_amd/lib/libhalo_rx.so /tmp/libhalo_rx_keep.so
cp tools/exp/libhalo_rx_$v.so halo_amd/lib/libhalo_rx.so
"$@"
rc=$?
cp /tmp/libhalo_rx_keep.so halo_amd/lib/libhalo_rx.so
exit $rc
