#!/bin/bash
# A/B library variants on one box by swapping the in-tree library file: tools/libhalo_bench.so
# links libhalo_rx.so through its rpath, so an HALO_RX_LIB override alone would leave the timed
# loop on the in-tree build. usage: ab_variants.sh "<command>" v1 v2 ...   (tools only)
cd "${GRAFT_REPO_ROOT:-.}"
cmd=$1; shift
cp halo_amd/lib/libhalo_rx.so /tmp/libhalo_rx_orig.so
for round in 1 2; do
  for v in "$@"; do
    echo "== $v round $round"
    cp tools/exp/libhalo_rx_$v.so halo_amd/lib/libhalo_rx.so
    timeout -k 10 300 bash -c "$cmd" || { cp /tmp/libhalo_rx_orig.so halo_amd/lib/libhalo_rx.so; exit 1; }
  done
done
cp /tmp/libhalo_rx_orig.so halo_amd/lib/libhalo_rx.so
