#!/bin/bash
# A/B library variants on one box by swapping the in-tree library file (the bench loop links it
# by name, so an env override alone would not switch it). usage: ab_variants.sh "<tune args>" v1 v2 ...
cd "${GRAFT_REPO_ROOT:-.}"
args=$1; shift
cp halo_amd/lib/libhalo_rx.so /tmp/libhalo_rx_orig.so
for round in 1 2; do
  for v in "$@"; do
    echo "== $v round $round"
    cp tools/exp/libhalo_rx_$v.so halo_amd/lib/libhalo_rx.so
    timeout -k 10 300 python tools/tune.py $args || { cp /tmp/libhalo_rx_orig.so halo_amd/lib/libhalo_rx.so; exit 1; }
  done
done
cp /tmp/libhalo_rx_orig.so halo_amd/lib/libhalo_rx.so
