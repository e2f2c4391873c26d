#!/bin/bash
# Run one pytest selection against each experimental library variant (swapping the in-tree
# libhalo_rx.so), stopping at the first crash/timeout. usage: variant_tests.sh "<pytest args>" v1 v2 ...
cd "${GRAFT_REPO_ROOT:-.}"
args=$1; shift
cp halo_amd/lib/libhalo_rx.so /tmp/libhalo_rx_orig.so
for v in "$@"; do
  cp tools/exp/libhalo_rx_$v.so halo_amd/lib/libhalo_rx.so
  timeout -k 10 300 python -u -m pytest $args -q -x --timeout 120 --timeout-method thread > gpurun_out/vt_$v.log 2>&1
  rc=$?
  echo "== $v rc=$rc $(tail -1 gpurun_out/vt_$v.log)"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then break; fi
done
cp /tmp/libhalo_rx_orig.so halo_amd/lib/libhalo_rx.so
