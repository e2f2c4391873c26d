#!/bin/bash
# A/B of non-temporal loads/stores: interleaved rounds, one box (tools only)
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
for round in 1 2; do
  for v in base ntl nts ntls; do
    echo "== $v round $round"
    HALO_RX_LIB=$PWD/tools/exp/libhalo_rx_$v.so timeout -k 10 120 python bench.py --no-cpu --no-secondary --steps 200 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['kernel_ms'])" || exit 1
  done
done
