#!/bin/bash
# A/B of non-temporal loads/stores on the headline workload (tools only). Build the variants with
#   tools/exp/build_variant.sh base; tools/exp/build_variant.sh ntl -DHALO_RX_NT_LOADS=1; ...
# (The first version of this script switched libraries with HALO_RX_LIB, which does not reach the
# native timed loop: its results compared the in-tree build with itself and were discarded.)
cd "${GRAFT_REPO_ROOT:-.}"
bash tools/exp/ab_variants.sh "python bench.py --no-cpu --no-secondary --steps 200 2>/dev/null | python -c \"import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['kernel_ms'])\"" base ntl nts ntls
