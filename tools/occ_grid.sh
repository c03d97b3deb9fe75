#!/bin/bash
# config-5 C3 time vs the occupancy pass's workgroup count (C3H_OCC_GRID, diagnostics build)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-occg}; shift
mkdir -p $O
for g in "$@"; do
  C3H_OCC_GRID=$g C3HLAC_LIB=$R/mapping-private_amd/lib/variants/diag.so timeout -k 10 200 python -u tools/config5.py > $O/g$g.log 2>&1 || exit 4
done
grep -H "config5: subdiv" $O/*.log
