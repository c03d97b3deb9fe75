#!/bin/bash
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r5d
for v in diag diag_rmw diag_ald; do
  C3HLAC_LIB=$R/mapping-private_amd/lib/variants/$v.so timeout -k 10 300 python3 tools/vox_dirty.py > $R/gpurun_out/r5d/dirty_$v.jsonl 2> $R/gpurun_out/r5d/dirty_$v.err || exit 1
done
