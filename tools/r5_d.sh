#!/bin/bash
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r5d
C3HLAC_LIB=$R/mapping-private_amd/lib/variants/diag.so timeout -k 10 300 python3 tools/vox_dirty.py > $R/gpurun_out/r5d/dirty.jsonl 2> $R/gpurun_out/r5d/dirty.err
