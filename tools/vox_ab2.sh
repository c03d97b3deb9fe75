#!/bin/bash
# single-frame voxeliser A/B: default build and each lib/variants/<name>.so, interleaved
# (3 rounds of tools/vox_bench.py 200).  usage: tools/vox_ab2.sh OUT VARIANT...
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-vab}; shift
mkdir -p $O
export C3H_REQUIRE_GPU=1
for rep in 1 2 3; do
  for v in default "$@"; do
    if [ $v = default ]; then unset C3HLAC_LIB; else export C3HLAC_LIB=$R/mapping-private_amd/lib/variants/$v.so; fi
    timeout -k 10 120 python -u tools/vox_bench.py 200 >> $O/vox_$v.jsonl 2>> $O/vox.err || exit 3
  done
done
