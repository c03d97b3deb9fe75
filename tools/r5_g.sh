#!/bin/bash
# round 5, session g: global atomic throughput (device scope vs an XCD-local copy), then the
# batched voxeliser skeleton (no flush) and workgroup-scope timing variants (timing only)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5g
mkdir -p $O
V=$R/mapping-private_amd/lib/variants
timeout -k 10 60 tools/atomic_bench > $O/atomic_bench.json 2> $O/atomic_bench.err || exit 1
for rep in 1 2; do
  for v in noovl vbskel r4_noovl; do
    export C3HLAC_LIB=$V/$v.so
    timeout -k 10 120 python3 tools/points_bench.py 128 512 32 | sed "s/^/{\"v\": \"$v\", \"d\": /; s/$/}/" >> $O/pb128.jsonl 2>> $O/err.log || exit 3
  done
done
