#!/bin/bash
# round 5, session v: batched accumulate skeletons -- no global flush (DIAG 1), and no LDS
# insert either (DIAG 2: loads, cell arithmetic and the DPP run merge only); timing only
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5v
mkdir -p $O
V=$R/mapping-private_amd/lib/variants
for rep in 1 2 3; do
  for v in noovl vbskel vbskel2; do
    export C3HLAC_LIB=$V/$v.so
    timeout -k 10 120 python3 tools/points_bench.py 128 512 32 2>> $O/err.log | sed "s/^/{\"v\": \"$v\", \"d\": /; s/$/}/" >> $O/pb128.jsonl || exit 3
  done
done
