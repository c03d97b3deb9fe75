#!/bin/bash
# round 5, session u: batched accumulate with the next round's point loads issued before
# this round's work (C3H_VB_PIPE=1), against the product, with and without the tick overlap
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5u
mkdir -p $O
V=$R/mapping-private_amd/lib/variants
for rep in 1 2 3; do
  for v in noovl pipe default pipeovl; do
    if [ $v = default ]; then unset C3HLAC_LIB; else export C3HLAC_LIB=$V/$v.so; fi
    timeout -k 10 120 python3 tools/points_bench.py 128 512 32 2>> $O/err.log | sed "s/^/{\"v\": \"$v\", \"d\": /; s/$/}/" >> $O/pb128.jsonl || exit 3
  done
done
