#!/bin/bash
# batched voxeliser A/B: points_bench.py (256^3 and 128^3) on the default build and variants
# (interleaved), then the rocprof kernel stats of each.  usage: tools/vb_ab.sh OUT VARIANT...
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-vbab}
shift
mkdir -p $O
for rep in 1 2; do
  for v in default "$@"; do
    if [ $v = default ]; then unset C3HLAC_LIB; else export C3HLAC_LIB=$R/mapping-private_amd/lib/variants/$v.so; fi
    timeout -k 10 120 python3 tools/points_bench.py 256 256 32 >> $O/pb256_$v.jsonl 2>> $O/err.log || exit 3
    timeout -k 10 120 python3 tools/points_bench.py 128 256 32 >> $O/pb128_$v.jsonl 2>> $O/err.log || exit 3
  done
done
unset C3HLAC_LIB
for v in default "$@"; do
  L=""; [ $v != default ] && L=mapping-private_amd/lib/variants/$v.so
  tools/prof_points.sh $(basename $O)/prof_$v 256 256 $L || exit 4
done
