#!/bin/bash
# round 5, session n: the points-in off-cell fixup as a dot4 recompute -- the points / real
# views / parity suites, then points_bench against the previous build (lib/variants/prefix*)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5n
mkdir -p $O
V=$R/mapping-private_amd/lib/variants
export C3H_REQUIRE_GPU=1
timeout -k 10 700 python -u -m pytest tests/test_gpu_points.py tests/test_gpu_real_views.py tests/test_gpu_production.py \
  -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || exit 1
for rep in 1 2; do
  for v in default prefix noovl prefix_noovl; do
    if [ $v = default ]; then unset C3HLAC_LIB; else export C3HLAC_LIB=$V/$v.so; fi
    timeout -k 10 120 python3 tools/points_bench.py 128 512 32 | sed "s/^/{\"v\": \"$v\", \"d\": /; s/$/}/" >> $O/pb128.jsonl 2>> $O/err.log || exit 3
    timeout -k 10 120 python3 tools/points_bench.py 256 256 32 | sed "s/^/{\"v\": \"$v\", \"d\": /; s/$/}/" >> $O/pb256.jsonl 2>> $O/err.log || exit 3
  done
done
unset C3HLAC_LIB
tools/prof_points.sh r5n/prof128 128 512 || exit 4
