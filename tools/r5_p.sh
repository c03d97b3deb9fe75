#!/bin/bash
# round 5, session p: the points-in exact pass spread over 16 blocks per frame (LDS sorts)
# and the dot4 fixup -- points / real views / production / parity suites, then the bench
# line's points-in pass against the previous build (lib/variants/prefix.so), interleaved
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5p
mkdir -p $O
V=$R/mapping-private_amd/lib/variants
export C3H_REQUIRE_GPU=1
timeout -k 10 700 python -u -m pytest tests/test_gpu_points.py tests/test_gpu_real_views.py tests/test_gpu_production.py \
  tests/test_gpu_parity.py tests/test_gpu_shape_fixtures.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || exit 1
for rep in 1 2; do
  for v in default prefix; do
    if [ $v = default ]; then unset C3HLAC_LIB; else export C3HLAC_LIB=$V/$v.so; fi
    timeout -k 10 300 python3 bench.py --steps 10 --warmup 4 --no-cpu-baseline --single-frames 0 \
      2>> $O/err.log | sed "s/^/{\"v\": \"$v\", \"d\": /; s/$/}/" >> $O/bench.jsonl || exit 2
  done
done
unset C3HLAC_LIB
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- \
  python3 $R/bench.py --steps 10 --warmup 4 --no-cpu-baseline --single-frames 0 > $O/prof.log 2>&1 || exit 5
