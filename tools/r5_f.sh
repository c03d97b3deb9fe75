#!/bin/bash
# round 5, session f: voxeliser / f16-row parity subset, then the single-frame voxeliser
# variants (count atomics per block, skeleton without the flush sums, chunk / workgroup
# sizes) interleaved with round 4, and config 5 with f16 rows (16-B row loads)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5f
mkdir -p $O
V=$R/mapping-private_amd/lib/variants
export C3H_REQUIRE_GPU=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_config5_nonperiodic.py tests/test_gpu_shape_fixtures.py \
  -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || exit 1
for rep in 1 2; do
  for v in default nocnt noflush c2k t512 r4; do
    if [ $v = default ]; then unset C3HLAC_LIB; else export C3HLAC_LIB=$V/$v.so; fi
    timeout -k 10 120 python3 tools/vox_bench.py 200 | sed "s/^/{\"v\": \"$v\", \"d\": /; s/$/}/" >> $O/vox1.jsonl 2>> $O/err.log || exit 2
  done
done
unset C3HLAC_LIB
for rep in 1 2; do
  timeout -k 10 180 python3 tools/config5.py --fp16 >> $O/c5_default.log 2>> $O/err.log || exit 3
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof_vox1 -o run --output-format csv -- python3 $R/tools/vox_bench.py 100 > $O/prof_vox1.log 2>&1 || exit 5
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof_c5 -o run --output-format csv -- python3 $R/tools/config5.py --fp16 > $O/prof_c5.log 2>&1 || exit 5
