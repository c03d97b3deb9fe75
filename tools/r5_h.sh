#!/bin/bash
# round 5, session h: brick-partitioned single-frame voxeliser -- bad-voxel check, the GPU
# suite, the single-frame rate against round 4, and a kernel trace
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5h
mkdir -p $O
V=$R/mapping-private_amd/lib/variants
timeout -k 10 200 python3 tools/vox_bad.py > $O/vox_bad.jsonl 2> $O/vox_bad.err || exit 1
export C3H_REQUIRE_GPU=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  -s > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc" >> $O/rc.txt; [ $rc -ge 124 ] && exit $rc
for rep in 1 2; do
  for v in default r4; do
    if [ $v = default ]; then unset C3HLAC_LIB; else export C3HLAC_LIB=$V/$v.so; fi
    timeout -k 10 120 python3 tools/vox_bench.py 200 | sed "s/^/{\"v\": \"$v\", \"d\": /; s/$/}/" >> $O/vox1.jsonl 2>> $O/err.log || exit 2
  done
done
unset C3HLAC_LIB
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof_vox1 -o run --output-format csv -- python3 $R/tools/vox_bench.py 100 > $O/prof_vox1.log 2>&1 || exit 5
