#!/bin/bash
# round 5, session i: first-touch flush (two adds per pair) in both voxelisers -- bad-voxel
# check, GPU suite, single-frame and batched rates against round 4, kernel trace
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5i
mkdir -p $O
V=$R/mapping-private_amd/lib/variants
timeout -k 10 200 python3 tools/vox_bad.py > $O/vox_bad.jsonl 2> $O/vox_bad.err || exit 1
export C3H_REQUIRE_GPU=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  -s > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc" >> $O/rc.txt; [ $rc -ne 0 ] && exit 1
for rep in 1 2; do
  for v in default r4; do
    if [ $v = default ]; then unset C3HLAC_LIB; else export C3HLAC_LIB=$V/$v.so; fi
    timeout -k 10 120 python3 tools/vox_bench.py 200 | sed "s/^/{\"v\": \"$v\", \"d\": /; s/$/}/" >> $O/vox1.jsonl 2>> $O/err.log || exit 2
  done
  for v in noovl r4_noovl default; do
    if [ $v = default ]; then unset C3HLAC_LIB; else export C3HLAC_LIB=$V/$v.so; fi
    timeout -k 10 120 python3 tools/points_bench.py 128 512 32 | sed "s/^/{\"v\": \"$v\", \"d\": /; s/$/}/" >> $O/pb128.jsonl 2>> $O/err.log || exit 3
    timeout -k 10 120 python3 tools/points_bench.py 256 256 32 | sed "s/^/{\"v\": \"$v\", \"d\": /; s/$/}/" >> $O/pb256.jsonl 2>> $O/err.log || exit 3
  done
done
unset C3HLAC_LIB
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof_vox1 -o run --output-format csv -- python3 $R/tools/vox_bench.py 100 > $O/prof_vox1.log 2>&1 || exit 5
