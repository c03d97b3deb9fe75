#!/bin/bash
# Round-4 single-frame voxeliser check: GPU tests given as arguments, c3h_voxelize rate
# (tools/vox_bench.py, 3 runs) and its kernel trace.  usage: tools/r4_vox.sh TAG [pytest files...]
set -o pipefail
TAG=${1:-r4v}; shift
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/vox_$TAG
mkdir -p $O
export C3H_REQUIRE_GPU=1
timeout -k 10 900 python -u -m pytest "$@" -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  > $O/tests.log 2>&1
rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for i in 1 2 3; do
  timeout -k 10 120 python -u tools/vox_bench.py 200 >> $O/vox.jsonl 2>> $O/vox.err || exit 3
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- \
  python3 $R/tools/vox_bench.py 200 > $O/trace.log 2>&1 || exit 4
exit $rc
