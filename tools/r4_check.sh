#!/bin/bash
# Round-4 GPU check: selected GPU test files, then config 5 under rocprofv3 --stats.
# usage: tools/r4_check.sh TAG [pytest files...]; continues past test failures (rc 1) only.
TAG=${1:-r4}
shift
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
export C3H_REQUIRE_GPU=1
timeout -k 10 900 python -u -m pytest "$@" -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  > $R/gpurun_out/gpu_tests_$TAG.log 2>&1
rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/c5_$TAG -o run --output-format csv -- \
  python3 $R/tools/config5.py --fp16 > $R/gpurun_out/c5_$TAG.log 2>&1 || exit $?
exit $rc
