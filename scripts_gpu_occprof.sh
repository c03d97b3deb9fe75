#!/bin/bash
# occupancy-only run under rocprofv3 kernel trace (isolated kernel durations)
set -o pipefail
TAG=$1
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
C3H_C3_DEBUG=3 LANES_CASES="1,4,,;1,8,," timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/occprof_$TAG -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools_lanes.py > $GRAFT_REPO_ROOT/gpurun_out/occprof_$TAG.log 2>&1 || exit 5
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/bwprof_$TAG -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools_bw.py > $GRAFT_REPO_ROOT/gpurun_out/bw_$TAG.log 2>&1 || exit 6
