#!/bin/bash
# round 5, session k: GPU suite, the driver's bench command, its kernel trace and the tick
# agreement (tools/gpu_round.sh), then the single-frame path's kernel + copy trace
set -o pipefail
R=$GRAFT_REPO_ROOT
tools/gpu_round.sh r5k || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $R/gpurun_out/prof_r5k_single -o run --output-format csv -- \
  python3 $R/tools/single_frame_trace.py 40 > $R/gpurun_out/prof_r5k_single.log 2>&1 || exit 6
