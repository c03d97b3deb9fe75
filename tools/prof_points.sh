#!/bin/bash
# kernel trace + stats of tools/points_bench.py: usage tools/prof_points.sh OUT [grid] [frames] [lib]
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-ppt}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
[ -n "$4" ] && export C3HLAC_LIB=$R/$4
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 $R/tools/points_bench.py ${2:-256} ${3:-256} 32 > $O/trace.log 2>&1
