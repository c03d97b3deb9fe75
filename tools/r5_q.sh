#!/bin/bash
# round 5, session q: smoke, GPU suite, the driver's bench command + trace + tick agreement
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $R/gpurun_out/smoke_r5r.txt 2>&1 || exit 7
tools/gpu_round.sh r5r || exit $?
