#!/bin/bash
# per-tick role timelines (C3H_TICK_PROF) at the default configuration
set -o pipefail
TAG=${1:-tp}
mkdir -p gpurun_out
rm -f gpurun_out/tprof_$TAG.txt
C3H_TICK_PROF=gpurun_out/tprof_$TAG.txt PIPE_CASES="${SWEEP:-8,,,,}" timeout -k 10 300 python -u tools_pipe.py > gpurun_out/tpipe_$TAG.log 2>&1
