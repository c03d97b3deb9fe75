#!/bin/bash
set -o pipefail
TAG=${1:-tp}
mkdir -p gpurun_out
rm -f gpurun_out/tprof_$TAG.txt
C3H_TICK_PROF=gpurun_out/tprof_$TAG.txt PIPE_CASES="4,,,,;8,,,," timeout -k 10 300 python -u tools_pipe.py > gpurun_out/tpipe_$TAG.log 2>&1 || exit 5
PIPE_CASES="4,,,,;8,,,,;4,64,,,;4,96,,,;4,192,,,;4,,32,,;4,,96,,;4,,,16,;4,,,64,;8,64,,,;8,96,32,,;lanes" timeout -k 10 400 python -u tools_pipe.py > gpurun_out/pipe_$TAG.log 2>&1 || exit 6
