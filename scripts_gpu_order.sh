#!/bin/bash
# tick role dispatch order: pipe sweep + per-tick role profile for two orders
set -o pipefail
TAG=${1:-ord}
mkdir -p gpurun_out
export C3H_REQUIRE_GPU=1
PIPE_CASES="${SWEEP:-8,64,,,;8,64,,,,,3210;8,64,,,,,3120;8,64,,,,,1320;8,64,,,,,3201;4,,,,,,3210;8,32,,,,,3210;8,96,,,,,3210}" timeout -k 10 400 python -u tools_pipe.py > gpurun_out/order_$TAG.log 2>&1 || exit 6
rm -f gpurun_out/tprof_${TAG}_*.txt
C3H_TICK_PROF=gpurun_out/tprof_${TAG}_a.txt PIPE_CASES="8,64,,," timeout -k 10 300 python -u tools_pipe.py >> gpurun_out/order_$TAG.log 2>&1 || exit 5
C3H_TICK_PROF=gpurun_out/tprof_${TAG}_b.txt PIPE_CASES="8,64,,,,,3210" timeout -k 10 300 python -u tools_pipe.py >> gpurun_out/order_$TAG.log 2>&1 || exit 5
