#!/bin/bash
# quick loop: GPU tests, occupancy-only (real and empty frames) + default lane sweeps
set -o pipefail
TAG=$1
mkdir -p gpurun_out
export C3H_REQUIRE_GPU=1
timeout -k 10 600 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/gpu_tests_$TAG.log 2>&1 || exit 3
C3H_C3_DEBUG=3 LANES_CASES="1,4,,;1,8,,;1,8,128,;1,8,512," timeout -k 10 300 python tools_lanes.py > gpurun_out/occ_$TAG.log 2>&1 || exit 5
LANES_ZERO=1 C3H_C3_DEBUG=3 LANES_CASES="1,8,,;1,8,128," timeout -k 10 300 python tools_lanes.py > gpurun_out/occz_$TAG.log 2>&1 || exit 6
timeout -k 10 300 python tools_lanes.py > gpurun_out/lanes_$TAG.log 2>&1 || exit 7
