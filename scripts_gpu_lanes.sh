#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export C3H_REQUIRE_GPU=1
timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -m gpu -q -p no:cacheprovider -k "lanes or golden or config3" > gpurun_out/lanes_tests_${1:-r1o}.log 2>&1 || exit 5
timeout -k 10 300 python tools_lanes.py > gpurun_out/lanes_${1:-r1o}.log 2>&1 || exit 4
