#!/bin/bash
# GPU parity tests, then a pipe sweep (SWEEP) on the in-tree library
set -o pipefail
TAG=${1:-ts}
mkdir -p gpurun_out
export C3H_REQUIRE_GPU=1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1 || exit 3
PIPE_CASES="${SWEEP:-8,,,,}" timeout -k 10 400 python -u tools_pipe.py 2>&1 | grep -v amdgpu.ids > gpurun_out/tsweep_$TAG.log || exit 6
