#!/bin/bash
# GPU parity tests, a tick sweep at 32 frames per tick and a role timeline
set -o pipefail
TAG=${1:-rot}
mkdir -p gpurun_out
export C3H_REQUIRE_GPU=1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 240 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1 || exit 3
PIPE_FRAMES=960 VARIANTS=default SWEEP="${SWEEP:-32,,,,;32,,,,,8;32,,,,}" bash scripts_gpu_variants.sh $TAG || exit 4
PIPE_FRAMES=480 SWEEP="32,,,," bash scripts_gpu_tprof2.sh tp_$TAG
