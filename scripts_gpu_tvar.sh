#!/bin/bash
# GPU parity tests on the in-tree library, then a pipe sweep per library variant
set -o pipefail
TAG=${1:-tv}
mkdir -p gpurun_out
export C3H_REQUIRE_GPU=1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1 || exit 3
bash scripts_gpu_variants.sh $TAG
