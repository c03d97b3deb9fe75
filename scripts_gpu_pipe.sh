#!/bin/bash
# pipeline session: GPU parity tests, tick role sweep, bench
set -o pipefail
TAG=${1:-pipe}
mkdir -p gpurun_out
export C3H_REQUIRE_GPU=1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1 || exit 3
timeout -k 10 300 python -u tools_pipe.py > gpurun_out/pipe_$TAG.log 2>&1 || exit 5
timeout -k 10 300 python bench.py --steps 200 --warmup 20 --cpu-seconds 3 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit 6
