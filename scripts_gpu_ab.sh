#!/bin/bash
# GPU parity tests, then A/B of the lane-per-item search bodies (bench + pipe sweep)
set -o pipefail
TAG=${1:-ab}
mkdir -p gpurun_out
export C3H_REQUIRE_GPU=1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1 || exit 3
for LB in 1 0 1 0; do
  C3H_LANE_BODIES=$LB timeout -k 10 300 python bench.py --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/bench_${TAG}_lb$LB.json 2>> gpurun_out/bench_${TAG}.err || exit 4
  echo "LB=$LB $(python -c "import json,sys;d=json.load(open('gpurun_out/bench_${TAG}_lb$LB.json'));print(d['value'],d['ms_per_step'],d['roofline']['frac'])")" >> gpurun_out/ab_$TAG.log
  C3H_LANE_BODIES=$LB PIPE_CASES="${SWEEP:-4,,,,;8,,,,;8,64,,,}" timeout -k 10 300 python -u tools_pipe.py >> gpurun_out/ab_$TAG.log 2>&1 || exit 6
done
