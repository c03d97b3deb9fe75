#!/bin/bash
# A/B of frames per tick: bench alternating C3H_BENCH_BATCH=32 and 64 (default 3840 frames)
set -o pipefail
TAG=${1:-abbatch}
mkdir -p gpurun_out
export C3H_REQUIRE_GPU=1
: > gpurun_out/ab_$TAG.log
for B in ${BATCHES:-32 64 32 64}; do
  C3H_BENCH_BATCH=$B timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_${TAG}_$B.json 2>> gpurun_out/bench_$TAG.err || exit 4
  echo "batch=$B $(python -c "import json;d=json.load(open('gpurun_out/bench_${TAG}_$B.json'));print(round(d['value']),d['ms_per_step'],round(d['roofline']['frac'],4),d['roofline']['launches'])")" >> gpurun_out/ab_$TAG.log
done
