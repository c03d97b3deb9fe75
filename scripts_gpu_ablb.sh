#!/bin/bash
# A/B of the tick kernel at 5 waves per SIMD: bench alternating the default library and lib/variants/lb5.so
set -o pipefail
TAG=${1:-abrot}
mkdir -p gpurun_out
export C3H_REQUIRE_GPU=1
: > gpurun_out/ab_$TAG.log
for V in default lb5 default lb5; do
  if [ "$V" = default ]; then unset C3HLAC_LIB; else export C3HLAC_LIB=$PWD/mapping-private_amd/lib/variants/$V.so; fi
  timeout -k 10 300 python bench.py --steps 960 --warmup 64 --no-cpu-baseline > gpurun_out/bench_${TAG}_$V.json 2>> gpurun_out/bench_$TAG.err || exit 4
  echo "$V $(python -c "import json;d=json.load(open('gpurun_out/bench_${TAG}_$V.json'));print(round(d['value']),d['ms_per_step'],round(d['roofline']['frac'],4))")" >> gpurun_out/ab_$TAG.log
done
