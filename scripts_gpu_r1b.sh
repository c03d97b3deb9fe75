#!/bin/bash
# round-1 GPU session b: tests, bench, rocprof kernel trace
set -o pipefail
mkdir -p gpurun_out
export C3H_REQUIRE_GPU=1
timeout -k 10 600 python -m pytest tests -m gpu -q -p no:cacheprovider > gpurun_out/gpu_tests_r1b.log 2>&1
echo "pytest rc=$?" >> gpurun_out/gpu_tests_r1b.log
timeout -k 10 300 python bench.py --steps 200 --warmup 20 --cpu-seconds 5 > gpurun_out/bench_r1b.json 2> gpurun_out/bench_r1b.err || exit 3
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_r1b -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 100 --warmup 10 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/prof_r1b.log 2>&1
echo "rocprof rc=$?" >> $GRAFT_REPO_ROOT/gpurun_out/prof_r1b.log
