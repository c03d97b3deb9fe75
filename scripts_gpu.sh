#!/bin/bash
# round-1 GPU session: tests, phase probes, bench, rocprof kernel trace
set -o pipefail
TAG=${1:-r1k}
mkdir -p gpurun_out
export C3H_REQUIRE_GPU=1
timeout -k 10 600 python -m pytest tests -m gpu -q -p no:cacheprovider > gpurun_out/gpu_tests_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/gpu_tests_$TAG.log
[ $rc -ge 124 ] && exit $rc
timeout -k 10 200 python tools_phase_probe.py gpurun_out/probe_$TAG.txt > gpurun_out/probe_$TAG.log 2>&1 || exit 4
timeout -k 10 300 python tools_lanes.py > gpurun_out/lanes_$TAG.log 2>&1 || exit 6
timeout -k 10 300 python bench.py --cpu-seconds 5 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit 3
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_$TAG -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 960 --warmup 64 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/prof_$TAG.log 2>&1
echo "rocprof rc=$?" >> $GRAFT_REPO_ROOT/gpurun_out/prof_$TAG.log
cd $GRAFT_REPO_ROOT
python tools_tick_trace.py gpurun_out/prof_$TAG/run_kernel_trace.csv 64 960 32 gpurun_out/bench_$TAG.json > gpurun_out/tick_trace_$TAG.json
