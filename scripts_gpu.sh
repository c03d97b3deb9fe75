#!/bin/bash
# round-1 GPU session: tests, bench, rocprof kernel trace
set -o pipefail
mkdir -p gpurun_out
export C3H_REQUIRE_GPU=1
timeout -k 10 600 python -m pytest tests -m gpu -q -p no:cacheprovider > gpurun_out/gpu_tests_r1i.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/gpu_tests_r1i.log
[ $rc -ge 124 ] && exit $rc
timeout -k 10 200 python tools_c3_phases.py > gpurun_out/phases_r1i.log 2>&1 || exit 4
timeout -k 10 300 python bench.py --steps 200 --warmup 20 --cpu-seconds 5 > gpurun_out/bench_r1i.json 2> gpurun_out/bench_r1i.err || exit 3
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_r1i -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 100 --warmup 10 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/prof_r1i.log 2>&1
echo "rocprof rc=$?" >> $GRAFT_REPO_ROOT/gpurun_out/prof_r1i.log
