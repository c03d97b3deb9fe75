#!/bin/bash
# round-end style GPU session: parity tests, smoke(), bench, rocprof kernel trace + tick check
set -o pipefail
TAG=${1:-fin}
mkdir -p gpurun_out
export C3H_REQUIRE_GPU=1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 240 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1 || exit 3
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || exit 4
timeout -k 10 300 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit 5
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_$TAG -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3840 --warmup 64 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/prof_$TAG.log 2>&1 || exit 6
cd $GRAFT_REPO_ROOT
python tools_tick_trace.py gpurun_out/prof_$TAG/run_kernel_trace.csv 64 3840 64 gpurun_out/bench_$TAG.json > gpurun_out/tick_trace_$TAG.json
