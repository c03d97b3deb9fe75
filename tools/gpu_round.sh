#!/bin/bash
# One GPU session: GPU tests, the driver's bench command, the same command under
# rocprofv3 --kernel-trace --stats, and the tick trace checked against the bench line.
# usage: tools/gpu_round.sh TAG [tests|notests]
set -o pipefail
TAG=${1:-r2}
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
export C3H_REQUIRE_GPU=1
if [ "${2:-tests}" = tests ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu ${PYTEST_X--x} -v --timeout 300 --timeout-method thread -p no:cacheprovider \
    > $R/gpurun_out/gpu_tests_$TAG.log 2>&1 || exit $?
fi
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $R/gpurun_out/bench_$TAG.json 2> $R/gpurun_out/bench_$TAG.err || exit 3
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$TAG -o run --output-format csv -- \
  python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $R/gpurun_out/prof_$TAG.log 2>&1 || exit 5
cd $R
python tools/tick_trace.py gpurun_out/prof_$TAG/run_kernel_trace.csv 5 20 gpurun_out/bench_$TAG.json > gpurun_out/tick_trace_$TAG.json
