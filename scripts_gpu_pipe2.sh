#!/bin/bash
# GPU parity tests, then tick-role profile and a role-size sweep
set -o pipefail
TAG=${1:-pp}
mkdir -p gpurun_out
export C3H_REQUIRE_GPU=1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1 || exit 3
rm -f gpurun_out/tprof_$TAG.txt gpurun_out/probe_$TAG.txt
C3H_TICK_PROF=gpurun_out/tprof_$TAG.txt PIPE_CASES="4,,,,;8,,,," timeout -k 10 300 python -u tools_pipe.py > gpurun_out/tpipe_$TAG.log 2>&1 || exit 5
timeout -k 10 200 python tools_phase_probe.py gpurun_out/probe_$TAG.txt > gpurun_out/probe_$TAG.log 2>&1 || exit 4
PIPE_CASES="${SWEEP:-4,,,,;8,,,,;8,64,,,;8,48,,,;8,64,32,,;8,64,96,,;8,64,,12,;8,64,,48,;lanes}" timeout -k 10 400 python -u tools_pipe.py > gpurun_out/pipe_$TAG.log 2>&1 || exit 6
