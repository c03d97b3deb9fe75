#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python tools_lanes.py 4 > gpurun_out/lanes_q4_${1:-r1x}.log 2>&1 || exit 4
timeout -k 10 300 python tools_lanes.py 8 > gpurun_out/lanes_q8_${1:-r1x}.log 2>&1 || exit 5
timeout -k 10 200 python tools_phase_probe.py gpurun_out/probe_${1:-r1x}.txt > gpurun_out/probe_${1:-r1x}.log 2>&1 || exit 6
