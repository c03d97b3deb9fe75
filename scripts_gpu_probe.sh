#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python tools_phase_probe.py gpurun_out/probe_${1:-r1y}.txt > gpurun_out/probe_${1:-r1y}.log 2>&1 || exit 4
