#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python tools_lanes.py > gpurun_out/lanes_${1:-r1ab}.log 2>&1 || exit 4
