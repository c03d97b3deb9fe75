#!/bin/bash
# Lane / launch-grid sweep: bash scripts_gpu_sweep.sh TAG "lanes,batch,occ,tile;..."
set -o pipefail
mkdir -p gpurun_out
LANES_CASES="$2" timeout -k 10 400 python tools_lanes.py > gpurun_out/sweep_${1}.log 2>&1 || exit 4
