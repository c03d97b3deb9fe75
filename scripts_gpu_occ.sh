#!/bin/bash
# occupancy-pass diagnostics: HBM reference rate + occupancy-only sweeps (tile kernel skipped)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 python tools_bw.py > gpurun_out/bw_${1}.log 2>&1 || exit 4
C3H_C3_DEBUG=3 LANES_CASES="${2:-1,1,,;1,4,,;1,8,,;1,4,512,;1,4,1024,;1,8,128,}" timeout -k 10 300 python tools_lanes.py > gpurun_out/occ_${1}.log 2>&1 || exit 5
LANES_ZERO=1 C3H_C3_DEBUG=3 LANES_CASES="1,4,,;1,8,,;1,8,128,;1,8,512," timeout -k 10 300 python tools_lanes.py > gpurun_out/occz_${1}.log 2>&1 || exit 6
