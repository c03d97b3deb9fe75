#!/bin/bash
# role-size sweep at 32 frames per tick
set -o pipefail
TAG=${1:-s3}
mkdir -p gpurun_out
: > gpurun_out/sweep3_$TAG.log
export PIPE_FRAMES=960
for Z in 8 2; do
  echo "== C3H_TICK_ZERO=$Z" >> gpurun_out/sweep3_$TAG.log
  C3H_TICK_ZERO=$Z PIPE_CASES="${SWEEP:-32,,,,;32,,24,,;32,,32,,;32,,16,,;32,,,8,;32,,,12,;32,,,,8;32,,,,16;32,,24,8,8}" timeout -k 10 300 python -u tools_pipe.py 2>&1 | grep -v amdgpu.ids >> gpurun_out/sweep3_$TAG.log || exit 6
done
