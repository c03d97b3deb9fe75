#!/bin/bash
set -o pipefail
TAG=${1:-sw}
mkdir -p gpurun_out
PIPE_CASES="4,,,,;4,,,,,1;4,,,,,2;4,,,,,4;4,,,,,8;4,,,,,12;4,,,,,3;4,64,,,;4,256,,,;4,,64,,;4,,384,,;4,,,32,;4,,,8,;4,128,96,32,32;lanes" timeout -k 10 400 python -u tools_pipe.py > gpurun_out/pipe_$TAG.log 2>&1 || exit 5
