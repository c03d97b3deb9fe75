#!/bin/bash
# per-role tick cost: each role alone / in pairs at the bench geometry
set -o pipefail
TAG=${1:-roles}
mkdir -p gpurun_out
export C3H_REQUIRE_GPU=1
PIPE_CASES="${SWEEP:-8,64,,,;8,64,,,,8;8,32,,,,8;8,128,,,,8;8,16,,,,8;8,64,,,,4;8,64,,,,2;8,64,,,,1;8,64,,,,12;8,64,,,,3;8,64,,,,7;8,64,,,,11}" timeout -k 10 400 python -u tools_pipe.py > gpurun_out/roles_$TAG.log 2>&1 || exit 6
