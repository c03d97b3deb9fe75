#!/bin/bash
# pipe sweep per library variant (tools/build_variant.sh): VARIANTS="default u4p ..."
set -o pipefail
TAG=${1:-var}
mkdir -p gpurun_out
export C3H_REQUIRE_GPU=1
: > gpurun_out/variants_$TAG.log
for V in ${VARIANTS:-default}; do
  if [ "$V" = default ]; then unset C3HLAC_LIB; else export C3HLAC_LIB=$PWD/mapping-private_amd/lib/variants/$V.so; fi
  echo "== $V" >> gpurun_out/variants_$TAG.log
  PIPE_CASES="${SWEEP:-8,64,,,;8,64,,,,8}" timeout -k 10 300 python -u tools_pipe.py 2>&1 | grep -v amdgpu.ids >> gpurun_out/variants_$TAG.log || exit 6
done
