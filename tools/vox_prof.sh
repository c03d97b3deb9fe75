#!/bin/bash
# kernel traces of tools/vox_bench.py for the default build and each variant.
# usage: tools/vox_prof.sh OUT VARIANT...
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-vprof}; shift
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for v in default "$@"; do
  if [ $v = default ]; then unset C3HLAC_LIB; else export C3HLAC_LIB=$R/mapping-private_amd/lib/variants/$v.so; fi
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/$v -o run --output-format csv -- \
    python3 $R/tools/vox_bench.py 200 > $O/$v.log 2>&1 || exit 3
done
