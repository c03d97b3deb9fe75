#!/bin/bash
# round 5, session l: HBM traffic of the final voxelisers (PMC FETCH_SIZE / WRITE_SIZE
# passes, each its own run): batched at 256^3 (tools/pmc_points.sh, overlap off) and the
# single-frame path (tools/vox_bench.py)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5l
mkdir -p $O
export C3HLAC_LIB=$R/mapping-private_amd/lib/variants/noovl.so
tools/pmc_points.sh r5l/pb256 256 256 || exit 2
unset C3HLAC_LIB
cd /tmp && export TMPDIR=/tmp
V="python3 $R/tools/vox_bench.py 100"
for p in "fetch FETCH_SIZE" "write WRITE_SIZE"; do
  set -- $p; n=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" -d $O/vox1_$n -o run --output-format csv -- $V > $O/vox1_$n.log 2>&1 || exit 4
done
