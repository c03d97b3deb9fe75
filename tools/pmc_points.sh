#!/bin/bash
# Batched voxeliser / points-in pipeline evidence: kernel trace + stats of tools/points_bench.py,
# then PMC passes (each its own rocprofv3 run).  usage: tools/pmc_points.sh OUT [grid] [frames]
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-pp}
G=${2:-256}
N=${3:-256}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
V="python3 $R/tools/points_bench.py $G $N 32"
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- $V > $O/trace.log 2>&1 || exit 3
for p in "fetch FETCH_SIZE" "write WRITE_SIZE" "sq SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT"; do
  set -- $p; n=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" -d $O/$n -o run --output-format csv -- $V > $O/$n.log 2>&1 || exit 4
done
