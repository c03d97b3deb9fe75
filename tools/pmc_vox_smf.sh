#!/bin/bash
# Voxeliser and matrix-core projection evidence: kernel trace + stats, then PMC passes
# (each its own rocprofv3 run: FETCH_SIZE, WRITE_SIZE, SQ wait/busy/MFMA counters).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-pvs}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
V="python3 $R/tools/vox_bench.py 200"
S="python3 $R/tools/config5.py --engine 0 --models 63 --r 70"
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/vox_trace -o run --output-format csv -- $V > $O/vox_trace.log 2>&1 || exit 3
for p in "fetch FETCH_SIZE" "write WRITE_SIZE" "sq SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT"; do
  set -- $p; n=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" -d $O/vox_$n -o run --output-format csv -- $V > $O/vox_$n.log 2>&1 || exit 4
done
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS \
  -d $O/smf_sq -o run --output-format csv -- $S > $O/smf_sq.log 2>&1 || exit 5
