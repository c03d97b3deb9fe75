#!/bin/bash
# PMC passes over the driver's bench command, each its own rocprofv3 run (--pmc is never
# combined with trace domains), then the per-frame / per-tick HBM traffic summary.
# usage: tools/pmc.sh TAG
set -o pipefail
TAG=${1:-r2}
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/pmc_$TAG
cd /tmp && export TMPDIR=/tmp
W=5; K=20; B=64
run() {  # name, counters...
  local name=$1; shift
  timeout -s KILL 240 rocprofv3 --pmc "$@" -d $R/gpurun_out/pmc_$TAG/$name -o run --output-format csv -- \
    python3 $R/bench.py --steps $K --warmup $W --no-cpu-baseline --point-frames 0 --single-frames 0 > $R/gpurun_out/pmc_$TAG/$name.log 2>&1
}
run fetch FETCH_SIZE && run write WRITE_SIZE && run sq SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY && run inst SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT
rc=$?
# frames through the pipeline: the allocation prime (4 x B) + warmup + steps (+ the lanes breakdown pass: no tick)
cd $R && python3 tools/pmc_summary.py gpurun_out/pmc_$TAG gpurun_out/pmc_$TAG/summary.json $B $((4 * B + (W + K) * B)) > /dev/null
exit $rc
