#!/bin/bash
# PMC passes (each its own rocprofv3 run; --pmc never combined with trace domains)
set -o pipefail
TAG=${1:-r1}
mkdir -p gpurun_out/pmc_$TAG
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
run() {  # name, counters...
  local name=$1; shift
  timeout -k 10 240 rocprofv3 --pmc "$@" -d $R/gpurun_out/pmc_$TAG/$name -o run --output-format csv -- python3 $R/bench.py --steps 960 --warmup 64 --no-cpu-baseline > $R/gpurun_out/pmc_$TAG/$name.log 2>&1
}
run fetch FETCH_SIZE && run write WRITE_SIZE && run sq SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY && run inst SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT
rc=$?
# frames through the pipeline: bench's allocation prime (4 x BATCH) + warmup + steps
cd $R && python3 tools_pmc_summary.py gpurun_out/pmc_$TAG gpurun_out/pmc_$TAG/summary.json 64 $((4 * 64 + 64 + 960)) > /dev/null
exit $rc
