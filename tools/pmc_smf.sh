#!/bin/bash
# PMC passes over the config-5 fp16 stress search (63 models x r = 70): SQ wait / busy / MFMA
# counters and LDS counters, each pass its own rocprofv3 run.  usage: tools/pmc_smf.sh OUT
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-psmf}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
S="python3 $R/tools/config5.py --engine 0 --models 63 --r 70 --fp16"
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS \
  -d $O/sq -o run --output-format csv -- $S > $O/sq.log 2>&1 || exit 4
timeout -s KILL 180 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_WAIT_INST_LDS \
  -d $O/inst -o run --output-format csv -- $S > $O/inst.log 2>&1 || exit 5
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE -d $O/fetch -o run --output-format csv -- $S > $O/fetch.log 2>&1 || exit 6
