#!/bin/bash
# diagnostics: SQ counter passes over tools/config5.py (one rocprofv3 run per pass, --pmc
# never combined with trace domains); per-kernel sums in gpurun_out/pmc_c5_TAG/*.txt
set -o pipefail
TAG=${1:-c5}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/pmc_c5_$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
run() {  # name, counters...
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" -d $O/$name -o run --output-format csv -- \
    python3 $R/tools/config5.py $C5ARGS > $O/$name.log 2>&1
}
run a SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES && \
run b SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_MFMA
rc=$?
cd $R && python3 - "$O" <<'PY'
import csv, glob, sys, collections
o = sys.argv[1]
for f in sorted(glob.glob(o + "/*/**/*counter_collection.csv", recursive=True)):
    acc = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"][:60]
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
    with open(f.split("/")[-4 if False else 0] if False else o + "/" + f.split(o + "/")[1].split("/")[0] + ".txt", "w") as w:
        for k, d in acc.items():
            w.write(k + "\n")
            for c, v in sorted(d.items()):
                w.write("   %-28s %.4g\n" % (c, v))
PY
exit $rc
