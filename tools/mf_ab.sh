#!/bin/bash
# dense C3 MFMA kernel diagnostics: config-5 C3 time for the default build and each
# lib/variants/<name>.so given (C3H_MF_EXP builds: 1 no K steps, 2 no plane conversion,
# 4 no bin epilogue)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-mfab}; shift
mkdir -p $O
timeout -k 10 200 python -u tools/config5.py > $O/base.log 2>&1 || exit 3
for v in "$@"; do
  C3HLAC_LIB=$R/mapping-private_amd/lib/variants/$v.so timeout -k 10 200 python -u tools/config5.py > $O/$v.log 2>&1 || exit 4
done
grep -H "config5: subdiv" $O/*.log
