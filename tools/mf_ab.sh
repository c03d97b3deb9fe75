#!/bin/bash
# config-5 C3 time (occupancy pass + dense MFMA body) for the default build and each
# lib/variants/<name>.so, interleaved twice; then a rocprof kernel summary of each.
# usage: tools/mf_ab.sh OUT VARIANT...
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-mfab}; shift
mkdir -p $O
for rep in 1 2; do
  for v in default "$@"; do
    if [ $v = default ]; then unset C3HLAC_LIB; else export C3HLAC_LIB=$R/mapping-private_amd/lib/variants/$v.so; fi
    timeout -k 10 200 python -u tools/config5.py > $O/$v.$rep.log 2>&1 || exit 3
  done
done
unset C3HLAC_LIB
grep -H "config5: subdiv" $O/*.log
cd /tmp && export TMPDIR=/tmp
for v in default "$@"; do
  if [ $v = default ]; then unset C3HLAC_LIB; else export C3HLAC_LIB=$R/mapping-private_amd/lib/variants/$v.so; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$v -o run --output-format csv -- python3 $R/tools/config5.py > $O/prof_$v.log 2>&1 || exit 4
done
