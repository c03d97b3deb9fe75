#!/bin/bash
# config 5 with fp16 search precision: default build vs lib/variants/<name>.so, interleaved
# twice (per-rep stage times printed by tools/config5.py).  usage: tools/c5_fp16_ab.sh OUT VARIANT...
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-c5f}; shift
mkdir -p $O
for rep in 1 2; do
  for v in default "$@"; do
    if [ $v = default ]; then unset C3HLAC_LIB; else export C3HLAC_LIB=$R/mapping-private_amd/lib/variants/$v.so; fi
    timeout -k 10 200 python -u tools/config5.py --fp16 > $O/$v.$rep.log 2>&1 || exit 3
  done
done
grep -H "^rep [123]" $O/*.log
