#!/bin/bash
# config-5 A/B: default build vs a variant .so, interleaved (C3 + search stage times)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-c5ab}
V=${2:-mf4}
mkdir -p $O
for i in 1 2; do
  unset C3HLAC_LIB
  timeout -k 10 200 python -u tools/config5.py > $O/default_$i.log 2>&1 || exit 3
  C3HLAC_LIB=$R/mapping-private_amd/lib/variants/$V.so timeout -k 10 200 python -u tools/config5.py > $O/${V}_$i.log 2>&1 || exit 4
done
