#!/bin/bash
# round 5, session j: where the config-5 MFMA body's time goes (diagnostics builds without
# the K steps / the layer conversion / the bin epilogue), interleaved
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5j
mkdir -p $O
V=$R/mapping-private_amd/lib/variants
for rep in 1 2; do
  for v in default mfx1 mfx2 mfx4 mfx6; do
    if [ $v = default ]; then unset C3HLAC_LIB; else export C3HLAC_LIB=$V/$v.so; fi
    echo "== $v" >> $O/c5.log
    timeout -k 10 180 python3 tools/config5.py --fp16 >> $O/c5.log 2>> $O/err.log || exit 2
  done
done
