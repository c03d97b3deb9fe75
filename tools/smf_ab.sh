#!/bin/bash
# matrix-core projection A/B: default build vs a variant .so on config 5 (10 x r=20 and the
# 63 x r=70 stress case), interleaved, then its parity tests on the default build.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-sab}
V=${2:-t1}
mkdir -p $O
export C3H_REQUIRE_GPU=1
for i in 1 2; do
  for lib in default $V; do
    if [ $lib = default ]; then unset C3HLAC_LIB; else export C3HLAC_LIB=$R/mapping-private_amd/lib/variants/$V.so; fi
    timeout -k 10 200 python -u tools/config5.py --engine 0 --models 63 --r 70 > $O/stress_${lib}_$i.log 2>&1 || exit 3
    timeout -k 10 200 python -u tools/config5.py --engine 2 > $O/m10_${lib}_$i.log 2>&1 || exit 4
  done
done
unset C3HLAC_LIB
timeout -k 10 600 python -u -m pytest tests/test_gpu_score_mfma.py -x -v --timeout 300 --timeout-method thread \
  -p no:cacheprovider > $O/tests.log 2>&1 || exit 5
