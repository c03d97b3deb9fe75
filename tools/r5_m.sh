#!/bin/bash
# round 5, session m: config-5 conversion split into (item, colour) tasks, and 2 vs 3 waves
# per SIMD (no spills at 2): dense-path tests on the product build, then interleaved timing
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5m
mkdir -p $O
V=$R/mapping-private_amd/lib/variants
export C3H_REQUIRE_GPU=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_config5_nonperiodic.py tests/test_gpu_slab.py tests/test_gpu_parity.py \
  -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || exit 1
for rep in 1 2; do
  for v in default nosplit minb2 minb2ns; do
    if [ $v = default ]; then unset C3HLAC_LIB; else export C3HLAC_LIB=$V/$v.so; fi
    echo "== $v" >> $O/c5.log
    timeout -k 10 180 python3 tools/config5.py --fp16 >> $O/c5.log 2>> $O/err.log || exit 2
  done
done
