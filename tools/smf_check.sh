#!/bin/bash
# matrix-core projection timing (config 5: 10 x r=20 on the matrix cores, 63 x r=70) under
# rocprof, then its parity tests and the production base-swap test.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-smc}
mkdir -p $O
export C3H_REQUIRE_GPU=1
timeout -k 10 200 python -u tools/config5.py --engine 2 > $O/m10.log 2>&1 || exit 3
timeout -k 10 200 python -u tools/config5.py --engine 0 --models 63 --r 70 > $O/stress.log 2>&1 || exit 4
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- \
  python3 $R/tools/config5.py --engine 0 --models 63 --r 70 > $O/prof.log 2>&1 || exit 5
cd $R
timeout -k 10 900 python -u -m pytest tests/test_gpu_score_mfma.py tests/test_gpu_slab.py tests/test_gpu_production.py -x -v \
  --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || exit 6
