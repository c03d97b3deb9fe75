#!/bin/bash
# fp16 projection: parity tests (projection file + the config-5 parity test), then config-5
# timings at fp16 search precision (63 x r=70 and 10 x r=20) and a rocprof summary.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-s16}
mkdir -p $O
export C3H_REQUIRE_GPU=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_score_mfma.py tests/test_gpu_parity.py -k "mfma or r70 or config5 or engines" -x -v \
  --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || exit 3
timeout -k 10 200 python -u tools/config5.py --engine 0 --models 63 --r 70 --fp16 > $O/stress16.log 2>&1 || exit 4
timeout -k 10 200 python -u tools/config5.py --engine 0 --fp16 > $O/m10_16.log 2>&1 || exit 5
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- \
  python3 $R/tools/config5.py --engine 0 --models 63 --r 70 --fp16 > $O/prof.log 2>&1 || exit 6
