#!/bin/bash
# GPU session for the matrix-core projection: its parity tests, config-5 timings per engine
# (10 x r=20 and the 63 x r=70 stress case) and a rocprof kernel summary of the stress run.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-smf}
mkdir -p $O
export C3H_REQUIRE_GPU=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_score_mfma.py tests/test_gpu_slab.py -x -v --timeout 300 --timeout-method thread \
  -p no:cacheprovider > $O/tests.log 2>&1 || exit 3
for e in 1 2; do
  timeout -k 10 300 python -u tools/config5.py --engine $e > $O/config5_e$e.log 2>&1 || exit 4
done
timeout -k 10 300 python -u tools/config5.py --engine 0 --models 63 --r 70 > $O/config5_stress.log 2>&1 || exit 5
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- \
  python3 $R/tools/config5.py --engine 0 --models 63 --r 70 > $O/prof.log 2>&1 || exit 6
