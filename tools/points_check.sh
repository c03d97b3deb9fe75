#!/bin/bash
# points-in pipeline: GPU tests, then the rate at 128^3 (configs[3]) and 256^3
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-pts}
mkdir -p $O
export C3H_REQUIRE_GPU=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_points.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || exit 3
timeout -k 10 200 python -u tools/points_bench.py 128 512 32 > $O/pb128.jsonl 2>&1 || exit 4
timeout -k 10 200 python -u tools/points_bench.py 256 256 32 > $O/pb256.jsonl 2>&1 || exit 5
