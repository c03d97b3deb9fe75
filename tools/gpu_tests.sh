#!/bin/bash
# GPU tests only (one pytest process): usage tools/gpu_tests.sh TAG [pytest args...]
set -o pipefail
TAG=${1:-t}
shift
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
export C3H_REQUIRE_GPU=1
timeout -k 10 1000 python -u -m pytest -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider "$@" \
  > $R/gpurun_out/gpu_tests_$TAG.log 2>&1
