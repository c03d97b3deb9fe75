#!/bin/bash
# round 5, session a: parity picks, the bench line with the single-frame block, the
# self-launched --gpus 2 rehearsal (both ranks on the one GPU of a pool box)
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r5a
export C3H_REQUIRE_GPU=1
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_parity.py -k "config2 or config3" > $R/gpurun_out/r5a/tests.log 2>&1 || exit 1
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $R/gpurun_out/r5a/bench.json 2> $R/gpurun_out/r5a/bench.err || exit 2
C3H_BENCH_REHEARSAL=1 timeout -k 10 400 python bench.py --gpus 2 --steps 10 --warmup 5 --no-cpu-baseline \
  --point-frames 128 --host-point-frames 16 > $R/gpurun_out/r5a/rehearsal2.json 2> $R/gpurun_out/r5a/rehearsal2.err || exit 3
