#!/bin/bash
# round 5, session t: the self-launch once more on the final code -- two ranks on the box's
# one GPU (rehearsal), and --gpus 2 without it (must exit 2: one device)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5t
mkdir -p $O
C3H_BENCH_REHEARSAL=1 timeout -k 10 400 python bench.py --gpus 2 --steps 10 --warmup 5 --no-cpu-baseline \
  --point-frames 128 --host-point-frames 16 --single-frames 0 > $O/rehearsal2.json 2> $O/rehearsal2.err || exit 3
timeout -k 10 120 python bench.py --gpus 2 --steps 5 --warmup 2 > $O/gpus2_one_device.out 2> $O/gpus2_one_device.err
echo "exit=$?" >> $O/gpus2_one_device.out
exit 0
