#!/bin/bash
# round 5, session o: the bench line's points-in pass (many off-cell voxels per frame) with
# the dot4 fixup against the previous build, interleaved; kernel trace of the product's run
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5o
mkdir -p $O
V=$R/mapping-private_amd/lib/variants
for rep in 1 2; do
  for v in default prefix; do
    if [ $v = default ]; then unset C3HLAC_LIB; else export C3HLAC_LIB=$V/$v.so; fi
    timeout -k 10 300 python3 bench.py --steps 10 --warmup 4 --no-cpu-baseline --single-frames 0 \
      | sed "s/^/{\"v\": \"$v\", \"d\": /; s/$/}/" >> $O/bench.jsonl 2>> $O/err.log || exit 2
  done
done
unset C3HLAC_LIB
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- \
  python3 $R/bench.py --steps 10 --warmup 4 --no-cpu-baseline --single-frames 0 > $O/prof.log 2>&1 || exit 5
