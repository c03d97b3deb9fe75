#!/bin/bash
# round 5, session b: the bad-voxel check, the whole GPU suite on the product build, then interleaved A/Bs against the
# round-4 kernels (lib/variants/r4*.so, built from the round-4 sources): single-frame
# voxeliser (tools/vox_bench.py), config 5 (tools/config5.py), the batched voxeliser
# (points_bench with and without the voxeliser / tick overlap), kernel traces
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5b
mkdir -p $O
V=$R/mapping-private_amd/lib/variants
STAGE=${1:-all}
if [ $STAGE = tests ] || [ $STAGE = all ]; then
timeout -k 10 200 python3 tools/vox_bad.py > $O/vox_bad.jsonl 2> $O/vox_bad.err || exit 1
export C3H_REQUIRE_GPU=1
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  -s > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc" >> $O/rc.txt; [ $rc -ge 124 ] && exit $rc
fi
[ $STAGE = tests ] && exit 0
if [ $STAGE = pmc ]; then
  tools/pmc_points.sh r5b/pmc256 256 256 || exit 6
  C5ARGS=--fp16 tools/pmc_config5.sh r5b_fp16 || exit 6
  exit 0
fi
for rep in 1 2; do
  for v in default r4; do
    if [ $v = default ]; then unset C3HLAC_LIB; else export C3HLAC_LIB=$V/$v.so; fi
    timeout -k 10 120 python3 tools/vox_bench.py 200 >> $O/vox1_$v.jsonl 2>> $O/err.log || exit 2
    timeout -k 10 180 python3 tools/config5.py --fp16 >> $O/c5_$v.log 2>> $O/err.log || exit 2
  done
done
for rep in 1 2; do
  for v in default r4 noovl r4_noovl; do
    if [ $v = default ]; then unset C3HLAC_LIB; else export C3HLAC_LIB=$V/$v.so; fi
    timeout -k 10 120 python3 tools/points_bench.py 128 512 32 >> $O/pb128_$v.jsonl 2>> $O/err.log || exit 3
    timeout -k 10 120 python3 tools/points_bench.py 256 256 32 >> $O/pb256_$v.jsonl 2>> $O/err.log || exit 3
  done
done
unset C3HLAC_LIB
tools/prof_points.sh r5b/prof_noovl128 128 512 mapping-private_amd/lib/variants/noovl.so || exit 4
tools/prof_points.sh r5b/prof_r4noovl128 128 512 mapping-private_amd/lib/variants/r4_noovl.so || exit 4
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof_vox1 -o run --output-format csv -- python3 $R/tools/vox_bench.py 100 > $O/prof_vox1.log 2>&1 || exit 5
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof_c5 -o run --output-format csv -- python3 $R/tools/config5.py --fp16 > $O/prof_c5.log 2>&1 || exit 5
