#!/bin/bash
# voxeliser A/B: default build vs a variant .so (interleaved, 3 runs each), then the
# voxeliser parity tests on the default build.  usage: tools/vox_ab.sh OUT VARIANT
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-vab}
V=${2:-noruns}
mkdir -p $O
export C3H_REQUIRE_GPU=1
for i in 1 2 3; do
  timeout -k 10 120 python -u tools/vox_bench.py 200 >> $O/vox_default.jsonl 2>> $O/vox.err || exit 3
  C3HLAC_LIB=$R/mapping-private_amd/lib/variants/$V.so timeout -k 10 120 python -u tools/vox_bench.py 200 >> $O/vox_$V.jsonl 2>> $O/vox.err || exit 4
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  -k "voxel or golden or cloud or boundary or centroid" > $O/vox_tests.log 2>&1 || exit 5
