#!/bin/bash
# round 5, session c: the GRSD wide-leaf test on the round-4 and current builds, then the
# rest of the GPU suite on the current build (a failing test goes on; a timeout, abort or
# fault ends the script)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5c
mkdir -p $O
export C3H_REQUIRE_GPU=1
stop() { echo "$1 rc=$2" >> $O/rc.txt; [ $2 -ge 124 ] && exit $2; return 0; }
T=tests/test_gpu_grsd.py::test_grsd_leaf_wider_than_four_normal_radii
C3HLAC_LIB=$R/mapping-private_amd/lib/variants/r4.so timeout -k 10 300 python -u -m pytest -x -v --timeout 200 \
  --timeout-method thread -p no:cacheprovider $T > $O/grsd_r4.log 2>&1
stop r4 $?
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider $T \
  > $O/grsd_new.log 2>&1
stop new $?
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  -s --deselect $T > $O/tests.log 2>&1
stop suite $?
