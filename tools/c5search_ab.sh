#!/bin/bash
# config-5 search (f32 precision) timings for the default build and variants, then the
# large-grid engine tests.  usage: tools/c5search_ab.sh OUT VARIANT...
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-c5s}; shift
mkdir -p $O
for rep in 1 2; do
  for v in default "$@"; do
    if [ $v = default ]; then unset C3HLAC_LIB; else export C3HLAC_LIB=$R/mapping-private_amd/lib/variants/$v.so; fi
    timeout -k 10 200 python -u tools/config5.py > $O/$v.$rep.log 2>&1 || exit 3
  done
done
unset C3HLAC_LIB
grep -H "config5: search" $O/*.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 $R/tools/config5.py > $O/prof.log 2>&1 || exit 4
cd $R
export C3H_REQUIRE_GPU=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_config5_nonperiodic.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || exit 5
