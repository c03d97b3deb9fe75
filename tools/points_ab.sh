#!/bin/bash
# points-in A/B: tools/points_bench.py at 128^3 (configs[3]) and 256^3 on the default build and
# lib/variants/<name>.so, interleaved.  usage: tools/points_ab.sh OUT VARIANT...
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-pab}
shift
mkdir -p $O
for rep in 1 2; do
  for v in default "$@"; do
    if [ $v = default ]; then unset C3HLAC_LIB; else export C3HLAC_LIB=$R/mapping-private_amd/lib/variants/$v.so; fi
    timeout -k 10 200 python -u tools/points_bench.py 128 512 32 > $O/p128_$v.$rep.jsonl 2>> $O/err.log || exit 3
    timeout -k 10 200 python -u tools/points_bench.py 256 256 32 > $O/p256_$v.$rep.jsonl 2>> $O/err.log || exit 4
  done
done
unset C3HLAC_LIB
for f in $O/p*.jsonl; do python3 -c "
import json
for l in open('$f'):
    if l.startswith('{'): d=json.loads(l)
print('$(basename $f)', round(d['frames_per_s']), round(d['vox_us_per_frame'],2), round(d['tick_us_per_frame'],2), d['batched'])"; done
