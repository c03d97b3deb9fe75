#!/bin/bash
# tick A/B: the driver's bench command on the default build and lib/variants/<name>.so,
# interleaved, 2 rounds.  usage: tools/tick_ab.sh OUT VARIANT...
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-tab}
shift
mkdir -p $O
for rep in 1 2; do
  for v in default "$@"; do
    if [ $v = default ]; then unset C3HLAC_LIB; else export C3HLAC_LIB=$R/mapping-private_amd/lib/variants/$v.so; fi
    timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --point-frames 0 > $O/b_$v.$rep.json 2>> $O/err.log || exit 3
  done
done
unset C3HLAC_LIB
for f in $O/b_*.json; do python3 -c "
import json,sys
d=json.loads(open('$f').read().strip().splitlines()[-1])
print('$(basename $f)', round(d['value']/1e3), round(d['roofline']['avg_launch_ms'],4), round(d['roofline']['frac'],4))"; done
