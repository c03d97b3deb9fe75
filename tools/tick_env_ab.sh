#!/bin/bash
# tick A/B over diagnostics-build environment knobs: the bench command on lib/variants/diag.so
# with each "NAME=VALUE" setting (and none), interleaved, 2 rounds; plus the default build.
# usage: tools/tick_env_ab.sh OUT "K=V" ...
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-teab}; shift
mkdir -p $O
for rep in 1 2; do
  timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --point-frames 0 > $O/b_default.$rep.json 2>> $O/err.log || exit 3
  for kv in none "$@"; do
    tag=${kv//=/_}
    if [ "$kv" = none ]; then
      C3HLAC_LIB=$R/mapping-private_amd/lib/variants/diag.so timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --point-frames 0 > $O/b_diag_$tag.$rep.json 2>> $O/err.log || exit 3
    else
      env "$kv" C3HLAC_LIB=$R/mapping-private_amd/lib/variants/diag.so timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --point-frames 0 > $O/b_diag_$tag.$rep.json 2>> $O/err.log || exit 3
    fi
  done
done
for f in $O/b_*.json; do python3 -c "
import json
d=json.loads(open('$f').read().strip().splitlines()[-1])
print('$(basename $f)', round(d['value']/1e3), round(d['roofline']['avg_launch_ms'],4), round(d['roofline']['frac'],4))"; done
