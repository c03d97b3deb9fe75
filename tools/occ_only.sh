#!/bin/bash
# occupancy-role-only tick (diagnostics builds): stream rate of each variant
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/occonly; mkdir -p $O
for rep in 1 2; do for v in diag diagring; do
  C3HLAC_LIB=$R/mapping-private_amd/lib/variants/$v.so C3H_TICK_ROLES=8 timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --point-frames 0 > $O/$v.$rep.json 2>>$O/err.log || exit 3
  python3 -c "import json; d=json.loads(open('$O/$v.$rep.json').read().strip().splitlines()[-1]); print('$v', d['ms_per_step'], d['roofline']['avg_launch_ms'])"
done; done
