#!/bin/bash
# per-role tick timeline (diagnostics build lib/variants/diag.so, C3H_TICK_PROF): the bench
# command once, every tick's role start/end spread appended to OUT/tick_roles.txt
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-tprof}
mkdir -p $O
rm -f $O/tick_roles.txt
C3HLAC_LIB=$R/mapping-private_amd/lib/variants/diag.so C3H_TICK_PROF=$O/tick_roles.txt \
  timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --point-frames 0 > $O/bench.json 2> $O/err.log
