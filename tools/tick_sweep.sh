#!/bin/bash
# diagnostics: bench.py at the driver shape with the diagnostics build's tick knobs
# (C3H_TICK_TILE / SCORE / COMP / OCC / ZERO); one line per setting.
# usage: tools/tick_sweep.sh "TILE=48 SCORE=16" "TILE=24 SCORE=8" ...
R=${GRAFT_REPO_ROOT:-$(pwd)}
export C3HLAC_LIB=$R/mapping-private_amd/lib/variants/${VARIANT:-diag}.so
for cfg in "$@"; do
  env $(for kv in $cfg; do echo C3H_TICK_$kv; done) timeout -k 10 120 python $R/bench.py --steps 30 --warmup 6 --no-cpu-baseline --point-frames 0 \
    > $R/gpurun_out/sweep.json 2>/dev/null || { echo "$cfg FAILED"; exit 3; }
  python -c "import json,sys; d=json.loads(open('$R/gpurun_out/sweep.json').read().strip().splitlines()[-1]); print('%-40s %.0f Mvox/s  %.3f ms/step  frac %.3f' % (sys.argv[1], d['value'], d['ms_per_step'], d['roofline']['frac']), flush=True)" "$cfg"
done
