#!/bin/bash
# smoke() on cuda:0, then the driver's bench command once more (box-to-box variance)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-fin}
mkdir -p $O
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit 3
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || exit 4
