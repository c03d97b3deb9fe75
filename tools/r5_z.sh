#!/bin/bash
# end of round 5: GPU tests, smoke(), the driver's bench command, and a kernel-trace summary
# of the same bench command (profiles/r5/bench/r5z_*)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5z
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.txt 2>&1 || exit 2
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit 3
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || exit 4
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 5 --single-frames 0 > $O/prof_bench.json 2> $O/prof_bench.err || exit 5
