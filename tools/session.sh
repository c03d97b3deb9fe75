#!/bin/bash
# One GPU session on the pool box (run through gpurun from the repo root): the named steps
# in order, each under its own time limit, stopping at the first failure.  Every round-6
# figure in DESIGN.md names the session command that produced it.
#   usage: bash tools/session.sh TAG STEP [STEP...]      output: gpurun_out/TAG/
# steps:
#   tests            pytest -m gpu (one process)           -> tests.txt
#   test=PATH[::K]   one test file or node                 -> test_<n>.txt
#   smoke            __graft_entry__.smoke()               -> smoke.log
#   bench            the driver's bench command            -> bench.json
#   prof             the bench under rocprofv3 --kernel-trace --stats, the timed ticks
#                    against the bench line (tools/tick_trace.py)  -> prof/, tick_trace.json
#   rehearse=N       bench.py --gpus N with every rank on device 0 over gloo (C3H_BENCH_REHEARSAL=1:
#                    the multi-rank code path on a one-GPU box; not a measurement) -> rehearse_N.json
#   pmc              HBM traffic passes of the bench (tools/pmc.sh) -> pmc/summary.json
#   shard            configs[3]'s per-rank shard at N = 1..8 (tools/points_shard.py) -> shard.jsonl
#   points[=G,F,B]   points-in rate (tools/points_bench.py, default 128,512,64) -> points.jsonl
#   points_prof[=G,F,B] the same under rocprofv3 --kernel-trace --stats -> points_prof_B/, points_timeline_B.txt
#   hiptrace=G,F,B   points_bench under rocprofv3 --kernel-trace --hip-trace (host API timeline)
#                    -> hiptrace_B/
#   roles            points-in tick roles, diagnostics build (lib/variants/diag.so,
#                    C3H_TICK_PROF)                         -> tick_roles_points.txt
#   single           the single-frame block under --kernel-trace --memory-copy-trace
#                    (tools/single_frame_trace.py)          -> single/
#   singleblock      the single-frame block alone, no profiler (tools/single_frame_trace.py 40)
#                    -> single_block_<VARIANT or product>.json
#   singlephase      the single-frame block with C3H_PROF phase lines (needs VARIANT=diag:
#                    a -DC3H_DIAG build)                    -> single_phases.txt, single_phase_block.json
#   singlehip        the same with --hip-trace (host API timeline)  -> singlehip/
#   config5          BASELINE configs[4] stage times (tools/config5.py --fp16) -> config5.log
#   real_views       the reference's 126 committed Kinect views (tools/real_views_bench.py) -> real_views.json
#   tileprof         the dot4 tile body's phases on a points-in frame (tools/tile_prof.py; with
#                    VARIANT=<a diagnostics build> the C3H_PROF phase lines) -> tile_prof.*
# Variants: VARIANT=name selects lib/variants/name.so for the python steps (C3HLAC_LIB).
set -o pipefail
TAG=$1
shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
export C3H_REQUIRE_GPU=1
if [ -n "$VARIANT" ]; then export C3HLAC_LIB=$R/mapping-private_amd/lib/variants/$VARIANT.so; fi
PYT="python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider"
prof() {  # rocprofv3 needs the program itself after --
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 "$@")
}
for step in "$@"; do
  echo "[session $TAG] $step $(date -u +%H:%M:%S)"
  case $step in
    tests) timeout -k 10 1000 $PYT tests -m gpu > $O/tests.txt 2>&1 || exit 10 ;;
    test=*) t=${step#test=}; n=$(basename ${t%%::*} .py)
      timeout -k 10 600 $PYT "$t" > $O/test_$n.txt 2>&1 || exit 11 ;;
    smoke) timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit 12 ;;
    bench) timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || exit 13 ;;
    prof) prof 600 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- \
            python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline --single-frames 0 > $O/prof_bench.json 2> $O/prof_bench.err || exit 14
          python3 tools/tick_trace.py $O/prof/run_kernel_trace.csv 5 20 $O/prof_bench.json > $O/tick_trace.json || exit 14 ;;
    rehearse=*) n=${step#rehearse=}
      C3H_BENCH_REHEARSAL=1 timeout -k 10 600 python -u bench.py --gpus $n --steps 5 --warmup 2 --no-cpu-baseline \
        > $O/rehearse_$n.json 2> $O/rehearse_$n.err || exit 25 ;;
    pmc) bash tools/pmc.sh $TAG > $O/pmc.log 2>&1 || exit 15 ;;
    shard) timeout -k 10 500 python -u tools/points_shard.py ${SHARD_B:-64,32,16} 3 > $O/shard.jsonl 2> $O/shard.err || exit 16 ;;
    points|points=*) a=${step#points}; a=${a#=}; IFS=, read G F B <<< "${a:-128,512,64}"
      timeout -k 10 300 python -u tools/points_bench.py $G $F $B > $O/points_${G}_${B}.jsonl 2> $O/points.err || exit 17 ;;
    points_prof|points_prof=*) a=${step#points_prof}; a=${a#=}; IFS=, read G F B <<< "${a:-128,512,64}"
      prof 300 rocprofv3 --kernel-trace --stats -d $O/points_prof_$B -o run --output-format csv -- \
            python3 $R/tools/points_bench.py $G $F $B > $O/points_prof_$B.jsonl 2> $O/points_prof.err || exit 18
      python3 tools/points_timeline.py $O/points_prof_$B/run_kernel_trace.csv > $O/points_timeline_$B.txt || exit 18 ;;
    hiptrace=*) a=${step#hiptrace=}; IFS=, read G F B <<< "$a"
      prof 300 rocprofv3 --kernel-trace --hip-trace -d $O/hiptrace_$B -o run --output-format csv -- \
            python3 $R/tools/points_bench.py $G $F $B > $O/hiptrace_$B.jsonl 2> $O/hiptrace.err || exit 27 ;;
    roles) rm -f $O/tick_roles_points.txt
      C3HLAC_LIB=$R/mapping-private_amd/lib/variants/diag.so C3H_TICK_PROF=$O/tick_roles_points.txt \
        timeout -k 10 300 python -u tools/points_bench.py 128 512 64 > $O/roles_points.jsonl 2> $O/roles.err || exit 19 ;;
    single) prof 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $O/single -o run --output-format csv -- \
            python3 $R/tools/single_frame_trace.py 40 > $O/single_block.json 2> $O/single.err || exit 20 ;;
    singleblock) timeout -k 10 300 python -u tools/single_frame_trace.py 40 > $O/single_block_${VARIANT:-product}.json 2> $O/singleblock.err || exit 26 ;;
    singlephase) rm -f $O/single_phases.txt
      C3H_PROF=$O/single_phases.txt timeout -k 10 300 python -u tools/single_frame_trace.py 20 > $O/single_phase_block.json 2> $O/singlephase.err || exit 24 ;;
    singlehip) prof 300 rocprofv3 --kernel-trace --memory-copy-trace --hip-trace -d $O/singlehip -o run --output-format csv -- \
            python3 $R/tools/single_frame_trace.py 40 > $O/singlehip_block.json 2> $O/singlehip.err || exit 28 ;;
    config5) timeout -k 10 300 python -u tools/config5.py --fp16 > $O/config5.log 2>&1 || exit 21 ;;
    real_views) timeout -k 10 300 python -u tools/real_views_bench.py tests/golden/kinect_views_126.npz > $O/real_views.json 2> $O/real_views.err || exit 22 ;;
    tileprof) C3H_PROF=$O/tile_prof_phases.txt timeout -k 10 200 python -u tools/tile_prof.py 20 981 10 > $O/tile_prof.json 2> $O/tile_prof.err || exit 23 ;;
    *) echo "unknown step $step" >&2; exit 2 ;;
  esac
done
echo "[session $TAG] done $(date -u +%H:%M:%S)"
