"""Average c3h_tick_kernel duration of bench.py's timed region from a rocprofv3 kernel trace,
to check against the bench line's roofline.avg_launch_ms.

bench.py's tick launches, in order: the allocation prime (c3h_run_frames of 4 batches:
4 + 3 drain ticks), W warmup ticks, the K timed ticks, 3 drain ticks; then (round 3) the
points-in pass's own ticks, which are not counted here.
usage: tools/tick_trace.py run_kernel_trace.csv WARMUP STEPS [bench.json]"""
import csv
import json
import sys

PIPE_DEPTH = 4
PRIME_TICKS = PIPE_DEPTH + PIPE_DEPTH - 1
trace, warmup, steps = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
rows = [r for r in csv.DictReader(open(trace)) if "c3h_tick_kernel" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
dur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in rows]
assert len(dur) >= PRIME_TICKS + warmup + steps + PIPE_DEPTH - 1, (len(dur), warmup, steps)
timed = dur[PRIME_TICKS + warmup:PRIME_TICKS + warmup + steps]
starts = [int(r["Start_Timestamp"]) for r in rows][PRIME_TICKS + warmup:PRIME_TICKS + warmup + steps]
ends = [int(r["End_Timestamp"]) for r in rows][PRIME_TICKS + warmup:PRIME_TICKS + warmup + steps]
out = {"tick_calls": len(dur), "bench_tick_calls": PRIME_TICKS + warmup + steps + PIPE_DEPTH - 1, "timed_ticks": len(timed),
       "timed_avg_ms": sum(timed) / len(timed), "timed_min_ms": min(timed), "timed_max_ms": max(timed),
       "timed_span_ms": (ends[-1] - starts[0]) / 1e6,
       "gap_fraction": 1 - sum(timed) / ((ends[-1] - starts[0]) / 1e6)}
if len(sys.argv) > 4:
    b = json.load(open(sys.argv[4]))
    out["bench_avg_launch_ms"] = b["roofline"]["avg_launch_ms"]
    out["bench_ms_per_step"] = b["ms_per_step"]
    out["ratio_trace_over_bench"] = out["timed_avg_ms"] / out["bench_avg_launch_ms"]
print(json.dumps(out, indent=1))
