"""Average c3h_tick_kernel duration of bench.py's timed region (its last t tick calls) from a rocprofv3 kernel
trace, to check against the bench line's roofline.avg_launch_ms.
usage: tools_tick_trace.py run_kernel_trace.csv WARMUP STEPS BATCH [bench.json]"""
import csv
import json
import sys

PIPE_DEPTH = 4
trace, warmup, steps, batch = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
if len(sys.argv) > 5:  # the bench line knows its frames per launch
    batch = json.load(open(sys.argv[5]))["config"].get("frames_per_launch", batch)
rows = [r for r in csv.DictReader(open(trace)) if "c3h_tick_kernel" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
ticks = lambda n: -(-n // batch) + PIPE_DEPTH - 1 if n else 0  # noqa: E731
w, t = ticks(warmup), ticks(steps)
dur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in rows]
timed = dur[len(dur) - t:]  # the timed region is the last bench run on the pipeline
out = {"tick_calls": len(dur), "warmup_ticks": w, "timed_ticks": len(timed),
       "timed_avg_ms": sum(timed) / len(timed), "timed_min_ms": min(timed), "timed_max_ms": max(timed),
       "all_avg_ms": sum(dur) / len(dur)}
if len(sys.argv) > 5:
    b = json.load(open(sys.argv[5]))
    out["bench_avg_launch_ms"] = b["roofline"]["avg_launch_ms"]
    out["ratio_trace_over_bench"] = out["timed_avg_ms"] / out["bench_avg_launch_ms"]
print(json.dumps(out, indent=1))
