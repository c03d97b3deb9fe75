"""Per-batch timeline of the last c3h_run_point_frames call in a rocprofv3 kernel trace
(tools/session.sh ... points_prof): every c3h kernel of the call with its queue, start,
end and duration relative to the call's first kernel, then per queue the busy time and the
gaps between consecutive kernels (the voxeliser's stream is the critical path of a
points-in call: accumulate -> reduce -> scatter -> bucket -> exact per batch).
usage: python tools/points_timeline.py TRACE.csv [kernels_per_call_gap_us]"""
import csv
import re
import sys


def name(s):
    s = s.replace("(anonymous namespace)", "")
    m = re.search(r"([A-Za-z_0-9]+)(<[^>]*>)?\(", s)
    return m.group(1) if m else s[:30]


def main():
    rows = [r for r in csv.DictReader(open(sys.argv[1])) if "c3h::" in r["Kernel_Name"]]
    gap_us = float(sys.argv[2]) if len(sys.argv) > 2 else 500.0
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Queue_Id"], name(r["Kernel_Name"]))
                for r in rows)
    # calls are separated by host gaps longer than gap_us with no kernel running
    calls, cur, end = [], [], 0
    for e in ev:
        if cur and e[0] - end > gap_us * 1e3:
            calls.append(cur)
            cur = []
        cur.append(e)
        end = max(end, e[1])
    calls.append(cur)
    last = calls[-1]
    t0 = last[0][0]
    for s, e, q, n in last:
        print("q%s %-26s %9.1f %9.1f %7.1f" % (q, n, (s - t0) / 1e3, (e - t0) / 1e3, (e - s) / 1e3))
    span = (max(e for _, e, _, _ in last) - t0) / 1e3
    print("calls in trace: %d; last call span %.1f us" % (len(calls), span))
    for q in sorted({x[2] for x in last}):
        ks = [x for x in last if x[2] == q]
        busy = sum(e - s for s, e, _, _ in ks) / 1e3
        gaps = [(ks[i + 1][0] - ks[i][1]) / 1e3 for i in range(len(ks) - 1)]
        print("queue %s: %d kernels, busy %.1f us, gaps total %.1f us (median %.1f)" %
              (q, len(ks), busy, sum(g for g in gaps if g > 0), sorted(gaps)[len(gaps) // 2] if gaps else 0.0))


if __name__ == "__main__":
    main()
