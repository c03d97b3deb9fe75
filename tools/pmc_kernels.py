"""Per-kernel averages of rocprofv3 --pmc counter CSVs (one directory per pass) and the
kernel-trace stats: python tools/pmc_kernels.py <dir> [kernel substrings...]"""
import collections
import csv
import json
import sys
from pathlib import Path


def main():
    d = Path(sys.argv[1])
    keys = sys.argv[2:] or ["voxb_accum", "voxb_scatter", "c3h_tick_kernel"]
    out = collections.defaultdict(dict)
    for f in d.glob("*/*counter_collection.csv"):
        acc = collections.defaultdict(list)
        for r in csv.DictReader(open(f)):
            for k in keys:
                if k in r["Kernel_Name"]:
                    acc[(k, r["Counter_Name"])].append(float(r["Counter_Value"]))
        for (k, c), v in acc.items():
            out[k][c] = sum(v) / len(v)
            out[k][c + "_n"] = len(v)
    for f in d.glob("trace/*kernel_stats.csv"):
        for r in csv.DictReader(open(f)):
            for k in keys:
                if k in r["Name"]:
                    out[k]["avg_ns"] = float(r["AverageNs"])
                    out[k]["calls"] = int(r["Calls"])
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
