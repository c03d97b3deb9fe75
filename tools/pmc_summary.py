"""Per-launch HBM traffic of the C3 stage from rocprofv3 --pmc passes (tools/pmc.sh).

FETCH_SIZE / WRITE_SIZE are in KB per dispatch.  gfx950 correction
(MI355X_MICROARCH.md, HBM/rocprofv3): FETCH_SIZE reports exactly half of the bytes of a
wide coalesced streaming read -> x2; WRITE_SIZE is exact for 16-B stores.
The pipelined path's dominant kernel is c3h_tick_kernel: its bytes are summed over all
tick dispatches and divided by the frames that went through the pipeline (each frame
passes every role exactly once).  Gathers (tile halos, box sums) are 4-16 B per lane and
uncalibrated: the x2 correction is exact only for the occupancy stream, which is ~90 %
of the bytes.
Usage: python tools/pmc_summary.py <pmc_dir> <out.json> [frames_per_dispatch] [pipeline_frames]"""
import collections
import csv
import json
import sys
from pathlib import Path

KERNELS = ("c3h_tick_kernel", "c3_occupancy_kernel", "c3hlac_tile_kernel", "compress_gate_kernel", "gate_kernel",
           "score_list_kernel")


def per_kernel(path, counter):
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        name = r["Kernel_Name"]
        for k in KERNELS:  # exact kernel identifier (gate_kernel is not compress_gate_kernel)
            if ("::" + k + "(") in name or ("::" + k + "<") in name or name.startswith(k + "("):
                acc[k].append(float(r["Counter_Value"]))
    return {k: (sum(v) / len(v), len(v), sum(v)) for k, v in acc.items()}


def main():
    d = Path(sys.argv[1])
    fetch = per_kernel(next((d / "fetch").glob("*counter_collection.csv")), "FETCH_SIZE")
    write = per_kernel(next((d / "write").glob("*counter_collection.csv")), "WRITE_SIZE")
    out = {"source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate passes; FETCH x2 (gfx950)",
           "kernels": {}}
    for k in KERNELS:
        if k in fetch or k in write:
            f = fetch.get(k, (0.0, 0))[0] * 1024 * 2
            w = write.get(k, (0.0, 0))[0] * 1024
            out["kernels"][k] = {"fetch_bytes": f, "write_bytes": w, "hbm_bytes": f + w,
                                 "dispatches": max(fetch.get(k, (0, 0))[1], write.get(k, (0, 0))[1])}
    if "c3h_tick_kernel" in fetch and "c3h_tick_kernel" in write and len(sys.argv) > 4:
        frames = int(sys.argv[4])
        tot = fetch["c3h_tick_kernel"][2] * 1024 * 2 + write["c3h_tick_kernel"][2] * 1024
        out["tick_pipeline_frames"] = frames
        out["tick_hbm_bytes_per_frame"] = tot / frames
    fpd = int(sys.argv[3]) if len(sys.argv) > 3 else 1
    out["frames_per_dispatch"] = fpd
    c3 = [out["kernels"][k]["hbm_bytes"] for k in ("c3_occupancy_kernel", "c3hlac_tile_kernel") if k in out["kernels"]]
    out["c3_stage_hbm_bytes_per_dispatch"] = sum(c3) if len(c3) == 2 else None
    out["c3_stage_hbm_bytes_per_frame"] = sum(c3) / fpd if len(c3) == 2 else None
    json.dump(out, open(sys.argv[2], "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
