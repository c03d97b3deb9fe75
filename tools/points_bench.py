"""Points-in pipeline rate (c3h_run_point_frames) on MI355X: batches of 1M-point Kinect-style
frames from device memory, voxelised by the batched voxeliser into canvas grids and pushed
through the pipelined tick.  Reports per-frame voxeliser time (HIP events around its two
launches per batch), tick time and end-to-end frames/s.
usage: python tools/points_bench.py [grid(128|256)] [frames] [batch] [variant] [M]"""
import json
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT / "mapping-private_amd")]


def main():
    import torch
    import c3hlac
    from c3hlac import synth
    G = int(sys.argv[1]) if len(sys.argv) > 1 else 128
    nfr = int(sys.argv[2]) if len(sys.argv) > 2 else 512
    B = int(sys.argv[3]) if len(sys.argv) > 3 else 32
    variant = int(sys.argv[4]) if len(sys.argv) > 4 else (981 if G == 128 else 117)
    M = int(sys.argv[5]) if len(sys.argv) > 5 else (1 if G == 128 else 10)
    leaf = 2.56 / G
    dev = torch.device("cuda", 0)
    nb = 8
    base = [torch.from_numpy(synth.kinect_scene(1_000_000, grid=G, leaf=leaf, seed=synth.BASE_SEED + 7000 + s)).to(dev)
            for s in range(nb)]

    def frame(i):
        t = base[i % nb].clone()
        k = i // nb
        t[:, 3] = (t[:, 3].view(torch.int32) ^ ((k * 0x2F1D37) & 0xFFFFFF)).view(torch.float32)
        t[:, 0] = (t[:, 0].double() + (k % 16) * leaf).float()
        return t

    frames = [frame(i) for i in range(nfr)]
    torch.cuda.synchronize()
    thr = (147, 146, 148)
    with c3hlac.Context(0) as ctx:
        axis_t, var, axis_q = synth.random_bases(variant, 100, M, 20, seed=31)
        ctx.search_setup(axis_t, var, axis_q)
        ctx.set_rank(1)
        ctx.set_batch(B)
        out = torch.zeros((nfr, 3 * M), dtype=torch.int64, device=dev)
        canvas = (G,) * 3  # frames' extents are G; their min_b differ (x shifts)
        ctx.run_point_frames(frames[:4 * B], leaf, canvas, variant, thr, 10, (2, 2, 2), 100, True, out)
        torch.cuda.synchronize()
        frames = ctx.prepare_point_frames(frames)  # checked once, outside the timed calls (as bench.py)
        res = {}
        for rep in range(6):  # reps 3-5 without the HIP events around the launches
            timed_events = rep < 3
            ctx.timing(c3hlac.timing_mask("voxelize", "pipeline") if timed_events else False)
            ctx.kernel_times(reset=True)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            _, info = ctx.run_point_frames(frames, leaf, canvas, variant, thr, 10, (2, 2, 2), 100, True, out)
            torch.cuda.synchronize()
            el = time.perf_counter() - t0
            kt = ctx.kernel_times(reset=True)
            ctx.timing(False)
            vms, vcnt = kt["voxelize"]
            pms, pcnt = kt["pipeline"]
            res = {"grid": G, "canvas": list(canvas), "frames": nfr, "batch": B, "variant": variant, "M": M,
                   "frames_per_s": nfr / el, "us_per_frame": el / nfr * 1e6,
                   "vox_us_per_frame": vms / max(vcnt, 1) * 1e3, "tick_ms_total": pms,
                   "tick_us_per_frame": pms / nfr * 1e3, "batched": int((info["status"] == 0).sum()),
                   "vox_gpoints_per_s": 1e6 * vcnt / (vms / 1e3) / 1e9 if vms else None, "events": timed_events}
            print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
