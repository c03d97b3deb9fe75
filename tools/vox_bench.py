"""Voxeliser rate on MI355X: c3h_voxelize of 1M-point Kinect-style frames (256^3, leaf
1 cm) from device-resident points, timed with the library's HIP events (the three
launches of one call; the call's host round trip for the grid info is outside them).
usage: python tools/vox_bench.py [reps]"""
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT / "mapping-private_amd")]


def main():
    import torch
    import c3hlac
    from c3hlac import synth
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 50
    dev = torch.device("cuda", 0)
    frames = [torch.from_numpy(synth.kinect_scene(1_000_000, grid=256, leaf=0.01, seed=synth.BASE_SEED + s)).to(dev)
              for s in range(4)]
    torch.cuda.synchronize()
    out = {}
    with c3hlac.Context(0) as ctx:
        for f in frames:  # warm: allocations, first-touch
            ctx.voxelize(f, 0.01)
        ctx.timing(True)
        ctx.kernel_times(reset=True)
        n_pts = 0
        for i in range(reps):
            gi = ctx.voxelize(frames[i % 4], 0.01)
            n_pts += frames[i % 4].shape[0]
        ms, cnt = ctx.kernel_times(reset=True)["voxelize"]
        ctx.timing(False)
        ctx.voxelize(frames[0], 0.01)
        w = ctx.grid()
        check = int((w.astype(np.uint64) * (np.arange(w.size, dtype=np.uint64) | np.uint64(1))).sum() & np.uint64(2**63 - 1))
        per = ms / reps
        occ = int(gi.n_occ)
        alg = 16 * 1_000_000 + 4 * 256 ** 3  # 16 B/point read + 4 B/voxel grid
        out = {"frames": reps, "us_per_frame": per * 1e3, "mpoints_per_s": n_pts / (ms / 1e3) / 1e6,
               "occupied_voxels": occ, "grid_checksum": check, "algorithmic_bytes": alg,
               "algorithmic_GBps": alg / (per / 1e3) / 1e9, "frac_of_8TBps": alg / (per / 1e3) / 8e12}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
