"""Automatic colour threshold on the GPU: per-channel histograms of the
occupied voxels of resident 256^3 grids + the threshold arithmetic.  Algorithmic bytes =
4 B/voxel (one read of the packed grid).  Prints the per-call time from HIP events on the
context's stream (memset + kernel + 6 KB readback) and the HBM rate; run under
`rocprofv3 --kernel-trace --stats` for the kernel-only duration (colour_hist_kernel)."""
import os
import sys
import time

sys.path[:0] = [os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "mapping-private_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402
import c3hlac  # noqa: E402
from c3hlac import synth  # noqa: E402

G, LEAF = 256, 0.01
dev = torch.device("cuda", 0)
with c3hlac.Context(0) as ctx:
    stream = torch.cuda.current_stream(dev)
    ctx.set_stream(stream.cuda_stream)
    grids = {}
    pts = synth.kinect_scene(1_000_000, grid=G, leaf=LEAF, seed=synth.BASE_SEED)
    ctx.voxelize(pts, LEAF)
    grids["kinect"] = torch.from_numpy(ctx.grid().reshape(-1).view(np.int32)).to(dev)
    grids["dense"] = torch.from_numpy(synth.dense_words(G, seed=3).reshape(-1).view(np.int32)).to(dev)
    for name, g in grids.items():
        ctx.lib.c3h_set_grid(ctx.h, c3hlac.ptr(g), c3hlac.i32x3((G, G, G)), c3hlac.i32x3((0, 0, 0)),
                             float(LEAF), 1)
        hist = np.zeros((3, 256), np.int64)
        ctx.color_histogram(hist)
        n = 50
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        e0.record(stream)
        for _ in range(n):
            ctx.color_histogram(hist)
        e1.record(stream)
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t0) / n
        ms = e0.elapsed_time(e1) / n
        thr, ave = c3hlac.auto_threshold(hist)
        print("%-6s occupied %d: %.1f us/call (events), %.1f us/call (host wall), %.2f TB/s of 4 B/voxel; "
              "threshold %s" % (name, hist[0].sum() // (n + 1), ms * 1e3, wall * 1e6, G ** 3 * 4 / (ms * 1e-3) / 1e12,
                                list(thr)), flush=True)
