"""Diagnostics: time the C3-HLAC kernel phases on one 256^3 frame (run on the GPU box)."""
import os, sys, time
sys.path[:0] = ["mapping-private_amd"]
import numpy as np
import c3hlac
from c3hlac import synth

pts = synth.kinect_scene(1_000_000, grid=256, leaf=0.01, seed=synth.BASE_SEED)
dense = synth.dense_words(256, seed=3)
res = {}
with c3hlac.Context(0) as ctx:
    for name, setup in (("kinect", lambda: ctx.voxelize(pts, 0.01)), ("dense", lambda: ctx.set_grid(dense.reshape(-1), (256, 256, 256)))):
        setup()
        for mode in ("0", "1", "2", "3", "4"):
            os.environ["C3H_C3_DEBUG"] = mode
            for variant, S in ((117, 10), (981, 10)):
                ctx.extract(variant, (147, 146, 148), S)
                ctx.synchronize()
                ctx.timing(True)
                ctx.kernel_times(reset=True)
                for _ in range(20):
                    ctx.extract(variant, (147, 146, 148), S)
                kt = ctx.kernel_times(reset=True)
                ctx.timing(False)
                ms, n = kt["c3hlac"]
                print("%-6s debug=%s variant=%d S=%d: %.1f us" % (name, mode, variant, S, ms / n * 1e3), flush=True)
        os.environ["C3H_C3_DEBUG"] = "0"
        for grid in ("256", "512", "768", "1024"):
            os.environ["C3H_TILE_GRID"] = grid
            ctx.extract(117, (147, 146, 148), 10)
            ctx.synchronize()
            ctx.timing(True)
            ctx.kernel_times(reset=True)
            for _ in range(20):
                ctx.extract(117, (147, 146, 148), 10)
            ms, n = ctx.kernel_times(reset=True)["c3hlac"]
            ctx.timing(False)
            print("%-6s grid=%s: %.1f us" % (name, grid, ms / n * 1e3), flush=True)
        os.environ.pop("C3H_TILE_GRID")
