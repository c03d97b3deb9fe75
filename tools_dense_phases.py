"""Diagnostics: C3-HLAC kernel phases on a dense grid (config 5 style): C3H_C3_DEBUG
3 = occupancy pass only, 1 = + halo loads, 2 = + compaction, 0 = full; and tile grids.
usage: python tools_dense_phases.py [grid]"""
import os
import sys
sys.path[:0] = [os.path.join(os.path.dirname(os.path.abspath(__file__)), "mapping-private_amd")]
import c3hlac  # noqa: E402
from c3hlac import synth  # noqa: E402

G = int(sys.argv[1]) if len(sys.argv) > 1 else 512
dense = synth.dense_words(G, seed=3).reshape(-1)
with c3hlac.Context(0) as ctx:
    ctx.set_grid(dense, (G, G, G))
    for variant in (981, 117):
        for mode, grid in (("3", ""), ("1", ""), ("2", ""), ("0", ""), ("0", "1024"), ("0", "2048")):
            os.environ["C3H_C3_DEBUG"] = mode
            if grid:
                os.environ["C3H_TILE_GRID"] = grid
            else:
                os.environ.pop("C3H_TILE_GRID", None)
            ctx.extract(variant, (147, 146, 148), 10)
            ctx.synchronize()
            ctx.timing(True)
            ctx.kernel_times(reset=True)
            for _ in range(3):
                ctx.extract(variant, (147, 146, 148), 10)
            kt = ctx.kernel_times(reset=True)
            ctx.timing(False)
            ms, n = kt["c3hlac"]
            print("dense %d variant=%d debug=%s grid=%s: %.3f ms" % (G, variant, mode, grid or "-", ms / n), flush=True)
