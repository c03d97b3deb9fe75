"""Diagnostics: per-block phase timestamps of the tile and score kernels on the bench
workload (env C3H_PROF).  Usage: python tools_phase_probe.py <out.txt>"""
import os
import sys

os.environ["C3H_PROF"] = sys.argv[1]
sys.path[:0] = ["mapping-private_amd"]
import numpy as np  # noqa: E402
import c3hlac  # noqa: E402
from c3hlac import synth  # noqa: E402

G, LEAF = 256, 0.01
with c3hlac.Context(0) as ctx:
    pts = synth.kinect_scene(1_000_000, grid=G, leaf=LEAF, seed=synth.BASE_SEED)
    ctx.voxelize(pts, LEAF)
    axis_t, var, axis_q = synth.random_bases(117, 100, 10, 20, seed=synth.BASE_SEED)
    ctx.search_setup(axis_t, var, axis_q)
    ctx.set_rank(1)
    for i in range(6):
        ctx.clean_max()
        ctx.extract(117, (147, 146, 148), 10)
        ctx.search((2, 2, 2), 100)
print(open(sys.argv[1]).read())
