"""Diagnostics: host enqueue time vs device time of c3h_run_frames for 1..4 lanes."""
import os
import sys
import time

if len(sys.argv) > 1:  # e.g. GPU_MAX_HW_QUEUES=8 (must precede the HIP runtime's start)
    os.environ["GPU_MAX_HW_QUEUES"] = sys.argv[1]

sys.path[:0] = [os.path.join(os.path.dirname(os.path.abspath(__file__)), "mapping-private_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402
import c3hlac  # noqa: E402
from c3hlac import synth  # noqa: E402

G, LEAF = 256, 0.01
dev = torch.device("cuda", 0)
with c3hlac.Context(0) as ctx:
    ctx.set_stream(torch.cuda.current_stream(dev).cuda_stream)
    grids = []
    for s in range(3):
        pts = synth.kinect_scene(1_000_000, grid=G, leaf=LEAF, seed=synth.BASE_SEED + s)
        ctx.voxelize(pts, LEAF)
        w = torch.empty(G ** 3, dtype=torch.int32, device=dev)
        ctx.lib.c3h_get_grid(ctx.h, c3hlac.ptr(w), 1)
        grids += [w, torch.roll(w.view(G, G, G), 37, 2).reshape(-1).contiguous()]
    if os.environ.get("LANES_ZERO"):  # diagnostics: empty frames (pure streaming)
        grids = [torch.zeros_like(g) for g in grids]
    axis_t, var, axis_q = synth.random_bases(117, 100, 10, 20, seed=synth.BASE_SEED)
    ctx.search_setup(axis_t, var, axis_q)
    ctx.set_rank(1)
    N = 200
    gptr = np.array([grids[i % 6].data_ptr() for i in range(N)], np.uint64)
    dets = torch.zeros((N, 30), dtype=torch.int64, device=dev)
    import os
    cases = [(1, 8, None, None), (1, 1, None, None), (3, 4, None, None), (3, 8, None, None)]
    if os.environ.get("LANES_CASES"):  # "lanes,batch,occ_grid,tile_grid;..." (empty grid = default)
        cases = [tuple(int(v) if i < 2 else (v or None) for i, v in enumerate(c.split(",")))
                 for c in os.environ["LANES_CASES"].split(";")]
    for lanes, batch, og, tg in cases:
        for k, v in (("C3H_TILE_GRID", tg), ("C3H_OCC_GRID", og)):
            if v:
                os.environ[k] = v
            else:
                os.environ.pop(k, None)
        ctx.set_lanes(lanes)
        ctx.set_batch(batch)
        for rep in range(2):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            ctx.run_frames(gptr, (G,) * 3, (0, 0, 0), LEAF, 117, (147, 146, 148), 10, (2, 2, 2), 100, True,
                           dets.data_ptr())
            t1 = time.perf_counter()
            torch.cuda.synchronize()
            t2 = time.perf_counter()
        print("lanes=%d batch=%d occ=%s tile=%s host_enqueue_us_per_frame=%.1f total_us_per_frame=%.1f" %
              (lanes, batch, og, tg, (t1 - t0) / N * 1e6, (t2 - t0) / N * 1e6), flush=True)
        ctx.timing(True)
        ctx.kernel_times(reset=True)
        ctx.run_frames(gptr, (G,) * 3, (0, 0, 0), LEAF, 117, (147, 146, 148), 10, (2, 2, 2), 100, True,
                       dets.data_ptr())
        kt = ctx.kernel_times(reset=True)
        ctx.timing(False)
        print("   per-frame stage us (events; overlapping lanes inflate):",
              {k: round(v[0] / v[1] * 1e3, 2) for k, v in kt.items() if v[1]}, flush=True)
