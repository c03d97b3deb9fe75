"""All 1,512 reference Kinect views through c3h_run_point_frames (VERDICT r3 item 3's
measurement): the status-1 share, off-cell voxels corrected in the batch, frames/s with the
views resident in HBM, and the batch's records against the single-frame path for every view.

Input: gpurun_data/kinect_views_all.npz (tests/golden/gen_kinect_views.py --all; not
committed, copied in-tree for the measurement run).  Prints one JSON line.

    python tools/real_views_bench.py [npz] [--exact 0|1]
"""
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
    src = Path(sys.argv[1]) if len(sys.argv) > 1 and not sys.argv[1].startswith("--") else \
        ROOT / "gpurun_data" / "kinect_views_all.npz"
    with np.load(src, allow_pickle=False) as z:
        st, P = z["starts"], z["pts"]
        views = [np.ascontiguousarray(P[st[i]:st[i + 1]]) for i in range(len(st) - 1)]
    dev = torch.device("cuda", 0)
    frames = [torch.from_numpy(v).to(dev) for v in views]
    ctx = c3hlac.Context(0)
    leaf, canvas, S, box, exist, thr = 0.01, (40, 40, 40), 4, (2, 2, 2), 4, (147, 146, 148)
    M = 3
    axis_t, var, axis_q = synth.random_bases(117, 30, M, 5, seed=synth.BASE_SEED + 91)
    ctx.search_setup(axis_t, var, axis_q)
    ctx.set_rank(1)
    ctx.set_batch(64)
    ctx.set_pipeline(True)
    n = len(frames)
    d_out = torch.zeros((n, 3 * M), dtype=torch.int64, device=dev)
    args = (leaf, canvas, 117, thr, S, box, exist, True, d_out)
    ctx.run_point_frames(frames, *args)  # untimed: sizes the buffers
    torch.cuda.synchronize()
    times = []
    for _ in range(5):
        t0 = time.perf_counter()
        _, info = ctx.run_point_frames(frames, *args)
        torch.cuda.synchronize()
        times.append(time.perf_counter() - t0)
    got = d_out.cpu().numpy().view(c3hlac.DET_DTYPE).reshape(n, M)
    mism = []
    for i in range(n):
        ctx.voxelize(views[i], leaf)
        ctx.extract(117, thr, S)
        ctx.set_rank(1)
        lists, _ = ctx.search(box, exist)
        if not np.array_equal(got[i], lists[:, 0]):
            mism.append(i)
    st_ = info["status"]
    print(json.dumps({
        "views": n, "points": int(st[-1]),
        "batched": int((st_ == 0).sum()), "single_frame_path": int((st_ == 1).sum()),
        "errors": int((st_ < 0).sum()),
        "batched_share": float((st_ == 0).mean()),
        "views_with_moved_voxels": int((info["n_moved"] > 0).sum()), "moved_voxels": int(info["n_moved"].sum()),
        "frames_per_s": n / min(times), "ms_per_call": 1e3 * min(times),
        "records_equal_single_frame_path": n - len(mism), "mismatches": mism[:20],
        "config": "leaf 0.01, canvas 40^3, C3-HLAC-117 S=4, 117->30, 3 models x r=5, box 2x2x2, rank 1, "
                  "views resident in HBM, batch 64",
    }))
    ctx.close()


if __name__ == "__main__":
    main()
