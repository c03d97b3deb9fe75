"""Benchmark of the C3-HLAC colour-voxel recognition hot path on MI355X.

Workload (BASELINE.json configs[2], the 256^3 configuration its metric is quoted on):
one step = C3-HLAC-117 over a device-resident 256^3 packed colour/occupancy grid
(subdivision 10 -> 17,576 subdivisions) + setData compression 117 -> 100 + sliding-box
search of 10 models x r=20 over 15,625 box positions (box 2x2x2 subdivisions, rank 1,
exist threshold 100).  Frames are Kinect-style synthetic RGB-D scenes (1M rays each),
voxelised on the GPU before the timed region; 6 distinct frames (> the 256 MiB
Infinity Cache) are cycled so every step reads its grid from HBM.

Multi-GPU (torch.distributed.run, one process per GPU): independent frames are sharded
over ranks with no data-path collective (weak scaling); the per-frame detections are
gathered to rank 0 with one all_gather over RCCL after the timed steps (inside the
timed region).  value = voxels processed by all ranks / max-over-ranks wall time.

Prints ONE JSON line on rank 0.
"""
import argparse
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
sys.path[:0] = [str(ROOT / "mapping-private_amd"), str(ROOT / "oracle")]

GRID, LEAF, VARIANT, SUBDIV = 256, 0.01, 117, 10
D, M, R = 100, 10, 20
BOX, RANK, EXIST_THR = (2, 2, 2), 1, 100
LANES = 3  # batches in flight per GPU on the lanes path (breakdown pass only)
BATCH_MAX = 64  # frames per tick (c3h_set_batch); the tick's latency-bound roles need many
                # frames in flight: 12.8 us/frame at 32 vs 14.1 at 16, 17.9 at 8 (profiles/r1/v8);
                # 64 beats 32 by 2.4 % on the bench (profiles/r1/abbatch_32_vs_64.log)
BATCH = BATCH_MAX  # set per run in main(): at least ~8 batches, so pipeline fill/drain stays small
PIPE_DEPTH = 4  # pipeline ticks a batch spends in flight (occupancy | tile | compress+gate | score)
THR = (147, 146, 148)
N_RAYS = 1_000_000
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table (spec)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3840)
    ap.add_argument("--warmup", type=int, default=64)
    ap.add_argument("--frames", type=int, default=0,
                    help="resident grids (0: BATCH + 8, at least 40; > the 256 MB Infinity Cache, and every "
                         "frame of a tick reads its own grid)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    return ap.parse_args()


def algorithmic_bytes_c3(G, H, F):
    """4 B/voxel packed-grid read + the feature rows + exist written."""
    return G ** 3 * 4 + H * F * 4 + H * 4


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    dist = None
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    import c3hlac
    from c3hlac import synth

    ctx = c3hlac.Context(local)
    stream = torch.cuda.current_stream(dev)
    ctx.set_stream(stream.cuda_stream)
    ctx.set_lanes(LANES)
    global BATCH
    BATCH = int(os.environ.get("C3H_BENCH_BATCH", "0")) or min(BATCH_MAX, max(8, args.steps // 8 // 8 * 8))
    ctx.set_batch(BATCH)
    ctx.set_pipeline(True)

    # ---- inputs: frames voxelised on the GPU, grids kept resident in HBM ------------
    nf = args.frames if args.frames > 0 else max(40, BATCH + 8)
    grids, frame_pts = [], []
    per_scene = 4  # frames per scene: the scene and three x-shifts of it (distinct buffers)
    n_scene = max(1, -(-nf // per_scene))
    t_vox_ms, n_points = [], 0
    for s in range(n_scene):
        seed = synth.BASE_SEED + 1000 * rank + s
        pts = synth.kinect_scene(N_RAYS, grid=GRID, leaf=LEAF, seed=seed)
        if s == 0:
            frame_pts.append(pts)
        d_pts = torch.from_numpy(pts).to(dev)
        ctx.timing(True)
        gi = ctx.voxelize(d_pts, LEAF)
        t_vox_ms.append(ctx.kernel_times(reset=True)["voxelize"][0])
        ctx.timing(False)
        n_points += pts.shape[0]
        assert list(gi.div_b) == [GRID] * 3, list(gi.div_b)
        words = torch.empty(GRID ** 3, dtype=torch.int32, device=dev)
        ctx.lib.c3h_get_grid(ctx.h, c3hlac.ptr(words), 1)
        grids.append(words)
        # more frames from the same scene: shifted along x by non-subdivision steps
        for k in range(1, per_scene):
            if len(grids) < nf:
                grids.append(torch.roll(words.view(GRID, GRID, GRID), shifts=37 * k, dims=2).reshape(-1).contiguous())
    grids = grids[:nf]
    torch.cuda.synchronize(dev)

    axis_t, var, axis_q = synth.random_bases(VARIANT, D, M, R, seed=synth.BASE_SEED)
    ctx.search_setup(axis_t, var, axis_q)
    ctx.set_rank(RANK)
    H = (GRID // SUBDIV + (GRID % SUBDIV > 0)) ** 3
    P = (round(np.ceil(GRID / SUBDIV)) - BOX[0] + 1) ** 3
    dets = torch.zeros((args.steps + args.warmup, M * RANK * 3), dtype=torch.int64, device=dev)

    gptr = np.array([grids[i % nf].data_ptr() for i in range(args.warmup + args.steps)], np.uint64)
    rec = dets.element_size() * dets.shape[1]

    def run(first, count):  # `count` steps = frames first .. first+count-1, one C-ABI call
        ctx.run_frames(gptr[first:first + count], (GRID,) * 3, (0, 0, 0), LEAF, VARIANT, THR, SUBDIV,
                       BOX, EXIST_THR, True, dets.data_ptr() + first * rec)

    # allocation prime (untimed, before the W warmup steps): the pipeline rotates batches
    # over PIPE_DEPTH contexts whose per-frame buffers are sized on first use; a warmup of
    # fewer than PIPE_DEPTH x BATCH frames would leave a context to be allocated (hipMalloc)
    # inside the timed region
    if args.warmup + args.steps >= PIPE_DEPTH * BATCH:
        run(0, PIPE_DEPTH * BATCH)
        torch.cuda.synchronize(dev)
    if args.warmup:
        run(0, args.warmup)
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    # HIP events bracket every pipeline tick inside the timed region (one fused launch per
    # tick: occupancy of batch t | tile of t-1 | compress+gate of t-2 | score of t-3)
    ctx.timing(c3hlac.timing_mask("pipeline"))
    ctx.kernel_times(reset=True)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    run(args.warmup, args.steps)
    if dist:  # gather every rank's detections (one RCCL all_gather) inside the timed region
        from c3hlac.dist import gather_records
        gather_records(dets[args.warmup:], args.steps * world, rank, world, dist)
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    kt = ctx.kernel_times(reset=True)
    ctx.timing(False)
    # per-stage breakdown: a separate, untimed pass on the lanes path (separate launches
    # per stage, events around each)
    n_sep = min(args.steps, 48)
    ctx.set_pipeline(False)
    ctx.timing(True)
    run(args.warmup, n_sep)
    kt_all = ctx.kernel_times(reset=True)
    ctx.timing(False)
    ctx.set_pipeline(True)
    if dist:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    # sanity: every frame produced a detection for every model
    d = dets[args.warmup:].view(args.steps, M * RANK, 3).cpu().numpy()
    scores = d[:, :, 0].view(np.float64)
    assert np.all(scores > 0), "no detection"

    voxels = GRID ** 3 * args.steps * world
    search_ms = kt_all["compress"][0] + kt_all["score"][0] + kt_all["replay"][0]
    # the dominant kernel is the tick: every launch streams one batch's grids and carries
    # the other stages of three more batches; ticks = batches + pipeline fill/drain
    tick_ms, tick_frames = kt["pipeline"]
    n_ticks = -(-args.steps // BATCH) + PIPE_DEPTH - 1
    tick_avg_s = tick_ms / n_ticks / 1e3
    alg_bytes = algorithmic_bytes_c3(GRID, H, VARIANT) * tick_frames / n_ticks
    achieved = alg_bytes / tick_avg_s / 1e9
    result = {
        "metric": "Mvoxels/s C3-HLAC + detections/s sliding-box, 256^3 grid",
        "value": voxels / elapsed / 1e6,
        "unit": "Mvoxels/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8 x u8 -> u32 (exact integer C3-HLAC), f32 search",
        "data": "synthetic Kinect-style RGB-D frames (ray-cast room, 1M rays/frame, seeded splitmix64)",
        "config": {
            "workload": "BASELINE configs[2]: 256^3 grid, C3-HLAC-117 subdivision 10 (17,576 subdivisions), "
                        "compress 117->100, 10 models x r=20, box 2x2x2 (15,625 positions), rank 1",
            "grid": GRID, "leaf": LEAF, "variant": VARIANT, "subdivision": SUBDIV, "D": D, "models": M,
            "r": R, "box": list(BOX), "positions": int(P), "frames_resident": nf,
            "parallelism": "frame-sharded x%d (no data-path collective), RCCL all_gather of detections" % world,
            "frames_per_launch": BATCH, "schedule": "software pipeline, %d batches in flight per GPU" % PIPE_DEPTH,
        },
        "detections_per_s": P * M * args.steps * world / elapsed,
        "detections_per_s_search_kernels": (P * M * max(kt_all["score"][1], 1) / (search_ms / 1e3)) if search_ms else None,
        "frames_per_s": args.steps * world / elapsed,
        "kernel_ms_avg": {k: (v[0] / v[1] if v[1] else None) for k, v in kt_all.items()},
        "kernel_ms_avg_note": "separate pass of %d steps on the lanes path (stand-alone launches per stage, "
                              "events around every stage; %d lanes x %d frames per launch, so stages overlap; times "
                              "are per frame); c3hlac = occupancy pass + tile kernel; score = compress(non-empty "
                              "rows)+gate launch + score launch with the fused rank-1 replay" % (n_sep, LANES, BATCH),
        "voxelize_mpoints_per_s": n_points / (sum(t_vox_ms) / 1e3) / 1e6 if sum(t_vox_ms) else None,
        "roofline": {
            "kernel": "c3h_tick_kernel (pipeline tick: occupancy stream of one batch + C3 tile pass, compress+gate "
                      "and scoring of the three previous batches)",
            "bound": "hbm",
            "achieved": achieved,
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS,
            "traffic": pmc_traffic(tick_frames / n_ticks),
            "algorithmic_bytes_per_launch": alg_bytes,
            "algorithmic_bytes_per_frame": algorithmic_bytes_c3(GRID, H, VARIANT),
            "frames_per_launch": BATCH,
            "launches": n_ticks,
            "avg_launch_ms": tick_avg_s * 1e3,
        },
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline(frame_pts[0], args.cpu_seconds)
    if rank == 0:
        print(json.dumps(result))
    ctx.close()
    if dist:
        dist.destroy_process_group()


def pmc_traffic(frames_per_tick):
    """HBM bytes per tick launch (the bench's average frames per tick, fill/drain
    included, like `achieved`) from the committed rocprofv3 --pmc summary of this build
    (scripts_pmc.sh -> tools_pmc_summary.py): FETCH_SIZE x2 (gfx950 correction) +
    WRITE_SIZE of c3h_tick_kernel, per frame through the pipeline.  PMC needs its own profiler pass, so
    it cannot be collected inside the timed run; None when no summary is committed."""
    f = ROOT / "profiles" / "pmc_c3_traffic.json"
    if not f.exists():
        return None
    per_frame = json.load(open(f)).get("tick_hbm_bytes_per_frame")
    return per_frame * frames_per_tick if per_frame is not None else None


def cpu_baseline(pts, seconds):
    """The oracle (single-threaded C restatement of the reference, -O2) on the same
    workload: C3-HLAC-117 + exist + setData/search of the 10 models, repeated on frame 0
    until `seconds` elapse (at least once)."""
    import pyoracle as po
    from c3hlac import synth
    g, layout, cloud = po.voxelize(pts, LEAF)
    axis_t, var, axis_q = synth.random_bases(VARIANT, D, M, R, seed=synth.BASE_SEED)
    ap = synth.whiten(axis_t, var)
    n, t_c3, t_s = 0, 0.0, 0.0
    t_start = time.perf_counter()
    while n == 0 or time.perf_counter() - t_start < seconds:
        t0 = time.perf_counter()
        f117, sb, _ = po.c3hlac(g, layout, cloud, 117, THR, LEAF, SUBDIV)
        ex = po.exist(f117)  # f[0], f[1] are the same 1/255-normalised sums in 117 and 981
        t1 = time.perf_counter()
        po.search(sb, f117, ex, ap, axis_q, BOX, RANK, EXIST_THR)
        t2 = time.perf_counter()
        t_c3 += t1 - t0
        t_s += t2 - t1
        n += 1
    tot = t_c3 + t_s
    return {
        "value": GRID ** 3 * n / tot / 1e6,
        "unit": "Mvoxels/s",
        "cores": 1,
        "kind": "port",
        "sample": "%d frame(s) of the same 256^3 workload (C3-HLAC-117 + exist gate + 10-model search), "
                  "C3 %.3f s/frame, search %.3f s/frame, host %s" % (n, t_c3 / n, t_s / n, os.uname().machine),
    }


if __name__ == "__main__":
    main()
