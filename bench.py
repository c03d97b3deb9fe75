"""Benchmark of the C3-HLAC colour-voxel recognition hot path on MI355X.

Workload (BASELINE.json configs[2], the 256^3 configuration its metric is quoted on):
C3-HLAC-117 over device-resident 256^3 packed colour/occupancy grids (subdivision 10 ->
17,576 subdivisions) + setData compression 117 -> 100 + sliding-box search of 10 models x
r=20 over 15,625 box positions (box 2x2x2 subdivisions, rank 1, exist threshold 100).
Frames are Kinect-style synthetic RGB-D scenes (1M rays each), voxelised on the GPU
before the timed region; BATCH + 8 distinct grids (4.8 GB, far above the 256 MB Infinity
Cache) stay resident and are cycled, so every frame of a step reads its own grid from HBM.

One step = one batch of BATCH frames through the software pipeline (c3h_stream_frames):
one tick launch in which the new batch's occupancy stream runs beside the tile, compress
+ gate and scoring stages of the three batches before it.  The W warmup steps fill the
pipeline, so each of the K timed steps completes exactly one batch (steady state, the
detect_object.cpp callback loop with frames arriving continuously); the pipeline is
drained after the timer stops.  value = voxels of the batches completed inside the timed
region / its wall time (W < 3 leaves fill ticks inside it, and fewer completed batches).

Multi-GPU (torch.distributed.run, one process per GPU): independent frames are sharded
over ranks with no data-path collective (weak scaling); the detections of the completed
frames are gathered to rank 0 with one all_gather over RCCL inside the timed region.

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
LANES = 3  # batches in flight per GPU on the lanes path (stage breakdown pass only)
BATCH = 64  # frames per step (c3h_set_batch): the tick's latency-bound roles need many frames
            # in flight (12.8 us/frame at 32 vs 14.1 at 16, 17.9 at 8, profiles/r1/v8; 64 beats
            # 32 by 2.4 %, profiles/r1/abbatch_32_vs_64.log)
PIPE_DEPTH = 4  # pipeline ticks a batch spends in flight (occupancy | tile | compress+gate | score)
THR = (147, 146, 148)
N_RAYS = 1_000_000
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table (spec)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=60, help="timed steps (one batch of %d frames each)" % BATCH)
    ap.add_argument("--warmup", type=int, default=8)
    ap.add_argument("--batch", type=int, default=BATCH)
    ap.add_argument("--frames", type=int, default=0,
                    help="resident grids (0: batch + 8; every frame of a tick reads its own grid)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--point-frames", type=int, default=512,
                    help="configs[3] points-in pass: frames over all ranks (0: skip)")
    ap.add_argument("--host-point-frames", type=int, default=128,
                    help="frames of the H2D-inclusive points-in pass per rank (pinned host memory)")
    ap.add_argument("--single-frames", type=int, default=40,
                    help="per-callback latency pass: 1M-point host clouds through voxelize/extract/search "
                         "one at a time (0: skip; N = 1 only)")
    return ap.parse_args()


def launch_plan(gpus, env, n_devices, argv, port=None):
    """What `python bench.py --gpus N` does before anything touches the GPU.

    Returns ("inline", None) when this process runs the bench itself (N = 1, or it is
    already one rank of a torch.distributed launch: WORLD_SIZE set), ("spawn", cmd) when it
    must start N ranks as a child `torch.distributed.run` (the parent only waits and relays
    the child's JSON line and exit code -- it never execs and never initialises HIP), and
    ("error", message) when the request cannot be met (fewer visible devices than N: never
    a silent one-rank run under an N-GPU label).  C3H_BENCH_REHEARSAL=1 allows N ranks on
    fewer devices (all on device 0, collectives staged over gloo; not a measurement)."""
    if gpus < 1:
        return "error", "--gpus must be >= 1 (got %d)" % gpus
    if "WORLD_SIZE" in env:
        world = int(env["WORLD_SIZE"])
        if world != gpus:
            return "error", "launched with WORLD_SIZE=%d but --gpus %d" % (world, gpus)
        return "inline", None
    if gpus == 1:
        return "inline", None
    rehearsal = env.get("C3H_BENCH_REHEARSAL") == "1"
    if n_devices < gpus and not rehearsal:
        return "error", "--gpus %d requested but only %d HIP device(s) are visible" % (gpus, n_devices)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(gpus),
           "--master-addr", "127.0.0.1", "--master-port", str(port or 29500),
           str(ROOT / "bench.py")] + list(argv)
    return "spawn", cmd


def relay(cmd, env, out=None, err=None):
    """Run the launcher child; its stdout lines that are the bench's JSON object go to our
    stdout (exactly one line from rank 0), anything else the ranks or their libraries print
    there (gloo's connection banner, ...) goes to stderr.  Returns the child's exit code."""
    import subprocess
    out = out or sys.stdout
    err = err or sys.stderr
    p = subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE, text=True, bufsize=1)
    for line in p.stdout:
        s = line.strip()
        is_result = False
        if s.startswith("{"):
            try:
                is_result = "metric" in json.loads(s)
            except ValueError:
                pass
        (out if is_result else err).write(line if line.endswith("\n") else line + "\n")
        (out if is_result else err).flush()
    return p.wait()


def child_env(env):
    out = dict(env)
    out["C3H_BENCH_CHILD"] = "1"
    out.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC only on this pool's driver
    return out


def _free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _visible_devices():
    """HIP devices visible to this process, counted without initialising HIP
    (torch.cuda.device_count() does not create a device context on this image)."""
    import torch
    return torch.cuda.device_count()


def algorithmic_bytes_c3(G, H, F):
    """4 B/voxel packed-grid read + the feature rows + exist written."""
    return G ** 3 * 4 + H * F * 4 + H * 4


def scene_points(synth, rank, s):
    """the 1M points of make_grids' scene s (grids 4 s .. 4 s + 3)"""
    return synth.kinect_scene(N_RAYS, grid=GRID, leaf=LEAF, seed=synth.BASE_SEED + 1000 * rank + s)


def make_grids(ctx, dev, nf, rank, synth, c3hlac, torch):
    """nf resident 256^3 grids: scenes voxelised on the GPU, plus x-shifted copies."""
    grids, t_vox_ms, n_points = [], [], 0
    per_scene = 4  # the scene and three x-shifts of it (distinct buffers)
    for s in range(-(-nf // per_scene)):
        pts = scene_points(synth, rank, s)
        d_pts = torch.from_numpy(pts).to(dev)
        torch.cuda.current_stream(dev).synchronize()
        # untimed first call per scene: a scene with more points than any before it grows the
        # voxeliser's buffers (hipMalloc); the timed call is the steady-state per-frame cost
        ctx.voxelize(d_pts, LEAF)
        ctx.timing(True)
        gi = ctx.voxelize(d_pts, LEAF)
        t_vox_ms.append(ctx.kernel_times(reset=True)["voxelize"][0])
        ctx.timing(False)
        n_points += pts.shape[0]
        assert list(gi.div_b) == [GRID] * 3, list(gi.div_b)
        words = torch.empty(GRID ** 3, dtype=torch.int32, device=dev)
        ctx.lib.c3h_get_grid(ctx.h, c3hlac.ptr(words), 1)  # synchronous
        grids.append(words)
        for k in range(1, per_scene):  # shifted along x by non-subdivision steps
            if len(grids) < nf:
                grids.append(torch.roll(words.view(GRID, GRID, GRID), shifts=37 * k, dims=2).reshape(-1).contiguous())
    torch.cuda.synchronize(dev)
    return grids[:nf], t_vox_ms, n_points


class _StagedGloo:
    """Rehearsal of the multi-GPU path on a one-GPU box (C3H_BENCH_REHEARSAL=1): every rank
    runs on device 0 and the collectives go over gloo, which has no GPU all_gather, so they
    are staged through host memory.  Not a measurement: the driver's N > 1 runs use RCCL."""

    def __init__(self, dist):
        self.d = dist
        self.ReduceOp = dist.ReduceOp

    def all_gather(self, parts, buf):
        host = [torch_mod().empty_like(buf, device="cpu") for _ in parts]
        self.d.all_gather(host, buf.cpu())
        for p, h in zip(parts, host):
            p.copy_(h)

    def all_reduce(self, t, op=None):
        h = t.cpu()
        self.d.all_reduce(h, op=op)
        t.copy_(h)

    def barrier(self):
        self.d.barrier()

    def get_world_size(self):
        return self.d.get_world_size()

    def destroy_process_group(self):
        self.d.destroy_process_group()


def torch_mod():
    import torch
    return torch


def main():
    args = parse()
    n_dev = _visible_devices() if args.gpus > 1 and "WORLD_SIZE" not in os.environ else 0
    action, what = launch_plan(args.gpus, os.environ, n_dev, sys.argv[1:], port=_free_port())
    if action == "error":
        print("bench.py: " + what, file=sys.stderr)
        sys.exit(2)
    if action == "spawn":  # child launcher; this process never touches the GPU
        sys.exit(relay(what, child_env(os.environ)))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    rehearsal = os.environ.get("C3H_BENCH_REHEARSAL") == "1" and world > 1
    if rehearsal:
        local = 0
    import torch
    dist = None
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        import torch.distributed as dist
        if rehearsal:
            dist.init_process_group("gloo")
            dist = _StagedGloo(dist)
        else:
            dist.init_process_group("nccl", device_id=dev)
        assert dist.get_world_size() == args.gpus == world, (dist.get_world_size(), args.gpus, world)

    import c3hlac
    from c3hlac import synth

    B = args.batch
    # the library and torch share one non-default stream: the RCCL gather and every torch
    # read of the detections are stream-ordered after the ticks that write them
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    ctx = c3hlac.Context(local)
    ctx.set_stream(stream.cuda_stream)
    ctx.set_lanes(LANES)
    ctx.set_batch(B)
    ctx.set_pipeline(True)

    nf = args.frames if args.frames > 0 else B + 8
    grids, t_vox_ms, n_points = make_grids(ctx, dev, nf, rank, synth, c3hlac, torch)

    axis_t, var, axis_q = synth.random_bases(VARIANT, D, M, R, seed=synth.BASE_SEED)
    ctx.search_setup(axis_t, var, axis_q)
    ctx.set_rank(RANK)
    H = (GRID // SUBDIV + (GRID % SUBDIV > 0)) ** 3
    P = (round(np.ceil(GRID / SUBDIV)) - BOX[0] + 1) ** 3
    n_total = (args.warmup + args.steps) * B
    dets = torch.zeros((n_total, M * RANK * 3), dtype=torch.int64, device=dev)
    rec = dets.element_size() * dets.shape[1]
    gptr = np.array([grids[i % nf].data_ptr() for i in range(n_total)], np.uint64)

    def push(first_step, nsteps, stream_mode=True):  # steps first .. first+nsteps-1, one C-ABI call
        f0 = first_step * B
        ctx.run_frames(gptr[f0:f0 + nsteps * B], (GRID,) * 3, (0, 0, 0), LEAF, VARIANT, THR, SUBDIV,
                       BOX, EXIST_THR, True, dets.data_ptr() + f0 * rec, stream=stream_mode)

    # allocation prime (untimed): the pipeline rotates batches over PIPE_DEPTH buffer sets
    # whose per-frame buffers are sized on first use; run_frames drains, so all four sets
    # are allocated and idle before the warmup steps start the stream
    prime = np.array([grids[i % nf].data_ptr() for i in range(PIPE_DEPTH * B)], np.uint64)
    prime_out = torch.zeros((PIPE_DEPTH * B, M * RANK * 3), dtype=torch.int64, device=dev)
    ctx.run_frames(prime, (GRID,) * 3, (0, 0, 0), LEAF, VARIANT, THR, SUBDIV, BOX, EXIST_THR, True,
                   prime_out.data_ptr())
    if args.warmup:
        push(0, args.warmup)  # fills the pipeline: its last 3 batches stay in flight
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    # HIP events bracket every pipeline tick inside the timed region (one fused launch per
    # tick: occupancy of batch t | tile of t-1 | compress+gate of t-2 | score of t-3)
    ctx.timing(c3hlac.timing_mask("pipeline"))
    ctx.kernel_times(reset=True)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    push(args.warmup, args.steps)
    # batches whose scoring ran inside the timed region
    done_first = max(0, args.warmup - (PIPE_DEPTH - 1))
    done_last = args.warmup + args.steps - (PIPE_DEPTH - 1)
    n_done = max(0, done_last - done_first)
    gather_ev = None
    if dist:  # gather every rank's completed detections (one RCCL all_gather) inside the timed region
        from c3hlac.dist import gather_records
        gather_ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
        gather_ev[0].record(stream)  # the library's stream = torch's current stream
        gather_records(dets[done_first * B:done_last * B], n_done * B * world, rank, world, dist)
        gather_ev[1].record(stream)
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    kt = ctx.kernel_times(reset=True)
    ctx.timing(False)
    ctx.stream_flush()  # drain (untimed): the last batches' detections
    torch.cuda.synchronize(dev)
    # per-stage breakdown: a separate, untimed pass on the lanes path (separate launches
    # per stage, events around each)
    n_sep = min(args.steps * B, 48)
    ctx.set_pipeline(False)
    ctx.timing(True)
    sep_out = torch.zeros((n_sep, M * RANK * 3), dtype=torch.int64, device=dev)
    ctx.run_frames(gptr[:n_sep], (GRID,) * 3, (0, 0, 0), LEAF, VARIANT, THR, SUBDIV, BOX, EXIST_THR, True,
                   sep_out.data_ptr())
    kt_all = ctx.kernel_times(reset=True)
    ctx.timing(False)
    ctx.set_pipeline(True)
    torch.cuda.synchronize(dev)
    if dist:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    # every frame (warmup, timed and drained) produced a detection for every model, and the
    # lanes path agrees with the pipeline on the frames both ran
    d = dets.view(n_total, M * RANK, 3).cpu().numpy()
    scores = d[:, :, 0].view(np.float64)
    # (diagnostics builds can run a subset of the tick's roles: C3H_TICK_ROLES, no checks)
    roles_subset = os.environ.get("C3H_TICK_ROLES") not in (None, "", "15")
    assert roles_subset or np.all(scores > 0), "no detection"
    assert roles_subset or np.array_equal(sep_out.cpu().numpy(), dets[:n_sep].cpu().numpy()), "pipeline != lanes"

    frames_done = n_done * B
    voxels = GRID ** 3 * frames_done * world
    search_ms = kt_all["compress"][0] + kt_all["score"][0] + kt_all["replay"][0]
    # the dominant kernel is the tick: in steady state every launch streams one batch's
    # grids and carries the other stages of the three batches before it
    tick_ms, tick_frames = kt["pipeline"]
    n_ticks = args.steps
    tick_avg_s = tick_ms / n_ticks / 1e3
    alg_bytes = algorithmic_bytes_c3(GRID, H, VARIANT) * B
    achieved = alg_bytes / tick_avg_s / 1e9
    # the bytes the tick must move: the grid stream plus the rows of the non-empty
    # subdivisions only (an empty subdivision keeps exist 0 and every reader gates on it)
    # and exist, from the frames of the timed region (the context holds the last one)
    nonempty = int((ctx.exist() > 0).sum())
    # positions of the last frame that passed the exist gate (scored; the rest are -1)
    try:
        scored = int((ctx.scores().reshape(M, -1)[0] >= 0).sum())
    except (c3hlac.C3HError, ValueError):
        scored = 0
    min_bytes = (GRID ** 3 * 4 + nonempty * VARIANT * 4 + H * 4) * B
    achieved_min = min_bytes / tick_avg_s / 1e9
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
            "step": "one batch of %d frames = one pipeline tick (steady state: the warmup steps fill the "
                    "pipeline, it is drained after the timer)" % B,
            "frames_per_step": B, "frames_completed_timed": frames_done * world,
            "frames_per_rank": frames_done,
            "schedule": "software pipeline, %d batches in flight per GPU" % PIPE_DEPTH,
        },
        "distributed": {
            "world_size": dist.get_world_size() if dist else 1,
            "backend": ("gloo (rehearsal: every rank on device 0, collectives staged through host memory; "
                        "not a measurement)" if rehearsal else "nccl (RCCL)") if dist else None,
            "launch": ("self-launched torch.distributed.run child" if os.environ.get("C3H_BENCH_CHILD") == "1"
                       else "torch.distributed.run") if dist else "single process",
            "gather_ms_rank0": gather_ev[0].elapsed_time(gather_ev[1]) if gather_ev else None,
            "gather_note": "HIP events on the library's stream around the all_gather of the timed region's "
                           "detection records (starts when the rank's last tick completes)",
        },
        "detections_per_s": P * M * frames_done * world / elapsed,
        "detections_note": "detections_per_s counts every box position x model (SURVEY 8(d)); only the positions "
                           "passing the exist gate are scored: scored_detections_per_s (gate-passing positions of "
                           "the last frame, %d of %d, x models x frames/s)" % (scored, P),
        "scored_detections_per_s": (scored * M * frames_done * world / elapsed) if scored else None,
        "detections_per_s_search_kernels": (P * M * max(kt_all["score"][1], 1) / (search_ms / 1e3)) if search_ms else None,
        "frames_per_s": frames_done * world / elapsed,
        "kernel_ms_avg": {k: (v[0] / v[1] if v[1] else None) for k, v in kt_all.items()},
        "kernel_ms_avg_note": "separate pass of %d frames on the lanes path (stand-alone launches per stage, "
                              "events around every stage; %d lanes x %d frames per launch, so stages overlap; times "
                              "are per frame); c3hlac = occupancy pass + tile kernel; score = compress(non-empty "
                              "rows)+gate launch + score launch with the fused rank-1 replay" % (n_sep, LANES, B),
        "voxelize_mpoints_per_s": n_points / (sum(t_vox_ms) / 1e3) / 1e6 if sum(t_vox_ms) else None,
        "voxelize_note": "c3h_voxelize of each 1M-ray scene, HIP events around all of its kernels (an untimed "
                         "call on the scene first sizes the context's buffers for its point count)",
        "roofline": {
            "kernel": "c3h_tick_kernel (pipeline tick: occupancy stream of one batch + C3 tile pass, compress+gate "
                      "and scoring of the three previous batches)",
            "bound": "hbm",
            "achieved": achieved,
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS,
            "traffic": pmc_traffic(B),
            "algorithmic_bytes_per_launch": alg_bytes,
            "algorithmic_bytes_per_frame": algorithmic_bytes_c3(GRID, H, VARIANT),
            "frames_per_launch": B,
            "launches": n_ticks,
            "avg_launch_ms": tick_avg_s * 1e3,
            "achieved_min_bytes": achieved_min,
            "frac_min_bytes": achieved_min / HBM_PEAK_GBS,
            "min_bytes_per_frame": min_bytes // B,
            "min_bytes_note": "the same tick time on the bytes the tick must move: the 4 B/voxel grid stream, "
                              "feature rows of the %d non-empty subdivisions only (of %d) and exist; 'achieved' / "
                              "'frac' use SURVEY 8(d)'s algorithmic bytes, which charge a row to every "
                              "subdivision" % (nonempty, H),
        },
    }
    if args.point_frames > 0:
        result["points_in"] = points_pass(ctx, dev, rank, world, dist, torch, synth, c3hlac, args.point_frames,
                                          args.host_point_frames)
        if world == 1:
            result["points_in_real_views"] = real_views_pass(ctx, dev, torch, synth, c3hlac)
    if world == 1 and args.single_frames > 0:
        result["single_frame"] = single_frame_pass(local, torch, synth, c3hlac, rank, args.single_frames)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        f0 = args.warmup * B  # the first timed frame: the oracle re-computes it as it is timed
        rec0 = d[f0]
        result["cpu_baseline"] = cpu_baseline(grids[f0 % nf].cpu().numpy().view(np.uint32), rec0, args.cpu_seconds,
                                              scene_points(synth, rank, (f0 % nf) // 4), grids[(f0 % nf) // 4 * 4])
        if "points_in" in result:
            result["points_in"]["cpu_baseline"] = cpu_baseline_points(synth, args.cpu_seconds)
            result["points_in"]["cpu_baseline_parallel"] = cpu_baseline_points_parallel(args.cpu_seconds)
    if rank == 0:
        from c3hlac import _capi
        result["build"] = _capi.build_provenance()
        print(json.dumps(result))
    ctx.close()
    if dist:
        dist.destroy_process_group()


P_GRID, P_LEAF, P_VARIANT, P_M = 128, 0.02, 981, 1  # BASELINE configs[3] (= configs[1] per frame)


def points_pass(ctx, dev, rank, world, dist, torch, synth, c3hlac, n_total, n_host):
    """BASELINE configs[3]: n_total independent 1M-point frames (128^3, C3-HLAC-981 S=10,
    compress 981->100, 1 model x r=20, box 2x2x2, rank 1) sharded round-robin over the ranks,
    each rank's shard through c3h_run_point_frames (voxelised on the GPU, no per-frame host
    round trip, the software-pipelined tick), then one RCCL all_gather of the detections.
    Timed twice: points already in HBM, and points in pinned host memory (H2D included,
    n_host frames per rank).  Frames: 16 ray-cast scenes, each under colour masks and x
    shifts by whole cells (distinct clouds, distinct grids and min_b)."""
    nb = 16
    base = [torch.from_numpy(synth.kinect_scene(N_RAYS, grid=P_GRID, leaf=P_LEAF,
                                                seed=synth.BASE_SEED + 7000 + s)).to(dev) for s in range(nb)]

    def frame(i):
        t = base[i % nb].clone()
        k = i // nb
        t[:, 3] = (t[:, 3].view(torch.int32) ^ ((k * 0x2F1D37) & 0xFFFFFF)).view(torch.float32)
        t[:, 0] = (t[:, 0].double() + k * P_LEAF).float()
        return t

    mine = list(range(rank, n_total, world))
    frames = frame_list = [frame(i) for i in mine]
    axis_t, var, axis_q = synth.random_bases(P_VARIANT, D, P_M, R, seed=synth.BASE_SEED + 31)
    ctx.search_setup(axis_t, var, axis_q)
    ctx.set_rank(1)
    out = torch.zeros((max(len(mine), 1), 3 * P_M), dtype=torch.int64, device=dev)
    canvas = (P_GRID,) * 3
    args = (P_LEAF, canvas, P_VARIANT, THR, SUBDIV, BOX, EXIST_THR, True)
    ctx.run_point_frames(frames[:4 * BATCH], *args[:7], True, out)  # untimed: sizes the buffers
    torch.cuda.synchronize(dev)

    def timed(fr, d_out, gather, batch=None):
        # frames per batch: the binding's choice for the call's frame count (32 from 256
        # frames up, else 64; Context.point_batch), or the one given
        ctx.set_batch(batch or ctx.point_batch(len(fr)))
        if dist:
            dist.barrier()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        _, info = ctx.run_point_frames(fr, *args[:7], True, d_out)
        if gather and dist:
            from c3hlac.dist import gather_records
            gather_records(d_out[:len(fr)], n_total, rank, world, dist)
        torch.cuda.synchronize(dev)
        el = time.perf_counter() - t0
        if dist:
            t = torch.tensor([el], dtype=torch.float64, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            el = float(t.item())
        return el, info

    # the frames' pointer array is built and checked once, outside the timed region (a C++
    # caller holds it; the per-frame Python checks cost ~1.5 ms per 512-frame call).  The
    # timed call runs without HIP events around the launches (they cost ~3 % here); a second
    # call with events gives the voxeliser's per-frame time
    frames = ctx.prepare_point_frames(frames)
    ctx.set_batch(ctx.point_batch(len(mine)))
    ctx.run_point_frames(frames, *args[:7], True, out)  # untimed: one whole call at the timed batch size
    torch.cuda.synchronize(dev)
    el_dev, info = timed(frames, out, True)
    ev_out = torch.zeros_like(out)
    ctx.timing(c3hlac.timing_mask("voxelize", "pipeline"))
    ctx.kernel_times(reset=True)
    timed(frames, ev_out, False)
    kt = ctx.kernel_times(reset=True)
    ctx.timing(False)
    batched = int((info["status"] == 0).sum())
    ok = bool((out[:len(mine)].cpu().numpy()[:, 0].view(np.float64) > 0).all())
    res = {
        "frames": n_total,
        "frames_per_s_from_points": n_total / el_dev,
        "batch": ctx.point_batch(len(mine)),
        "note": "configs[3]: %d independent 1M-point frames (128^3, C3-HLAC-981 S=10, 981->100, 1 model x r=20, "
                "box 2x2x2, rank 1) sharded over %d GPU(s), c3h_run_point_frames per rank (GPU voxeliser + "
                "pipelined tick, one host sync per call) + RCCL all_gather; points resident in HBM" % (n_total, world),
        "ms_per_call": el_dev * 1e3,
        "frames_batched": batched * world,
        "all_frames_detected": ok,
        "events_run_equal": bool(torch.equal(ev_out, out)),
        "voxelize_batched_us_per_frame": (kt["voxelize"][0] / kt["voxelize"][1] * 1e3) if kt["voxelize"][1] else None,
        "voxelize_batched_gpoints_per_s": (N_RAYS * kt["voxelize"][1] / (kt["voxelize"][0] / 1e3) / 1e9)
        if kt["voxelize"][0] else None,
    }
    if world == 1:
        # the shard one rank gets at N = 2, 4, 8 (frames 0, N, 2N, ... of this run), timed the
        # same way on this GPU: the 1 -> 8 strong-scaling shape without an 8-GPU node
        # (VERDICT r5 item 2); records must equal the full run's for the same frames
        shard = {}
        want = out[:len(mine)].cpu()
        for n_w in (2, 4, 8):
            sel = list(range(0, len(frames), n_w))
            s_out = torch.zeros((len(sel), 3 * P_M), dtype=torch.int64, device=dev)
            s_frames = ctx.prepare_point_frames([frame_list[i] for i in sel])
            best = None
            for _ in range(3):
                el_s, _ = timed(s_frames, s_out, False)
                best = el_s if best is None else min(best, el_s)
            shard[str(len(sel))] = {"frames_per_s": len(sel) / best, "ms_per_call": best * 1e3,
                                    "batch": ctx.point_batch(len(sel)),
                                    "records_equal_full_run": bool(torch.equal(s_out.cpu(), want[sel]))}
        # the full run again at the shards' batch of 64: the fill cost of a small shard alone,
        # without the full run's gain from its smaller batches
        b64_out = torch.zeros_like(out)
        el_64, _ = timed(frames, b64_out, False, batch=64)
        res["shard_frames_per_s"] = {k: v["frames_per_s"] for k, v in shard.items()}
        res["shard_over_full"] = {k: v["frames_per_s"] / res["frames_per_s_from_points"] for k, v in shard.items()}
        res["frames_per_s_from_points_b64"] = len(frames) / el_64
        res["b64_equals"] = bool(torch.equal(b64_out, out))
        res["shard_over_full_b64"] = {k: v["frames_per_s"] * el_64 / len(frames) for k, v in shard.items()}
        res["shard"] = shard
        res["shard_note"] = ("rank 0's shard of %d frames at N = 2, 4, 8 (every N-th frame), one c3h_run_point_frames "
                             "call each on this GPU, best of 3, at Context.point_batch's batch (32 from 256 frames up, "
                             "else 64); shard_over_full: per-frame rate against the %d-frame run; shard_over_full_b64: "
                             "against the %d-frame run at 64 frames per batch (the fill cost alone)"
                             % (len(frames), len(frames), len(frames)))
    if n_host > 0:  # H2D included: the frames start in pinned host memory
        hf = [f.cpu().pin_memory() for f in frame_list[:n_host]]
        hout = torch.zeros((len(hf), 3 * P_M), dtype=torch.int64, device=dev)
        el_h, _ = timed(ctx.prepare_point_frames([h.numpy() for h in hf]), hout, False)
        res["frames_per_s_from_points_h2d"] = len(hf) * world / el_h
        res["h2d_note"] = "%d frames per GPU from pinned host memory (16 MB each), H2D inside the timed call" % len(hf)
        res["h2d_equals_device"] = bool(torch.equal(hout, out[:len(hf)]))
    return res


def single_frame_pass(local, torch, synth, c3hlac, rank, n_frames, n_scenes=4):
    """The drop-in per-callback latency (detect_object.cpp:139-186, queue 1): one 1M-point
    host cloud at a time (pageable numpy memory, as fromROSMsg leaves it) through
    c3h_voxelize -> c3h_extract -> c3h_search at configs[2]'s shape (256^3, C3-HLAC-117 S=10,
    117 -> 100, 10 models x r = 20, box 2^3, rank 1), detections back on the host.  Its own
    context on its own stream.  Two timed loops over the same frames:
    Each frame's lists start empty (c3h_clean_max, the callback's cleanData, in the C3 phase
    as detect_object.cpp:168-170 times it).
    - end_to_end: the calls back to back, exactly what the callback does (the host
      syncs are the API's own: voxelize returns the grid info, search the lists);
    - phases: the same with a device sync after extract, so the wall clock splits as the
      reference prints it (detect_object.cpp:182-186), plus the HIP-event kernel time of
      each phase (voxelize = its kernels, not the H2D copy)."""
    ctx = c3hlac.Context(local)
    try:
        scenes = [scene_points(synth, rank, s) for s in range(n_scenes)]
        axis_t, var, axis_q = synth.random_bases(VARIANT, D, M, R, seed=synth.BASE_SEED)
        ctx.search_setup(axis_t, var, axis_q)
        ctx.set_rank(RANK)

        def frame(i, sync_phases):
            t0 = time.perf_counter()
            ctx.voxelize(scenes[i % n_scenes], LEAF)
            t1 = time.perf_counter()
            ctx.clean_max()  # search_obj.cleanData() (detect_object.cpp:169): each frame's lists start empty
            ctx.extract(VARIANT, THR, SUBDIV)
            if sync_phases:
                ctx.synchronize()
            t2 = time.perf_counter()
            lists, _ = ctx.search(BOX, EXIST_THR)
            t3 = time.perf_counter()
            assert float(lists[0, 0]["score"]) > 0, "no detection"
            return t1 - t0, t2 - t1, t3 - t2

        for i in range(2 * n_scenes):  # untimed: buffers sized for the scenes
            frame(i, False)
        e2e = [sum(frame(i, False)) for i in range(n_frames)]
        ctx.timing(c3hlac.timing_mask("voxelize", "c3hlac", "compress", "score", "replay"))
        ctx.kernel_times(reset=True)
        ph = np.array([frame(i, True) for i in range(n_frames)])
        kt = ctx.kernel_times(reset=True)
        ctx.timing(False)
    finally:
        ctx.close()
    native = native_single_frame(scenes, axis_t, var, axis_q, n_frames)
    med = lambda a: float(np.median(a)) * 1e3  # noqa: E731
    kms = lambda *names: sum(kt[n][0] for n in names) / n_frames  # noqa: E731
    return {
        "native": native,
        "ms_per_frame_end_to_end": med(e2e),
        "ms_per_frame_end_to_end_mean": float(np.mean(e2e)) * 1e3,
        "frames_per_s": 1e3 / med(e2e),
        "phases_ms_per_frame": {"voxelize": med(ph[:, 0]), "c3hlac": med(ph[:, 1]), "search": med(ph[:, 2])},
        "kernel_ms_per_frame": {"voxelize": kms("voxelize"), "c3hlac": kms("c3hlac"),
                                "search": kms("compress", "score", "replay")},
        "frames": n_frames,
        "note": "detect_object.cpp's per-callback path, one frame at a time: %d 1M-point host clouds (pageable, %d "
                "distinct Kinect scenes) -> c3h_voxelize (H2D inside) -> c3h_extract -> c3h_search (lists to the "
                "host); medians; compare cpu_baseline.phases_s_per_frame (same scene shape, one core)"
                % (n_frames, n_scenes),
    }


def native_single_frame(scenes, axis_t, var, axis_q, n_frames, lists_out=None):
    """The same per-callback loop in C++ on the C-ABI alone (tools/single_frame_native.cpp,
    built by the library's Makefile): the frames and bases go through a scratch file to a
    child process with its own context, which prints its medians (steady_clock around each
    call) as one JSON line.  None when the tool was not built."""
    exe = ROOT / "mapping-private_amd" / "lib" / "single_frame_native"
    if not exe.exists():
        return None
    import subprocess
    import tempfile
    M, r, Dq = axis_q.shape
    with tempfile.TemporaryDirectory() as td:
        f = Path(td) / "frames.bin"
        with open(f, "wb") as fh:
            fh.write(np.array([len(scenes), D, VARIANT, M, r, VARIANT, SUBDIV, 0], np.int32).tobytes())
            fh.write(np.array([LEAF, EXIST_THR], np.float32).tobytes())
            fh.write(np.array(list(THR) + list(BOX), np.int32).tobytes())
            for a in (axis_t, var, axis_q):
                fh.write(np.ascontiguousarray(a, dtype=np.float32).tobytes())
            for sc in scenes:
                sc = np.ascontiguousarray(sc, dtype=np.float32)
                fh.write(np.int64(sc.shape[0]).tobytes())
                fh.write(sc.tobytes())
        cmd = [str(exe), str(f), str(n_frames)] + ([str(lists_out)] if lists_out else [])
        p = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    if p.returncode != 0:
        raise RuntimeError("single_frame_native failed (%d): %s" % (p.returncode, p.stderr[-2000:]))
    res = json.loads(p.stdout.strip().splitlines()[-1])
    res["frames_per_s"] = 1e3 / res["ms_per_frame_end_to_end"]
    res["note"] = ("the same frames through tools/single_frame_native.cpp: C++ on the C-ABI, no Python "
                   "(steady_clock medians, its own process and context)")
    return res


def real_views_pass(ctx, dev, torch, synth, c3hlac, reps=10):
    """The reference's own sensor frames through c3h_run_point_frames: the committed sample
    of 126 captured Kinect object views (tests/golden/kinect_views_126.npz, 258..19,005
    points each; quantised depth puts many points on cell faces), leaf 0.01 on a 40^3 canvas,
    C3-HLAC-117 S = 4 + 3 models x r = 5 (117 -> 30), rank 1, views resident in HBM.  Reports
    the batched share, the voxels whose centroid lies in another cell (corrected in the
    batch) and frames/s (best of `reps` calls)."""
    f = ROOT / "tests" / "golden" / "kinect_views_126.npz"
    if not f.exists():
        return None
    with np.load(f, allow_pickle=False) as z:
        st, P = z["starts"], z["pts"]
        frames = [torch.from_numpy(np.ascontiguousarray(P[st[i]:st[i + 1]])).to(dev) for i in range(len(st) - 1)]
    M = 3
    axis_t, var, axis_q = synth.random_bases(117, 30, M, 5, seed=synth.BASE_SEED + 91)
    ctx.search_setup(axis_t, var, axis_q)
    ctx.set_rank(1)
    out = torch.zeros((len(frames), 3 * M), dtype=torch.int64, device=dev)
    args = (0.01, (40, 40, 40), 117, THR, 4, BOX, 4, True, out)
    ctx.set_batch(64)  # (the views are small: 64 per batch)
    ctx.run_point_frames(frames, *args)  # untimed: sizes the buffers
    torch.cuda.synchronize(dev)
    best = None
    for _ in range(reps):
        t0 = time.perf_counter()
        _, info = ctx.run_point_frames(frames, *args)
        torch.cuda.synchronize(dev)
        el = time.perf_counter() - t0
        best = el if best is None else min(best, el)
    return {
        "frames": len(frames), "points": int(st[-1]),
        "frames_batched": int((info["status"] == 0).sum()),
        "views_with_offcell_voxels": int((info["n_moved"] > 0).sum()), "offcell_voxels": int(info["n_moved"].sum()),
        "frames_per_s": len(frames) / best, "ms_per_call": best * 1e3,
        "note": "126 captured Kinect views of color_feature_classification/demos/data (every 12th), leaf 0.01, "
                "canvas 40^3, C3-HLAC-117 S=4, 117->30, 3 models x r=5, box 2x2x2, rank 1; one call, one host sync",
    }


def pmc_traffic(frames_per_tick):
    """HBM bytes per tick launch from the committed rocprofv3 --pmc summary of this build
    (tools/pmc.sh -> tools/pmc_summary.py): FETCH_SIZE x2 (gfx950 correction) +
    WRITE_SIZE of c3h_tick_kernel per frame through the pipeline, times the frames per tick.
    PMC needs its own profiler pass, so it cannot be collected inside the timed run; None
    when no summary is committed."""
    f = ROOT / "profiles" / "pmc_c3_traffic.json"
    if not f.exists():
        return None
    per_frame = json.load(open(f)).get("tick_hbm_bytes_per_frame")
    return per_frame * frames_per_tick if per_frame is not None else None


def host_cpu():
    model = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    try:
        avail = len(os.sched_getaffinity(0))
    except AttributeError:
        avail = os.cpu_count()
    return model, os.cpu_count(), avail


def cpu_baseline(words, gpu_rec, seconds, scene_pts=None, scene_grid=None):
    """The oracle (single-threaded C restatement of the reference, -O2) on the same
    workload -- C3-HLAC-117 + exist + setData/search of the 10 models in the reference's
    fp32 order -- repeated on the first timed frame's grid until `seconds` elapse (at least
    once).  It is also the check of that frame: the GPU detection of every model must be
    the float64 oracle's (position, mode) with the score within 1e-5.  The voxelise phase
    of detect_object.cpp:182-186's split (getVoxelGrid on the 1M points) is timed on the
    scene the frame's grid was voxelised from, and its grid checked against the GPU's."""
    import pyoracle as po
    from c3hlac import synth
    t_vox, vox_check = None, None
    if scene_pts is not None:
        nv, tv0 = 0, time.perf_counter()
        while nv == 0 or time.perf_counter() - tv0 < seconds / 4:
            gv, lay_v, cl_v = po.voxelize(scene_pts, LEAF)
            nv += 1
        t_vox = (time.perf_counter() - tv0) / nv
        if scene_grid is not None:  # packed words of the oracle's voxels vs the GPU's grid
            w = scene_grid.cpu().numpy().view(np.uint32)
            occ = np.flatnonzero(lay_v >= 0)
            ok = (list(gv.div_b) == [GRID] * 3 and np.array_equal(np.flatnonzero(w), occ) and
                  np.array_equal(w[occ] & np.uint32(0xFFFFFF), cl_v[lay_v[occ], 3].view(np.uint32)))
            vox_check = "oracle getVoxelGrid of the scene == the GPU's grid: %s" % ("yes" if ok else "MISMATCH")
    g, layout, cloud = po.grid_inputs(words, (GRID,) * 3, LEAF)
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
    # check (untimed): float64 search on the oracle's features vs the GPU's record; a
    # different position is accepted only where the float64 scores tie within 2e-5
    _, _, sc = po.search(sb, f117, ex, ap, axis_q, BOX, RANK, EXIST_THR, dbl=True, want_scores=True)
    sc = sc.reshape(M, -1)
    pe = int(np.ceil(GRID / SUBDIV)) - BOX[0] + 1
    got = gpu_rec.reshape(M * RANK, 3)
    bad = []
    for m in range(M):
        s = float(got[m, 0:1].view(np.float64)[0])
        x, y, z, mode = (int(v) for v in got[m, 1:3].view(np.int32))
        p = (z * pe + y) * pe + x
        best = int(np.argmax(sc[m]))
        ok = mode == 0 and abs(s - sc[m, p]) <= 1e-5 * sc[m, p] and (p == best or sc[m, p] >= sc[m, best] * (1 - 2e-5))
        if not ok:
            bad.append(m)
    tot = t_c3 + t_s
    model, ncpu, avail = host_cpu()
    return {
        "value": GRID ** 3 * n / tot / 1e6,
        "unit": "Mvoxels/s",
        "cores": 1,
        "kind": "port",
        "sample": "%d run(s) of the first timed frame (256^3 grid; C3-HLAC-117 + exist gate + 10-model search "
                  "in the reference's fp32 order), C3 %.3f s/frame, search %.3f s/frame" % (n, t_c3 / n, t_s / n),
        "cpu_model": model,
        "nproc": ncpu,
        "cpus_available": avail,
        "frame_check": "GPU detections of the first timed frame vs the float64 oracle on its grid: %s" % (
            "all %d models equal (score within 1e-5)" % M if not bad else "MISMATCH in models %s" % bad),
        "phases_s_per_frame": {"voxelize": t_vox, "c3hlac": t_c3 / n, "search": t_s / n},
        "phases_note": "detect_object.cpp:182-186's split, one core: getVoxelGrid of the 1M-point scene (%s), "
                       "C3-HLAC + exist, setData + search; 'value' covers the C3 + search phases over the 256^3 "
                       "voxels (the metric's grid-resident region)" % (vox_check or "not timed"),
        "frames_per_s_end_to_end": 1.0 / (t_vox + (t_c3 + t_s) / n) if t_vox else None,
    }


def cpu_baseline_points(synth, seconds):
    """configs[3]'s unit of work on one core (single-thread frames/s): one
    1M-point frame of the points-in pass through the oracle -- getVoxelGrid (128^3),
    C3-HLAC-981 S=10 + exist, setData (981 -> 100) + search of 1 model x r=20 -- timed per
    phase, repeated over the pass's base scenes until `seconds` elapse (at least once)."""
    import pyoracle as po
    axis_t, var, axis_q = synth.random_bases(P_VARIANT, D, P_M, R, seed=synth.BASE_SEED + 31)
    ap = synth.whiten(axis_t, var)
    tv = tc = ts = 0.0
    n = 0
    t_start = time.perf_counter()
    while n == 0 or time.perf_counter() - t_start < seconds:
        pts = synth.kinect_scene(N_RAYS, grid=P_GRID, leaf=P_LEAF, seed=synth.BASE_SEED + 7000 + n % 16)
        t0 = time.perf_counter()
        g, layout, cloud = po.voxelize(pts, P_LEAF)
        t1 = time.perf_counter()
        f, sb, _ = po.c3hlac(g, layout, cloud, P_VARIANT, THR, P_LEAF, SUBDIV)
        ex = po.exist(f)
        t2 = time.perf_counter()
        po.search(sb, f, ex, ap, axis_q, BOX, RANK, EXIST_THR)
        t3 = time.perf_counter()
        tv, tc, ts = tv + t1 - t0, tc + t2 - t1, ts + t3 - t2
        n += 1
    tot = tv + tc + ts
    return {
        "value": n / tot,
        "unit": "frames/s",
        "cores": 1,
        "kind": "port",
        "sample": "%d 1M-point frame(s) of the points-in pass's base scenes, one core: voxelize %.3f s, C3-HLAC-981 "
                  "%.3f s, search %.3f s per frame" % (n, tv / n, tc / n, ts / n),
        "phases_s_per_frame": {"voxelize": tv / n, "c3hlac": tc / n, "search": ts / n},
    }


def _cpu_points_worker(seconds, k):
    """One core of cpu_baseline_points_parallel (a child process: numpy + the C oracle only)."""
    from c3hlac import synth
    import pyoracle as po
    axis_t, var, axis_q = synth.random_bases(P_VARIANT, D, P_M, R, seed=synth.BASE_SEED + 31)
    ap = synth.whiten(axis_t, var)
    n, busy = 0, 0.0
    t_start = time.perf_counter()
    while n == 0 or time.perf_counter() - t_start < seconds:
        pts = synth.kinect_scene(N_RAYS, grid=P_GRID, leaf=P_LEAF, seed=synth.BASE_SEED + 7000 + (k + n) % 16)
        t0 = time.perf_counter()
        g, layout, cloud = po.voxelize(pts, P_LEAF)
        f, sb, _ = po.c3hlac(g, layout, cloud, P_VARIANT, THR, P_LEAF, SUBDIV)
        po.search(sb, f, po.exist(f), ap, axis_q, BOX, RANK, EXIST_THR)
        busy += time.perf_counter() - t0
        n += 1
    return {"frames": n, "busy_s": busy}


def cpu_baseline_points_parallel(seconds, procs=None):
    """configs[3]'s frame-parallel CPU upper bound: the
    single-core loop of cpu_baseline_points in `procs` independent processes at once (frames
    are independent: OpenMP over frames would do the same), each for `seconds`; frames/s is
    the sum of the processes' rates.  Children are started as new interpreters (never a fork
    of this GPU process's state) and touch no GPU."""
    import subprocess
    if procs is None:
        procs = max(1, min(16, len(os.sched_getaffinity(0))))
    env = dict(os.environ)
    env["OMP_NUM_THREADS"] = "1"
    cmd = [sys.executable, str(ROOT / "bench.py"), "--cpu-points-worker", str(seconds)]
    ps = [subprocess.Popen(cmd + [str(k)], stdout=subprocess.PIPE, stderr=subprocess.DEVNULL, env=env)
          for k in range(procs)]
    outs = [json.loads(p.communicate()[0].decode().strip().splitlines()[-1]) for p in ps]
    rate = sum(o["frames"] / o["busy_s"] for o in outs)
    return {"value": rate, "unit": "frames/s", "cores": procs, "kind": "port",
            "sample": "%d processes x >= %.0f s of the single-core loop (voxelize + C3-HLAC-981 + search per 1M-point "
                      "frame), %d frames in total; frames/s summed over the processes" %
                      (procs, seconds, sum(o["frames"] for o in outs))}


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "--cpu-points-worker":
        print(json.dumps(_cpu_points_worker(float(sys.argv[2]), int(sys.argv[3]))))
        sys.exit(0)
    main()
