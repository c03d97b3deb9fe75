"""configs[3]'s per-rank shard on one GPU: the bench's points-in pass
(bench.points_pass: 16 Kinect base scenes, frames made distinct by colour XOR and whole-cell
x shifts, 128^3 canvas, C3-HLAC-981 S = 10, 981 -> 100, 1 model x r = 20, rank 1) run on the
shard rank 0 gets at N = 1, 2, 4, 8 (frames 0, N, 2N, ... of 512), each timed as bench.py
times it (one c3h_run_point_frames call between device synchronisations), 3 repetitions.
Prints one JSON line per (shard, batch, repetition) and a summary line with each shard's
per-frame rate against the 512-frame rate.  Records of every shard equal the 512-frame run's
records of the same frames (checked).
usage: python tools/points_shard.py [batches, e.g. 64,32] [reps]"""
import json
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "mapping-private_amd")]


def main():
    import torch
    import c3hlac
    from c3hlac import synth
    import bench
    batches = [int(b) for b in (sys.argv[1] if len(sys.argv) > 1 else "64").split(",")]
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    nb = 16
    base = [torch.from_numpy(synth.kinect_scene(bench.N_RAYS, grid=bench.P_GRID, leaf=bench.P_LEAF,
                                                seed=synth.BASE_SEED + 7000 + s)).to(dev) for s in range(nb)]

    def frame(i):  # bench.points_pass's frame(i)
        t = base[i % nb].clone()
        k = i // nb
        t[:, 3] = (t[:, 3].view(torch.int32) ^ ((k * 0x2F1D37) & 0xFFFFFF)).view(torch.float32)
        t[:, 0] = (t[:, 0].double() + k * bench.P_LEAF).float()
        return t

    n_total = 512
    frames = [frame(i) for i in range(n_total)]
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    ctx = c3hlac.Context(0)
    ctx.set_stream(stream.cuda_stream)
    ctx.set_lanes(bench.LANES)
    ctx.set_pipeline(True)
    axis_t, var, axis_q = synth.random_bases(bench.P_VARIANT, bench.D, bench.P_M, bench.R, seed=synth.BASE_SEED + 31)
    ctx.search_setup(axis_t, var, axis_q)
    ctx.set_rank(1)
    canvas = (bench.P_GRID,) * 3
    args = (bench.P_LEAF, canvas, bench.P_VARIANT, bench.THR, bench.SUBDIV, bench.BOX, bench.EXIST_THR, True)
    ref = torch.zeros((n_total, 3 * bench.P_M), dtype=torch.int64, device=dev)
    summary = {}
    for B in batches:
        ctx.set_batch(B)
        ctx.run_point_frames(frames[:4 * B], *args, ref)  # untimed: sizes the buffers (as bench.py)
        torch.cuda.synchronize(dev)
        ctx.run_point_frames(frames, *args, ref)
        torch.cuda.synchronize(dev)
        want = ref.cpu()
        for world in (1, 2, 4, 8):
            mine = list(range(0, n_total, world))
            fr = ctx.prepare_point_frames([frames[i] for i in mine])
            out = torch.zeros((len(fr), 3 * bench.P_M), dtype=torch.int64, device=dev)
            rates = []
            for rep in range(reps):
                ctx.timing(c3hlac.timing_mask("voxelize", "pipeline"))
                ctx.kernel_times(reset=True)
                torch.cuda.synchronize(dev)
                t0 = time.perf_counter()
                ctx.run_point_frames(fr, *args, out)
                torch.cuda.synchronize(dev)
                el = time.perf_counter() - t0
                kt = ctx.kernel_times(reset=True)
                ctx.timing(False)
                same = bool(torch.equal(out.cpu(), want[mine]))
                rates.append(len(fr) / el)
                print(json.dumps({"batch": B, "world": world, "shard_frames": len(fr), "rep": rep,
                                  "frames_per_s": len(fr) / el, "ms_per_call": el * 1e3,
                                  "vox_us_per_frame": kt["voxelize"][0] / max(kt["voxelize"][1], 1) * 1e3,
                                  "tick_ms_total": kt["pipeline"][0], "ticks": kt["pipeline"][1],
                                  "records_equal_512_run": same}), flush=True)
                assert same, "shard records differ from the 512-frame run"
            summary["B%d_shard%d" % (B, len(fr))] = max(rates)
    full = {B: summary["B%d_shard512" % B] for B in batches}
    print(json.dumps({"summary": summary,
                      "shard_over_full_best_B": {k: v / max(full.values()) for k, v in summary.items()}}), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
