"""Diagnostics: does a c3h_voxelize frame leave state that corrupts the next frame?  Each
case voxelises frame X, then a probe frame P (random colours, several points per voxel,
cells -20..20), and checks P's grid words against the oracle.  Prints one JSON line per case."""
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT / "mapping-private_amd"), str(ROOT / "oracle")]


def cloud(rng, n, lo, hi, leaf=0.01):
    cells = rng.integers(lo, hi, (n, 3))
    xyz = ((cells + 0.1 + 0.8 * rng.random((n, 3))) * leaf).astype(np.float32)
    col = rng.integers(0, 256, (n, 3))
    from c3hlac import synth
    return np.concatenate([xyz, synth.pack_rgb(col[:, 0], col[:, 1], col[:, 2])[:, None]], 1).astype(np.float32)


def check(ctx, pts, leaf, po):
    gi = ctx.voxelize(pts, leaf)
    g, layout, cl = po.voxelize(pts, leaf)
    words = ctx.grid()
    occ = layout >= 0
    exp = (1 << 24) | cl[layout[occ], 3].view(np.uint32)
    bad = int((words[occ] != exp).sum())
    return {"n_occ_ok": int(gi.n_occ) == int(occ.sum()), "bad_words": bad, "n_occ": int(occ.sum())}


def main():
    import c3hlac
    import pyoracle as po
    from c3hlac import synth
    rng = np.random.default_rng(3)
    probe = cloud(rng, 30000, -20, 20)
    cases = {
        "fresh": [],
        "multipoint": [cloud(rng, 20000, 0, 6)],
        "two_probes": [probe],
        "nan_one": [np.full((10, 4), np.nan, np.float32), np.array([[0.123, -0.456, 0.789, 1.0]], np.float32)],
        "kinect256": [synth.kinect_scene(1_000_000, grid=256, leaf=0.01, seed=5)],
        "wide": [cloud(rng, 50000, 0, 300)],
        "zlimit": [synth.parity_cloud(500, grid=8, leaf=0.01, seed=3)],
    }
    def dense(ctx, G, variant):
        words = synth.random_words(G, 0.9, seed=7, colour_max=255)
        ctx.set_grid(words.reshape(-1), (G, G, G))
        ctx.extract(variant, (147, 146, 148), 10)

    def grsd(ctx):
        pts = c3hlac.read_pcd(ROOT / "tests" / "golden" / "ref_fixtures" / "pcd" / "noisy_sphere_green.pcd")
        ctx.voxelize(pts, 0.01)
        ctx.compute_normals(0.02)
        ctx.extract_grsd(0)

    def down(ctx):
        ctx.voxelize(probe, 0.01)
        ctx.downsampled()

    def search(ctx):
        ctx.voxelize(synth.kinect_scene(300_000, grid=96, leaf=0.02, seed=77), 0.02)
        ctx.extract(981, (147, 146, 148), 8)
        axis_t, var, axis_q = synth.random_bases(981, 40, 3, 8, seed=9)
        ctx.search_setup(axis_t, var, axis_q)
        ctx.set_rank(4)
        ctx.search((1, 2, 3), 50)

    acts = {"dense128_981": lambda c: dense(c, 128, 981), "dense128_117": lambda c: dense(c, 128, 117),
            "grsd": grsd, "downsampled": down, "search": search}
    for name in acts:
        cases[name] = name
    for name, frames in cases.items():
        with c3hlac.Context(0) as ctx:
            pre = []
            if isinstance(frames, str):
                acts[frames](ctx)
                frames = []
            for f in frames:
                gi = ctx.voxelize(f, 0.01, 0.04 if name == "zlimit" else float("inf"))
                pre.append(int(gi.n_occ))
            r = check(ctx, probe, 0.01, po)
            r2 = check(ctx, probe, 0.01, po)  # the probe again
            print(json.dumps({"case": name, "pre_n_occ": pre, "probe": r, "probe_again": r2}), flush=True)


if __name__ == "__main__":
    main()
