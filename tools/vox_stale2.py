"""Diagnostics: frame sequences of the GPU parity tests on one fresh context, every frame's
grid words against the oracle (bad words per frame)."""
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT / "mapping-private_amd"), str(ROOT / "oracle")]


def main():
    import c3hlac
    import pyoracle as po
    from c3hlac import synth

    def words_bad(ctx, pts, leaf, zl=float("inf")):
        gi = ctx.voxelize(pts, leaf, zl)
        g, layout, cl = po.voxelize(pts, leaf, zl)
        w = ctx.grid()
        occ = layout >= 0
        exp = (1 << 24) | cl[layout[occ], 3].view(np.uint32)
        return {"n": int(occ.sum()), "n_ok": int(gi.n_occ) == int(occ.sum()), "bad": int((w[occ] != exp).sum()),
                "stray": int((w[~occ] != 0).sum())}

    rng = np.random.default_rng(11)

    def cloud(n, span):
        xyz = (rng.random((n, 3)) * np.asarray(span, np.float64)).astype(np.float32)
        col = rng.integers(0, 256, (n, 3))
        return np.concatenate([xyz, synth.pack_rgb(col[:, 0], col[:, 1], col[:, 2])[:, None]], 1).astype(np.float32)

    seqs = {
        "regrows": [cloud(2000, 0.05), cloud(400_000, 1.0), cloud(3000, 0.08), cloud(50_000, (3.0, 0.2, 0.2)),
                    cloud(60_000, (0.2, 2.7, 1.6)), cloud(1500, 0.04)],
        "sparse_then_small": [cloud(400_000, 1.0), cloud(3000, 0.08), cloud(3000, 0.08)],
        "sparse100k_then_small": [cloud(100_000, 1.0), cloud(3000, 0.08)],
        "sparse_twice": [cloud(400_000, 1.0), cloud(400_000, 1.0), cloud(3000, 0.08)],
    }
    for name, frames in seqs.items():
        with c3hlac.Context(0) as ctx:
            res = [words_bad(ctx, f, 0.01) for f in frames]
            print(json.dumps({"seq": name, "frames": res}), flush=True)


if __name__ == "__main__":
    main()
