"""Generate the committed golden fixtures under tests/golden/ (run in the build container).

Every expected output comes from the C oracle (oracle/c3hlac_oracle.c) and is asserted
equal to the independent numpy restatement (oracle/np_ref.py, which takes its bin map
from the reference's own unrolled code) before it is written.  Fixtures are data only:
seeded inputs + expected outputs, stored as .npz (no pickle).

Usage: python oracle/gen_golden.py
"""
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT / "oracle"), str(ROOT / "mapping-private_amd")]
import np_ref as npr  # noqa: E402
import pyoracle as po  # noqa: E402
from c3hlac import synth  # noqa: E402

OUT = ROOT / "tests" / "golden"
THR = (147, 146, 148)


def one(name, pts, leaf, subdiv, offset, D, M, r, ranges, rank, thr_exist, seed, z_limit=np.inf):
    g, layout, cloud = po.voxelize(pts, leaf, z_limit)
    div, mb, words, lay_np = npr.voxelize(pts, leaf, z_limit)
    assert tuple(g.div_b) == div and tuple(g.min_b) == mb
    assert np.array_equal(layout, lay_np)
    rec = dict(pts=pts, leaf=np.float32(leaf), z_limit=np.float32(z_limit), div_b=np.array(div, np.int32),
               min_b=np.array(mb, np.int32), leaf_layout=layout, cloud=cloud,
               grid_words=words.reshape(-1), thr=np.array(THR, np.int32), subdiv=np.int32(subdiv),
               offset=np.array(offset, np.int32))
    for variant in (981, 117):
        fe, sb, hn = po.c3hlac(g, layout, cloud, variant, THR, leaf, subdiv, offset, exact=True)
        ff, _, _ = po.c3hlac(g, layout, cloud, variant, THR, leaf, subdiv, offset, exact=False)
        fn, exn, sbn = npr.c3hlac(words, variant, THR, subdiv, offset)
        assert np.array_equal(fe, fn), name
        assert tuple(sb) == tuple(sbn)
        rec["feat%d_exact" % variant] = fe
        rec["feat%d_faithful" % variant] = ff
        rec["exist"] = po.exist(ff if variant == 981 else rec["feat981_faithful"])
        assert np.array_equal(rec["exist"], exn)
        rec["subdiv_b"] = np.array(sb, np.int32)
    # search on the 981 features
    axis_t, var, axis_q = synth.random_bases(981, D, M, r, seed=seed)
    ap = synth.whiten(axis_t, var)
    feat = rec["feat981_faithful"]
    ex = rec["exist"]
    sb = tuple(rec["subdiv_b"])
    L, nm, sc = po.search(sb, feat, ex, ap, axis_q, ranges, rank, thr_exist, rotate=True, dbl=False, want_scores=True)
    Ld, _, scd = po.search(sb, feat, ex, ap, axis_q, ranges, rank, thr_exist, rotate=True, dbl=True, want_scores=True)
    ms = npr.scores(sb, feat, ex, ap, axis_q, ranges, thr_exist)
    flat = np.concatenate([s.reshape(-1) for (_, _, _, s) in ms]) if ms else np.zeros(0)
    assert np.allclose(flat, scd[: flat.size], rtol=1e-12, atol=1e-12)
    rec.update(axis_t=axis_t, var=var, axis_q=axis_q, ranges=np.array(ranges, np.int32), rank=np.int32(rank),
               thr_exist=np.int32(thr_exist), scores_f32=sc, scores_f64=scd,
               lists_f32=np.array([[list(e) for e in m] for m in L.records()], np.float64),
               lists_f64=np.array([[list(e) for e in m] for m in Ld.records()], np.float64))
    np.savez_compressed(OUT / (name + ".npz"), **rec)
    size = (OUT / (name + ".npz")).stat().st_size
    print(name, "grid", div, "occ", int((words != 0).sum()), "sb", sb, "modes", nm, "bytes", size)


def main():
    OUT.mkdir(parents=True, exist_ok=True)
    # BASELINE configs[0] at its stated size: 50k-point parity cloud -> 64^3, C3-HLAC-981,
    # subdivision 10 (7^3 = 343 subdivisions), 1-model search
    one("cfg0_parity_64", synth.parity_cloud(50_000, grid=64, leaf=0.01, seed=0xC3A1AC), 0.01, 10, (0, 0, 0),
        D=100, M=1, r=20, ranges=(2, 2, 2), rank=1, thr_exist=100, seed=10)
    one("cfg1_parity_24", synth.parity_cloud(4000, grid=24, leaf=0.01, seed=101), 0.01, 8, (0, 0, 0),
        D=12, M=2, r=4, ranges=(1, 1, 2), rank=1, thr_exist=10, seed=11)
    one("kinect_40_offsets", synth.kinect_scene(25_000, grid=40, leaf=0.02, seed=202), 0.02, 6, (1, 2, 0),
        D=16, M=3, r=5, ranges=(2, 1, 2), rank=3, thr_exist=20, seed=12)
    one("kinect_32_whole", synth.kinect_scene(15_000, grid=32, leaf=0.02, seed=303), 0.02, 0, (0, 0, 0),
        D=8, M=1, r=3, ranges=(1, 1, 1), rank=1, thr_exist=0, seed=13)


if __name__ == "__main__":
    main()
