"""Points-in batches on the reference's own sensor data (round 4).

126 of the 1,512 captured Kinect views of color_feature_classification/demos/data (every
12th, two angles of each of the 63 objects; tests/golden/kinect_views_126.npz, made by
tests/golden/gen_kinect_views.py) through c3h_run_point_frames at leaf 0.01 on a 40^3
canvas.  Quantised depth puts many points on cell faces: 23 of the 126 views hold voxels
whose centroid (sum * (1/n), PCL 1.0 on Eigen 3.0) lies in another cell, where the
reference takes the centroid's cell as subdivision and neighbour base (c3_hlac.cpp:349-377).
The batch sums those voxels exactly and recomputes their subdivisions after its C3 stage,
so every view stays batched (status 0), and:
  - n_moved equals the oracle's count of off-cell voxels, per view;
  - every view's records equal the single-frame path's (c3h_voxelize's exact pass +
    offcell correction), bit for bit;
  - every view with a moved voxel, and every 8th other view, equals the float64 oracle run
    from the points (position and mode exact unless scores tie within 1e-5; score within
    1e-5).
C3-HLAC-117 (S = 4) and C3-HLAC-981 (S = 5), both with offsets; and the other colour
tables (ColorCHLAC's (v, 255 - v), C3's float sin/cos) on a sample of the views."""
import numpy as np
import pytest

import c3hlac
import pyoracle as po
from c3hlac import synth
from conftest import GOLDEN, THR

pytestmark = pytest.mark.gpu

LEAF, CANVAS, BOX, EXIST, RTOL = 0.01, (40, 40, 40), (2, 2, 2), 4, 1e-5


def _views():
    with np.load(GOLDEN / "kinect_views_126.npz", allow_pickle=False) as z:
        st, P = z["starts"], z["pts"]
        return [np.ascontiguousarray(P[st[i]:st[i + 1]]) for i in range(len(st) - 1)]


def _moved(pts):
    po.set_voxel_semantics(True)
    g, lay, cl = po.voxelize(pts, LEAF)
    occ = np.flatnonzero(lay >= 0)
    d = np.array(g.div_b)
    own = np.stack([occ % d[0], (occ // d[0]) % d[1], occ // (d[0] * d[1])], 1) + np.array(g.min_b)
    c = cl[lay[occ], :3]
    return int((np.floor(c / np.float32(LEAF)) != own).any(1).sum())


@pytest.mark.parametrize("variant,S,off", [(117, 4, (0, 0, 0)), (981, 5, (1, 0, 2))])
def test_real_views_batched_with_offcell_fixup(ctx, variant, S, off):
    import torch
    views = _views()
    nfr = len(views)
    dev = torch.device("cuda", 0)
    frames = [torch.from_numpy(v).to(dev) for v in views]
    torch.cuda.synchronize()
    M = 3
    axis_t, var, axis_q = synth.random_bases(variant, 30, M, 5, seed=synth.BASE_SEED + 91)
    ap = synth.whiten(axis_t, var)
    ctx.search_setup(axis_t, var, axis_q)
    ctx.set_rank(1)
    ctx.set_batch(32)
    ctx.set_pipeline(True)
    d_out = torch.zeros((nfr, 3 * M), dtype=torch.int64, device=dev)
    nm, info = ctx.run_point_frames(frames, LEAF, CANVAS, variant, THR, S, BOX, EXIST, True, d_out, offset=off)
    got = d_out.cpu().numpy().view(c3hlac.DET_DTYPE).reshape(nfr, M)
    moved = np.array([_moved(v) for v in views])
    assert (moved > 0).sum() >= 20  # the case under test is in the sample
    assert (info["status"] == 0).all(), np.flatnonzero(info["status"])
    assert np.array_equal(info["n_moved"], moved), np.flatnonzero(info["n_moved"] != moved)
    # every view: the single-frame path's records
    for i in range(nfr):
        ctx.voxelize(views[i], LEAF)
        ctx.extract(variant, THR, S, off)
        ctx.set_rank(1)
        lists, _ = ctx.search(BOX, EXIST)
        assert np.array_equal(got[i], lists[:, 0]), (i, moved[i])
    # the float64 oracle from the points: the moved views and every 8th view
    for i in [i for i in range(nfr) if moved[i] or i % 8 == 0]:
        g, layout, cloud = po.voxelize(views[i], LEAF)
        fe, sb, hn = po.c3hlac(g, layout, cloud, variant, THR, LEAF, S, off, exact=True)
        assert hn > 0, i
        ex = po.exist(fe)
        _, _, sc = po.search(sb, fe, ex, ap, axis_q, BOX, 1, EXIST, dbl=True, want_scores=True)
        assert list(info["div_b"][i]) == list(g.div_b) and list(info["subdiv_b"][i]) == list(sb), i
        xe, ye = sb[0] - 1, sb[1] - 1
        if min(sb) < 2:  # no 2 x 2 x 2 box fits: searchPart runs no position
            assert (got[i]["score"] == 0).all(), i
            continue
        sc = sc.reshape(M, -1)
        for m in range(M):
            e = got[i, m]
            if sc[m].max() <= 0:  # no position passes the gate: the fresh setRank record
                assert float(e["score"]) == 0.0, (i, m)
                continue
            p = (int(e["z"]) * ye + int(e["y"])) * xe + int(e["x"])
            best = int(np.argmax(sc[m]))
            assert int(e["mode"]) == 0
            assert abs(float(e["score"]) - sc[m, p]) <= RTOL * sc[m, p], (i, m, float(e["score"]), sc[m, p])
            if p != best:
                assert sc[m, p] >= sc[m, best] * (1 - 2 * RTOL), (i, m, p, best)


@pytest.mark.parametrize("color_mode", [c3hlac.COLOR_CHLAC, c3hlac.COLOR_C3_FLOAT])
def test_real_views_batched_colour_modes(ctx, color_mode):
    """The other setColor tables through the points-in batch (round 4): ColorCHLAC's
    (v, 255 - v) and C3's float sin/cos, every 5th of the committed views, records equal
    to the single-frame path with the same table and the sampled views to the oracle."""
    import torch
    views = _views()[::5]
    nfr = len(views)
    dev = torch.device("cuda", 0)
    frames = [torch.from_numpy(v).to(dev) for v in views]
    M = 2
    axis_t, var, axis_q = synth.random_bases(117, 24, M, 4, seed=synth.BASE_SEED + 92)
    ap = synth.whiten(axis_t, var)
    ctx.search_setup(axis_t, var, axis_q)
    ctx.set_rank(1)
    ctx.set_batch(16)
    ctx.set_pipeline(True)
    d_out = torch.zeros((nfr, 3 * M), dtype=torch.int64, device=dev)
    _, info = ctx.run_point_frames(frames, LEAF, CANVAS, 117, THR, 4, BOX, EXIST, True, d_out, color_mode=color_mode)
    got = d_out.cpu().numpy().view(c3hlac.DET_DTYPE).reshape(nfr, M)
    assert (info["status"] == 0).all(), np.flatnonzero(info["status"])
    for i in range(nfr):
        ctx.voxelize(views[i], LEAF)
        ctx.extract(117, THR, 4, color_mode=color_mode)
        ctx.set_rank(1)
        lists, _ = ctx.search(BOX, EXIST)
        assert np.array_equal(got[i], lists[:, 0]), i
    for i in range(0, nfr, 6):
        g, layout, cloud = po.voxelize(views[i], LEAF)
        fe, sb, hn = po.c3hlac(g, layout, cloud, 117, THR, LEAF, 4, color_mode=color_mode, exact=True)
        if min(sb) < 2:
            continue
        ex = po.exist(fe)
        _, _, sc = po.search(sb, fe, ex, ap, axis_q, BOX, 1, EXIST, dbl=True, want_scores=True)
        sc = sc.reshape(M, -1)
        xe, ye = sb[0] - 1, sb[1] - 1
        for m in range(M):
            e = got[i, m]
            if sc[m].max() <= 0:
                assert float(e["score"]) == 0.0, (i, m)
                continue
            p = (int(e["z"]) * ye + int(e["y"])) * xe + int(e["x"])
            assert abs(float(e["score"]) - sc[m, p]) <= RTOL * sc[m, p], (i, m)
            assert sc[m, p] >= sc[m].max() * (1 - 2 * RTOL), (i, m)
