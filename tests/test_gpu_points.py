"""Points-in frame pipeline (c3h_run_point_frames): BASELINE configs[3]'s unit of work --
a point cloud per callback, limitPoint + getVoxelGrid + extractC3HLACSignature981 + search
(color_voxel_recognition/test/detect_object.cpp:139-186) -- for batches of frames with no
per-frame host round trip.

- configs[3] at its stated size on one GPU: 512 independent 1M-point frames at 128^3
  (C3-HLAC-981, S = 10, compress 981 -> 100, 1 model x r = 20, box 2x2x2, rank 1), frames
  on the device; every 4th frame (128 of 512) re-computed by the oracle from its points
  (grid geometry and counts exact, detection within 1e-5 of the float64 oracle); sampled
  frames bit-identical to the single-frame path.
- host-resident frames (the H2D-inclusive path) give the same records as device frames.
- mixed geometries in one batch: frames of different extents and min_b inside the canvas,
  a frame beyond the canvas, an empty frame, a frame whose centroids may round across a
  cell boundary -- records equal the single-frame path's, statuses as documented."""
import concurrent.futures as cf

import numpy as np
import pytest

import c3hlac
import pyoracle as po
from c3hlac import synth
from conftest import THR

pytestmark = pytest.mark.gpu

G, LEAF, S, D, R, BOX, EXIST = 128, 0.02, 10, 100, 20, (2, 2, 2), 100
RTOL = 1e-5


def _single(ctx, pts, variant=981, subdiv=S, z_limit=float("inf")):
    """The single-frame path (c3h_voxelize + c3h_extract + search from fresh lists)."""
    ctx.voxelize(pts, LEAF, z_limit)
    ctx.extract(variant, THR, subdiv)
    ctx.set_rank(1)
    lists, _ = ctx.search(BOX, EXIST)
    return lists.copy()


@pytest.fixture(scope="module")
def bases():
    return [synth.kinect_scene(1_000_000, grid=G, leaf=LEAF, seed=synth.BASE_SEED + 1300 + s) for s in range(8)]


def _variant(torch, base_dev, k):
    """Frame k of a base scene: colours XOR-masked, x shifted by k whole cells (float64 add,
    rounded to float32 -- the same arithmetic numpy does for the oracle's copy)."""
    t = base_dev.clone()
    bits = t[:, 3].view(torch.int32)
    t[:, 3] = (bits ^ ((k * 0x2F1D37) & 0xFFFFFF)).view(torch.float32)
    t[:, 0] = (t[:, 0].double() + k * LEAF).float()
    return t


def _variant_host(base, k):
    pts = base.copy()
    pts[:, 3] = (pts[:, 3].view(np.uint32) ^ np.uint32((k * 0x2F1D37) & 0xFFFFFF)).view(np.float32)
    pts[:, 0] = (pts[:, 0].astype(np.float64) + k * LEAF).astype(np.float32)
    return pts


def test_config4_512_frames_points_in(ctx, bases):
    import torch
    dev = torch.device("cuda", 0)
    bdev = [torch.from_numpy(b).to(dev) for b in bases]
    nfr = 512
    frames = [_variant(torch, bdev[i % 8], i // 8) for i in range(nfr)]
    torch.cuda.synchronize()
    axis_t, var, axis_q = synth.random_bases(981, D, 1, R, seed=synth.BASE_SEED + 31)
    ap = synth.whiten(axis_t, var)
    ctx.search_setup(axis_t, var, axis_q)
    ctx.set_rank(1)
    ctx.set_batch(32)
    ctx.set_pipeline(True)
    d_out = torch.zeros((nfr, 3), dtype=torch.int64, device=dev)
    nm, info = ctx.run_point_frames(frames, LEAF, (G,) * 3, 981, THR, S, BOX, EXIST, True, d_out)
    assert nm == 1
    got = d_out.cpu().numpy().view(c3hlac.DET_DTYPE).reshape(nfr, 1)
    assert (info["status"] == 0).all(), np.flatnonzero(info["status"])
    assert (info["div_b"] == G).all()
    assert np.array_equal(info["min_b"][:, 0], np.arange(nfr) // 8)  # the x shift moves min_b
    assert (info["subdiv_b"] == 13).all()
    assert (got["score"] > 0).all()
    # the oracle from the points, every 4th frame
    P = (-(-G // S) - BOX[0] + 1,) * 3

    def oracle(i):
        pts = _variant_host(bases[i % 8], i // 8)
        g, layout, cloud = po.voxelize(pts, LEAF)
        fe, sb, _ = po.c3hlac(g, layout, cloud, 981, THR, LEAF, S, exact=True)
        ex = po.exist(fe)
        L, _, sc = po.search(sb, fe, ex, ap, axis_q, BOX, 1, EXIST, dbl=True, want_scores=True)
        return i, g, cloud, sc

    with cf.ThreadPoolExecutor(8) as pool:  # the C oracle releases the GIL
        for i, g, cloud, sc in pool.map(oracle, range(1, nfr, 4)):  # 128 of the 512 frames
            assert list(info["div_b"][i]) == list(g.div_b) and list(info["min_b"][i]) == list(g.min_b), i
            assert info["n_valid"][i] == g.n_valid and info["n_occ"][i] == g.n_occ == len(cloud), i
            e = got[i, 0]
            p = (int(e["z"]) * P[1] + int(e["y"])) * P[0] + int(e["x"])
            best = int(np.argmax(sc))
            assert int(e["mode"]) == 0
            assert abs(float(e["score"]) - sc[p]) <= RTOL * sc[p], (i, float(e["score"]), sc[p])
            if p != best:
                assert sc[p] >= sc[best] * (1 - 2 * RTOL), (i, p, best)
    # the single-frame path gives the same records (bit-identical)
    for i in range(0, nfr, 37):
        ref = _single(ctx, frames[i])
        assert np.array_equal(got[i], ref[:, 0]), i


def test_host_frames_equal_device_frames(ctx, bases):
    import torch
    dev = torch.device("cuda", 0)
    nfr = 40
    host = [_variant_host(bases[i % 8], 3 + i // 8) for i in range(nfr)]
    devf = [torch.from_numpy(h).to(dev) for h in host]
    torch.cuda.synchronize()
    axis_t, var, axis_q = synth.random_bases(981, D, 2, R, seed=synth.BASE_SEED + 32)
    ctx.search_setup(axis_t, var, axis_q)
    ctx.set_rank(1)
    ctx.set_batch(16)
    a = torch.zeros((nfr, 6), dtype=torch.int64, device=dev)
    b = torch.zeros((nfr, 6), dtype=torch.int64, device=dev)
    _, ia = ctx.run_point_frames(host, LEAF, (G,) * 3, 981, THR, S, BOX, EXIST, True, a)
    _, ib = ctx.run_point_frames(devf, LEAF, (G,) * 3, 981, THR, S, BOX, EXIST, True, b)
    assert np.array_equal(a.cpu().numpy(), b.cpu().numpy())
    assert np.array_equal(ia, ib)
    ctx.set_batch(32)


def test_mixed_geometries_in_one_batch(ctx, bases):
    """Frames of different extents / origins share one canvas; each frame's positions are
    bounded by its own subdivisions.  Statuses: 0 batched (a centroid near a cell boundary
    too: the exact pass), 1 recomputed on the single-frame path (beyond the canvas, empty)."""
    import torch
    dev = torch.device("cuda", 0)
    axis_t, var, axis_q = synth.random_bases(117, D, 3, R, seed=synth.BASE_SEED + 33)
    ctx.search_setup(axis_t, var, axis_q)
    ctx.set_rank(1)
    ctx.set_batch(8)
    frames, expect_status = [], []
    for i in range(20):
        pts = _variant_host(bases[i % 8], i)[2:]  # no sentinels: the extent is the scene's own
        kind = i % 5
        if kind == 1:  # only near points: a smaller grid, another min_b
            pts = pts[np.isfinite(pts[:, 2]) & (pts[:, 2] < np.float32(0.55 * G * LEAF))]
        elif kind == 2:  # a slab of x
            pts = pts[np.isfinite(pts[:, 0]) & (pts[:, 0] > np.float32((i + 20) * LEAF))]
        frames.append(np.ascontiguousarray(pts))
        expect_status.append(0)
    far = frames[0].copy()
    fin = np.flatnonzero(np.isfinite(far[:, 0]))
    far[fin[0], :3] = far[fin[1], :3] + np.float32(140 * LEAF)  # extent beyond the 128 canvas
    frames.append(far)
    expect_status.append(1)
    frames.append(np.full((1000, 4), np.nan, np.float32))  # no valid point
    expect_status.append(1)
    edge = frames[3].copy()  # a point right on a cell face: its voxel's centroid is flagged,
    k = np.flatnonzero(np.isfinite(edge[:, 0]))[7]  # summed exactly in the batch (round 4)
    edge[k, 0] = np.float32(np.floor(edge[k, 0] / np.float32(LEAF)) * np.float32(LEAF))
    frames.append(edge)
    expect_status.append(0)
    nfr = len(frames)
    devf = [torch.from_numpy(f).to(dev) for f in frames]
    torch.cuda.synchronize()
    d_out = torch.zeros((nfr, 9), dtype=torch.int64, device=dev)
    _, info = ctx.run_point_frames(devf, LEAF, (G,) * 3, 117, THR, S, BOX, EXIST, True, d_out)
    got = d_out.cpu().numpy().view(c3hlac.DET_DTYPE).reshape(nfr, 3)
    assert list(info["status"]) == expect_status, info["status"]
    assert len(set(map(tuple, info["div_b"][:20]))) > 2  # the geometries differ
    for i in range(nfr):
        if i == nfr - 2:  # empty frame: fresh setRank lists
            assert (got[i]["score"] == 0).all()
            continue
        ref = _single(ctx, devf[i], variant=117)
        assert np.array_equal(got[i], ref[:, 0]), (i, got[i], ref[:, 0])
        gi = ctx.info
        assert list(info["div_b"][i]) == list(gi.div_b) and list(info["min_b"][i]) == list(gi.min_b), i
        assert info["n_occ"][i] == gi.n_occ
    ctx.set_batch(32)


def test_centroid_rounding_past_a_full_canvas(ctx):
    """A frame whose extent fills the canvas (32^3 at leaf 0.01) with a voxel in the last
    x cell whose three points' fp32 centroid rounds up onto the face x = 32 * leaf: the
    reference counts it in subdivision 5 of 6 ((32 - 0) % 6 != 0, c3_hlac.cpp:349-362), the
    batch's canvas maps have no cell 32, so the frame must leave the batch (status 1) and
    give the single-frame path's records; a control frame without that voxel stays batched."""
    import torch
    dev = torch.device("cuda", 0)
    f32 = np.float32
    leaf = f32(0.01)
    rng = np.random.default_rng(5)
    xyz = (rng.integers(0, 32, (4000, 3)) + rng.random((4000, 3)) * 0.8 + 0.1).astype(f32) * leaf
    special = np.array([31, 10, 12])
    cells = np.floor(xyz * (f32(1) / leaf)).astype(int)
    xyz = xyz[~(cells == special).all(1)]
    corners = np.array([[0.5, 0.5, 0.5], [31.5, 31.5, 31.5]], f32) * leaf  # extent 0..31 on every axis
    x_face = f32(0.31999996)  # 3 points: fp32 sum * fl(1/3) = 0.32 -> floor(c / leaf) = 32
    pts3 = np.array([[x_face, (10.5 * leaf), (12.5 * leaf)]] * 3, f32)
    col = rng.integers(0, 256, (len(xyz) + 5, 3))
    rgb = synth.pack_rgb(col[:, 0], col[:, 1], col[:, 2])

    def cloud(with_special):
        p = np.concatenate([xyz, corners] + ([pts3] if with_special else []), 0)
        return np.ascontiguousarray(np.concatenate([p, rgb[:len(p), None]], 1), f32)

    frames = [cloud(True), cloud(False)]
    g, layout, cl = po.voxelize(frames[0], float(leaf))
    assert list(g.div_b) == [32, 32, 32] and list(g.min_b) == [0, 0, 0]
    occ = np.flatnonzero(layout >= 0)
    k = occ[np.flatnonzero(occ == special[0] + 32 * (special[1] + 32 * special[2]))[0]]
    assert int(np.floor(cl[layout[k], 0] / leaf)) == 32  # the case under test is there
    axis_t, var, axis_q = synth.random_bases(117, 24, 2, 6, seed=41)
    ctx.search_setup(axis_t, var, axis_q)
    ctx.set_rank(1)
    ctx.set_batch(8)
    devf = [torch.from_numpy(f).to(dev) for f in frames]
    torch.cuda.synchronize()
    d_out = torch.zeros((2, 6), dtype=torch.int64, device=dev)
    _, info = ctx.run_point_frames(devf, float(leaf), (32, 32, 32), 117, THR, 6, BOX, 0, True, d_out)
    got = d_out.cpu().numpy().view(c3hlac.DET_DTYPE).reshape(2, 2)
    assert list(info["status"]) == [1, 0], info
    for i in range(2):
        ctx.voxelize(devf[i], float(leaf))
        ctx.extract(117, THR, 6)
        ctx.set_rank(1)
        ref, _ = ctx.search(BOX, 0)
        assert np.array_equal(got[i], ref[:, 0]), (i, got[i], ref[:, 0])
    # the single-frame path on the special frame against the oracle's exact features
    ctx.voxelize(devf[0], float(leaf))
    ctx.extract(117, THR, 6)
    fe, _, _ = po.c3hlac(g, layout, cl, 117, THR, float(leaf), 6, exact=True)
    assert np.array_equal(ctx.features(), fe)
    ctx.set_batch(32)


def test_points_in_256_canvas_overlap_and_repeat(ctx):
    """256^3 canvases (C3-HLAC-117 + 3 models): the batch scatter stamps the tick's tiles
    (no occupancy stream), the voxeliser runs on its own stream beside the tick.  Two calls
    on one context (the second reuses the buffer sets, epochs and word lists of the first)
    give identical records, and sampled frames equal the single-frame path bit for bit."""
    import torch
    dev = torch.device("cuda", 0)
    g2, leaf2 = 256, 0.01
    base = [synth.kinect_scene(1_000_000, grid=g2, leaf=leaf2, seed=synth.BASE_SEED + 1400 + s) for s in range(3)]
    bdev = [torch.from_numpy(b).to(dev) for b in base]
    nfr = 40
    frames = []
    for i in range(nfr):
        t = bdev[i % 3].clone()
        t[:, 3] = (t[:, 3].view(torch.int32) ^ ((i * 0x2F1D37) & 0xFFFFFF)).view(torch.float32)
        t[:, 0] = (t[:, 0].double() + (i % 5) * leaf2).float()
        frames.append(t)
    torch.cuda.synchronize()
    axis_t, var, axis_q = synth.random_bases(117, D, 3, R, seed=synth.BASE_SEED + 34)
    ctx.search_setup(axis_t, var, axis_q)
    ctx.set_rank(1)
    ctx.set_batch(16)
    a = torch.zeros((nfr, 9), dtype=torch.int64, device=dev)
    b = torch.zeros((nfr, 9), dtype=torch.int64, device=dev)
    _, ia = ctx.run_point_frames(frames, leaf2, (g2,) * 3, 117, THR, S, BOX, EXIST, True, a)
    _, ib = ctx.run_point_frames(frames[::-1], leaf2, (g2,) * 3, 117, THR, S, BOX, EXIST, True, b)
    assert (ia["status"] == 0).all(), ia["status"]
    ga = a.cpu().numpy().view(c3hlac.DET_DTYPE).reshape(nfr, 3)
    gb = b.cpu().numpy().view(c3hlac.DET_DTYPE).reshape(nfr, 3)
    assert np.array_equal(ga, gb[::-1])
    assert (ga["score"] > 0).all()
    for i in (0, 7, 13, 22, 39):
        ctx.voxelize(frames[i], leaf2, float("inf"))
        ctx.extract(117, THR, S)
        ctx.set_rank(1)
        ref, _ = ctx.search(BOX, EXIST)
        assert np.array_equal(ga[i], ref[:, 0]), (i, ga[i], ref[:, 0])
    ctx.set_batch(32)


def test_records_do_not_depend_on_batch_size_or_prepared_frames(ctx, bases):
    """The same 96 frames at 32 and at 64 frames per batch (Context.point_batch's two
    choices), as a list and as a PointFrames: identical detection records and frame info."""
    import torch
    dev = torch.device("cuda", 0)
    bdev = [torch.from_numpy(b).to(dev) for b in bases]
    nfr = 96
    frames = [_variant(torch, bdev[i % 8], 3 + i // 8) for i in range(nfr)]
    axis_t, var, axis_q = synth.random_bases(981, D, 1, R, seed=synth.BASE_SEED + 31)
    ctx.search_setup(axis_t, var, axis_q)
    ctx.set_rank(1)
    ctx.set_pipeline(True)
    outs, infos = [], []
    for batch, prepared in ((32, False), (64, True), (32, True)):
        ctx.set_batch(batch)
        d_out = torch.zeros((nfr, 3), dtype=torch.int64, device=dev)
        fr = ctx.prepare_point_frames(frames) if prepared else frames
        _, info = ctx.run_point_frames(fr, LEAF, (G,) * 3, 981, THR, S, BOX, EXIST, True, d_out)
        outs.append(d_out.cpu())
        infos.append(info)
    assert (infos[0]["status"] == 0).all()
    assert (outs[0][:, 0].numpy().view(np.float64) > 0).all()
    for o, inf in zip(outs[1:], infos[1:]):
        assert torch.equal(o, outs[0])
        assert np.array_equal(inf, infos[0])


def test_z_limit_in_the_batch(ctx, bases):
    """limitPoint's depth cut (detect_object.cpp:68-87) inside the batch: 12 frames with
    z_limit at 60 % of the scene depth give the single-frame path's records and geometry
    with the same cut, and frame 0's grid geometry and voxel count equal the oracle's."""
    import torch
    dev = torch.device("cuda", 0)
    axis_t, var, axis_q = synth.random_bases(981, D, 1, R, seed=synth.BASE_SEED + 31)
    ctx.search_setup(axis_t, var, axis_q)
    ctx.set_rank(1)
    ctx.set_batch(8)
    frames = [np.ascontiguousarray(_variant_host(bases[i % 8], i)) for i in range(12)]
    z = frames[0][:, 2]
    zl = float(np.float32(np.nanmin(z[np.isfinite(z)]) + 0.6 * (np.nanmax(z[np.isfinite(z)]) -
                                                                  np.nanmin(z[np.isfinite(z)]))))
    devf = [torch.from_numpy(f).to(dev) for f in frames]
    d_out = torch.zeros((len(frames), 3), dtype=torch.int64, device=dev)
    _, info = ctx.run_point_frames(devf, LEAF, (G,) * 3, 981, THR, S, BOX, EXIST, True, d_out, z_limit=zl)
    got = d_out.cpu().numpy().view(c3hlac.DET_DTYPE).reshape(len(frames), 1)
    assert (info["status"] == 0).all(), info["status"]
    g, layout, _ = po.voxelize(frames[0], LEAF, zl)
    assert list(info["div_b"][0]) == list(g.div_b) and list(info["min_b"][0]) == list(g.min_b)
    assert info["n_occ"][0] == (layout >= 0).sum()
    for i in range(len(frames)):
        ref = _single(ctx, devf[i], z_limit=zl)
        assert np.array_equal(got[i], ref[:, 0]), (i, got[i], ref[:, 0])
        assert list(info["div_b"][i]) == list(ctx.info.div_b), i
    ctx.set_batch(32)
