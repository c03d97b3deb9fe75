"""GPU parity tests: the HIP path through the C-ABI against the oracle and the golden
fixtures.  Integer/index outputs must be bit-exact; features are compared bit-exactly
with the oracle's exact-integer mode and within 1e-4 relative with its fp32-faithful
mode; scores within the tolerances stated per test."""
import numpy as np
import pytest

import c3hlac
import np_ref as npr
import pyoracle as po
from c3hlac import synth
from conftest import GOLDEN_CASES, THR, load_golden

pytestmark = pytest.mark.gpu

SCORE_RTOL_F64 = 1e-5   # GPU (fp32, direct box sums) vs the float64 oracle
SCORE_RTOL_F32 = 1e-4   # vs the reference-order fp32 oracle (summed-volume table error)


def _words_xyz(ctx):
    d = ctx.info.div_b
    return ctx.grid().reshape(d[2], d[1], d[0])


@pytest.mark.parametrize("name", GOLDEN_CASES)
def test_golden_voxelize(ctx, name):
    z = load_golden(name)
    gi = ctx.voxelize(z["pts"], float(z["leaf"]), float(z["z_limit"]))
    assert list(gi.div_b) == list(z["div_b"]) and list(gi.min_b) == list(z["min_b"])
    assert gi.n_occ == z["cloud"].shape[0]
    assert np.array_equal(ctx.grid(), z["grid_words"])
    assert np.array_equal(ctx.leaf_layout(), z["leaf_layout"])
    ds = ctx.downsampled()  # centroids: fp32 sequential sums in input order, bit-exact
    assert np.array_equal(ds.view(np.uint32), z["cloud"].view(np.uint32))


@pytest.mark.parametrize("name", GOLDEN_CASES)
@pytest.mark.parametrize("variant", [981, 117])
def test_golden_extract(ctx, name, variant):
    z = load_golden(name)
    ctx.voxelize(z["pts"], float(z["leaf"]), float(z["z_limit"]))
    sb, hn = ctx.extract(variant, tuple(z["thr"]), int(z["subdiv"]), tuple(z["offset"]))
    assert tuple(sb) == tuple(z["subdiv_b"])
    f = ctx.features()
    assert np.array_equal(f, z["feat%d_exact" % variant])
    np.testing.assert_allclose(f, z["feat%d_faithful" % variant], rtol=1e-4)
    assert np.array_equal(ctx.exist(), z["exist"])


@pytest.mark.parametrize("name", [n for n in GOLDEN_CASES if n != "kinect_32_whole"])
def test_golden_search(ctx, name):
    z = load_golden(name)
    ctx.voxelize(z["pts"], float(z["leaf"]), float(z["z_limit"]))
    ctx.extract(981, tuple(z["thr"]), int(z["subdiv"]), tuple(z["offset"]))
    ctx.search_setup(z["axis_t"], z["var"], z["axis_q"])
    ctx.set_rank(int(z["rank"]))
    lists, nm = ctx.search(tuple(z["ranges"]), int(z["thr_exist"]), rotate=True)
    sc = ctx.scores()
    ref = z["scores_f64"]
    assert sc.shape == ref.shape
    assert np.array_equal(sc < 0, ref < 0)  # identical exist gate
    ok = ref > 0
    np.testing.assert_allclose(sc[ok], ref[ok], rtol=SCORE_RTOL_F64)
    np.testing.assert_allclose(sc[ok], z["scores_f32"][ok], rtol=SCORE_RTOL_F32)
    # the GPU's rank lists are exactly the reference replay of its own scores
    _assert_replay_matches(ctx, tuple(z["ranges"]), int(z["rank"]), lists)
    np.testing.assert_allclose(lists["score"], z["lists_f64"][:, :, 0], rtol=SCORE_RTOL_F64)


def _assert_replay_matches(ctx, ranges, rank, lists, prior=None, rotate=True):
    sc = ctx.scores()
    M = lists.shape[0]
    xn, yn, zn = ctx.subdiv
    ms, off = [], 0
    for mode in npr.mode_schedule(ranges, rotate):
        xr, yr, zr = npr._ranges(mode, ranges)
        xe, ye, ze = xn - xr + 1, yn - yr + 1, zn - zr + 1
        if xe <= 0 or ye <= 0 or ze <= 0:
            continue
        P = xe * ye * ze
        ms.append((mode, xe, ye, sc[off:off + M * P].reshape(M, P)))
        off += M * P
    nl = npr.replay(ms, ranges, rank, prior)
    got = [[(float(e["score"]), int(e["x"]), int(e["y"]), int(e["z"]), int(e["mode"])) for e in m] for m in lists]
    assert got == [[tuple(e) for e in m] for m in nl]


@pytest.mark.parametrize("variant", [981, 117])
@pytest.mark.parametrize("subdiv,offset", [(10, (0, 0, 0)), (7, (2, 1, 3)), (0, (0, 0, 0)), (3, (0, 0, 0)),
                                           (20, (0, 0, 0)), (25, (1, 0, 2)), (16, (0, 0, 0)), (17, (0, 0, 0)),
                                           (40, (1, 1, 1))])
def test_extract_subdivision_cases(ctx, variant, subdiv, offset):
    """Single-tile, multi-tile (64-bit partials), whole-grid and hist_num==1 paths."""
    pts = synth.parity_cloud(9000, grid=30, leaf=0.01, seed=7)
    g, layout, cloud = po.voxelize(pts, 0.01)
    ctx.voxelize(pts, 0.01)
    sb, hn = ctx.extract(variant, THR, subdiv, offset)
    fe, sbo, hno = po.c3hlac(g, layout, cloud, variant, THR, 0.01, subdiv, offset, exact=True)
    assert tuple(sb) == tuple(sbo) and hn == hno
    assert np.array_equal(ctx.features(), fe)
    fa, _, _ = po.c3hlac(g, layout, cloud, 981, THR, 0.01, subdiv, offset, exact=False)
    assert np.array_equal(ctx.exist(), po.exist(fa))


@pytest.mark.parametrize("k", range(13))
def test_kat_pair_per_offset(ctx, k):
    rel = npr.REL[k]
    words = np.zeros((3, 3, 3), np.uint32)
    c1, c2 = (200, 30, 149), (10, 250, 147)
    words[1, 1, 1] = (1 << 24) | (c1[0] << 16) | (c1[1] << 8) | c1[2]
    words[1 + rel[2], 1 + rel[1], 1 + rel[0]] = (1 << 24) | (c2[0] << 16) | (c2[1] << 8) | c2[2]
    ctx.set_grid(words.reshape(-1), (3, 3, 3))
    for variant in (981, 117):
        ctx.extract(variant, THR, 0)
        fn, ex, _ = npr.c3hlac(words, variant, THR, 0)
        assert np.array_equal(ctx.features(), fn)


@pytest.mark.parametrize("color_mode", [c3hlac.COLOR_C3_DOUBLE, c3hlac.COLOR_C3_FLOAT, c3hlac.COLOR_CHLAC])
def test_colour_255_lut_flag(ctx, color_mode):
    """v = 255 under every setColor table (C3 double: (254, 0), C3 float: (255, 0),
    ColorCHLAC: (255, 0)), against the numpy restatement."""
    words = synth.random_words(12, 0.5, seed=5, colour_max=255)
    words[words != 0] |= np.uint32(0xFF0000)  # force r = 255
    ctx.set_grid(words.reshape(-1), (12, 12, 12))
    for variant in (981, 117):
        ctx.extract(variant, THR, 4, color_mode=color_mode)
        fn, ex, _ = npr.c3hlac(words, variant, THR, 4, color_mode=color_mode)
        assert np.array_equal(ctx.features(), fn)


@pytest.mark.parametrize("color_mode", [c3hlac.COLOR_C3_FLOAT, c3hlac.COLOR_CHLAC])
def test_colour_modes_random_grids(ctx, color_mode):
    """The other setColor tables on random colours, every variant / subdivision shape, on
    the tile kernels and (dense) the matrix-core body."""
    for occ, dims in ((0.05, (33, 27, 21)), (1.0, (24, 24, 24))):
        words = synth.random_words(dims, occ, seed=17, colour_max=255)
        ctx.set_grid(words.reshape(-1), dims)
        for variant, S, off in ((981, 10, (0, 0, 0)), (117, 6, (1, 2, 3)), (117, 0, (0, 0, 0))):
            ctx.extract(variant, (100, 200, 50), S, off, color_mode=color_mode)
            fn, ex, _ = npr.c3hlac(words, variant, (100, 200, 50), S, off, color_mode=color_mode)
            assert np.array_equal(ctx.features(), fn), (occ, variant, S, off)
            assert np.array_equal(ctx.exist(), ex)


def test_colour_mode_rejected(ctx):
    words = synth.random_words(8, 0.5, seed=5)
    ctx.set_grid(words.reshape(-1), (8, 8, 8))
    with pytest.raises(c3hlac.C3HError):
        ctx.extract(117, THR, 4, color_mode=3)


@pytest.mark.parametrize("occ", [0.02, 0.3, 1.0])
def test_random_grids_vs_numpy(ctx, occ):
    words = synth.random_words((37, 29, 23), occ, seed=int(occ * 100) + 1, colour_max=255)
    ctx.set_grid(words.reshape(-1), (37, 29, 23))
    for variant, S, off in ((981, 10, (0, 0, 0)), (117, 6, (1, 2, 3)), (981, 0, (0, 0, 0))):
        ctx.extract(variant, (100, 200, 50), S, off)
        fn, ex, _ = npr.c3hlac(words, variant, (100, 200, 50), S, off)
        assert np.array_equal(ctx.features(), fn)
        assert np.array_equal(ctx.exist(), ex)


def test_edge_cases(ctx):
    # empty cloud / all NaN: empty grid; subdiv > 0 -> setVoxelFilter fails -> no features
    nan = np.full((10, 4), np.nan, np.float32)
    gi = ctx.voxelize(nan, 0.01)
    assert gi.n_valid == 0 and gi.n_occ == 0
    sb, hn = ctx.extract(981, THR, 10)
    assert hn == 0
    sb, hn = ctx.extract(981, THR, 0)
    assert hn == 1 and not ctx.features().any()
    # single point
    one = np.array([[0.123, -0.456, 0.789, synth.pack_rgb(10, 200, 30)]], np.float32)
    gi = ctx.voxelize(one, 0.01)
    assert gi.n_occ == 1 and list(gi.div_b) == [1, 1, 1]
    ctx.extract(981, THR, 0)
    g, layout, cloud = po.voxelize(one, 0.01)
    fe, _, _ = po.c3hlac(g, layout, cloud, 981, THR, 0.01, 0, exact=True)
    assert np.array_equal(ctx.features(), fe)
    # offsets >= grid and negative thresholds: the reference's silent empty output
    pts = synth.parity_cloud(500, grid=8, leaf=0.01, seed=3)
    ctx.voxelize(pts, 0.01)
    assert ctx.extract(981, THR, 4, (8, 0, 0))[1] == 0
    assert ctx.extract(981, (-1, 0, 0), 4)[1] == 0
    # z limit drops points
    gi = ctx.voxelize(pts, 0.01, z_limit=0.04)
    g, layout, cloud = po.voxelize(pts, 0.01, 0.04)
    assert gi.n_valid == g.n_valid and np.array_equal(ctx.leaf_layout(), layout)


def test_multipoint_voxel_colour_mean(ctx):
    rng = np.random.default_rng(5)
    n = 20000
    cells = rng.integers(0, 6, (n, 3))
    xyz = ((cells + 0.1 + 0.8 * rng.random((n, 3))) * 0.01).astype(np.float32)
    col = rng.integers(0, 256, (n, 3))
    pts = np.concatenate([xyz, synth.pack_rgb(col[:, 0], col[:, 1], col[:, 2])[:, None]], 1).astype(np.float32)
    ctx.voxelize(pts, 0.01)
    g, layout, cloud = po.voxelize(pts, 0.01)
    d = g.div_b
    assert np.array_equal(ctx.leaf_layout(), layout)
    words = ctx.grid()
    occ = layout >= 0
    exp = (1 << 24) | cloud[layout[occ], 3].view(np.uint32)
    assert np.array_equal(words[occ], exp) and not words[~occ].any()
    ds = ctx.downsampled()
    assert np.array_equal(ds.view(np.uint32), cloud.view(np.uint32))


def test_voxel_table_regrows(ctx):
    """The single-frame voxeliser accumulates into toroidal arrays of 2^tb cells per axis
    sized by the frames so far (round 5; 128^3 at first): a frame whose extent exceeds them
    on any axis runs again on dims that fit it.  Small, large (400k scattered points), long
    (300 cells in x, then 270 in y and 160 in z) and small frames again: the grid, colours
    and downsampled cloud are the oracle's after every change of dims."""
    rng = np.random.default_rng(11)

    def cloud(n, span):
        xyz = (rng.random((n, 3)) * np.asarray(span, np.float64)).astype(np.float32)
        col = rng.integers(0, 256, (n, 3))
        return np.concatenate([xyz, synth.pack_rgb(col[:, 0], col[:, 1], col[:, 2])[:, None]], 1).astype(np.float32)

    for pts in (cloud(2000, 0.05), cloud(400_000, 1.0), cloud(3000, 0.08), cloud(50_000, (3.0, 0.2, 0.2)),
                cloud(60_000, (0.2, 2.7, 1.6)), cloud(1500, 0.04)):
        gi = ctx.voxelize(pts, 0.01)
        g, layout, cl = po.voxelize(pts, 0.01)
        assert list(gi.div_b) == list(g.div_b) and gi.n_occ == (layout >= 0).sum()
        assert np.array_equal(ctx.leaf_layout(), layout)
        words = ctx.grid()
        occ = layout >= 0
        assert np.array_equal(words[occ], (1 << 24) | cl[layout[occ], 3].view(np.uint32)) and not words[~occ].any()
        assert np.array_equal(ctx.downsampled().view(np.uint32), cl.view(np.uint32))


def _assert_pick(m, got, sb, feats, scd, Ld, L32):
    """The GPU's rank-1 position of model m against the oracles (search.cpp:464-474: the
    strict '>' over the scan order (mode, z, y, x) keeps the first of equal scores).

    Accepted when it is the float64 oracle's pick, or:
    (a) both boxes hold bit-identical feature sums (exact tie: the GPU's direct box sums
        give equal scores, so the strict '>' keeps the earlier scan position -- the GPU's
        must come first; the oracle's float64 summed-volume table differences break such a
        tie by rounding: config 3's model 7, (7, 12, 17) vs (7, 13, 17), 3.5e-16 apart, moved
        with round 4's PCL-1.0 centroid semantics, which changed the oracle's rounding, not
        the boxes: they are equal under both semantics); or
    (b) it is the fp32-reference-order oracle's pick; or
    (c) the two float64 scores differ by < 1e-5 relative (a tie within the stated tolerance)."""
    best = Ld.records()[m][0]
    if got == tuple(best[1:4]):
        return
    e = sb[0] - 1
    pg = (got[2] * e + got[1]) * e + got[0]
    pb = (best[3] * e + best[2]) * e + best[1]
    gap = (scd[pb] - scd[pg]) / scd[pb]
    F = feats.reshape(sb[2], sb[1], sb[0], -1).astype(np.float64)
    box = lambda x, y, z: F[z:z + 2, y:y + 2, x:x + 2].sum(axis=(0, 1, 2))  # noqa: E731
    exact_tie = np.array_equal(box(*got), box(*best[1:4]))
    f32 = tuple(L32.records()[m][0][1:4]) if L32 is not None else None
    ok = (exact_tie and pg < pb) or got == f32 or abs(gap) < 1e-5
    assert ok, ("model %d: GPU %s, f64 oracle %s, fp32 oracle %s, f64 gap %.3g, exact tie %s"
                % (m, got, tuple(best[1:4]), f32, gap, exact_tie))


def test_config2_kinect_128(ctx):
    """Config 2: 1M-pt Kinect-style scene, 128^3, C3-HLAC-981 + 1-model search."""
    pts = synth.kinect_scene(1_000_000, grid=128, leaf=0.02, seed=synth.BASE_SEED)
    g, layout, cloud = po.voxelize(pts, 0.02)
    gi = ctx.voxelize(pts, 0.02)
    assert list(gi.div_b) == [128, 128, 128] and gi.n_occ == g.n_occ
    assert np.array_equal(ctx.leaf_layout(), layout)
    sb, hn = ctx.extract(981, THR, 10)
    fe, sbo, _ = po.c3hlac(g, layout, cloud, 981, THR, 0.02, 10, exact=True)
    ff, _, _ = po.c3hlac(g, layout, cloud, 981, THR, 0.02, 10, exact=False)
    f = ctx.features()
    assert np.array_equal(f, fe)
    np.testing.assert_allclose(f, ff, rtol=1e-4)
    ex = ctx.exist()
    assert np.array_equal(ex, po.exist(ff))
    axis_t, var, axis_q = synth.random_bases(981, 100, 1, 20, seed=1)
    ctx.search_setup(axis_t, var, axis_q)
    ctx.set_rank(1)
    ctx.clean_max()
    lists, nm = ctx.search((2, 2, 2), 100)
    Ld, _, scd = po.search(sb, ff, ex, synth.whiten(axis_t, var), axis_q, (2, 2, 2), 1, 100, dbl=True,
                           want_scores=True)
    L32, _, sc32 = po.search(sb, ff, ex, synth.whiten(axis_t, var), axis_q, (2, 2, 2), 1, 100, dbl=False,
                             want_scores=True)
    sc = ctx.scores()
    assert np.array_equal(sc < 0, scd < 0)
    ok = scd > 0
    np.testing.assert_allclose(sc[ok], scd[ok], rtol=SCORE_RTOL_F64)
    np.testing.assert_allclose(sc[ok], sc32[ok], rtol=SCORE_RTOL_F32)
    got = (int(lists[0, 0]["x"]), int(lists[0, 0]["y"]), int(lists[0, 0]["z"]))
    _assert_pick(0, got, sb, ff, scd, Ld, L32)
    _assert_replay_matches(ctx, (2, 2, 2), 1, lists)


def test_config3_kinect_256_ri117_multimodel(ctx):
    """Config 3: 256^3, RI-117, compress 117->100, 10 models x r=20, v2-style rank = M."""
    pts = synth.kinect_scene(1_000_000, grid=256, leaf=0.01, seed=synth.BASE_SEED + 1)
    g, layout, cloud = po.voxelize(pts, 0.01)
    gi = ctx.voxelize(pts, 0.01)
    assert list(gi.div_b) == [256, 256, 256]
    sb, hn = ctx.extract(117, THR, 10)
    assert sb == (26, 26, 26)
    fe, _, _ = po.c3hlac(g, layout, cloud, 117, THR, 0.01, 10, exact=True)
    f = ctx.features()
    assert np.array_equal(f, fe)
    f981, _, _ = po.c3hlac(g, layout, cloud, 981, THR, 0.01, 10, exact=False)
    ex = po.exist(f981)
    assert np.array_equal(ctx.exist(), ex)
    M = 10
    axis_t, var, axis_q = synth.random_bases(117, 100, M, 20, seed=2)
    ctx.search_setup(axis_t, var, axis_q)
    ctx.set_rank(M)
    ctx.clean_max()
    lists, nm = ctx.search((2, 2, 2), 100)
    Ld, _, scd = po.search(sb, f, ex, synth.whiten(axis_t, var), axis_q, (2, 2, 2), M, 100, dbl=True,
                           want_scores=True)
    sc = ctx.scores()
    assert np.array_equal(sc < 0, scd < 0)
    ok = scd > 0
    np.testing.assert_allclose(sc[ok], scd[ok], rtol=SCORE_RTOL_F64)
    _assert_replay_matches(ctx, (2, 2, 2), M, lists)
    # same detections as the float64 oracle (top entry of every model); the one pick that
    # differs is an exact tie (model 7, see _assert_pick)
    L32, _, _ = po.search(sb, f, ex, synth.whiten(axis_t, var), axis_q, (2, 2, 2), M, 100, dbl=False)
    scm = scd.reshape(M, -1)
    for m in range(M):
        got = (int(lists[m, 0]["x"]), int(lists[m, 0]["y"]), int(lists[m, 0]["z"]))
        _assert_pick(m, got, sb, f, scm[m], Ld, L32)


@pytest.mark.parametrize("ranges", [(1, 2, 1), (1, 2, 3), (2, 1, 1), (3, 3, 1)])
def test_rotation_modes_and_rank(ctx, ranges):
    pts = synth.kinect_scene(300_000, grid=96, leaf=0.02, seed=77)
    ctx.voxelize(pts, 0.02)
    sb, hn = ctx.extract(981, THR, 8)
    f = ctx.features()
    ex = ctx.exist()
    axis_t, var, axis_q = synth.random_bases(981, 40, 3, 8, seed=9)
    ctx.search_setup(axis_t, var, axis_q)
    ctx.set_rank(4)
    lists, nm = ctx.search(ranges, 50)
    assert nm == len(npr.mode_schedule(ranges, True))
    _assert_replay_matches(ctx, ranges, 4, lists)
    Ld, _, scd = po.search(sb, f, ex, synth.whiten(axis_t, var), axis_q, ranges, 4, 50, dbl=True, want_scores=True)
    sc = ctx.scores()
    ok = scd > 0
    np.testing.assert_allclose(sc[ok], scd[ok], rtol=SCORE_RTOL_F64)
    # a second search continues from the current lists (no cleanMax): same semantics
    prior = [[(float(e["score"]), int(e["x"]), int(e["y"]), int(e["z"]), int(e["mode"])) for e in m] for m in lists]
    lists2, _ = ctx.search(ranges, 50)
    _assert_replay_matches(ctx, ranges, 4, lists2, prior=[[list(e) for e in m] for m in prior])
    # removeOverlap on the lists (SearchObjMulti) equals the host function
    ctx.clean_max()
    l3, _ = ctx.search(ranges, 50, remove_overlap=True)
    ctx.clean_max()
    l4, _ = ctx.search(ranges, 50, remove_overlap=False)
    assert np.array_equal(c3hlac.remove_overlap(l4, ranges), l3)


def test_search_after_a_frame_without_positions(ctx):
    """A frame whose subdivisions hold no box (xe, ye or ze < 1: searchPart runs no
    position) launches nothing; the next frame's sparse search must not inherit stale
    list counters (round 4: every later frame lost its records)."""
    axis_t, var, axis_q = synth.random_bases(117, 24, 3, 6, seed=17)
    ctx.search_setup(axis_t, var, axis_q)
    small = synth.kinect_scene(20_000, grid=12, leaf=0.02, seed=17)
    big = synth.kinect_scene(100_000, grid=40, leaf=0.02, seed=18)
    ctx.voxelize(small, 0.02)
    sb, _ = ctx.extract(117, THR, 6)
    assert min(sb) < 3, sb  # no 3 x 3 x 3 box fits
    ctx.set_rank(1)
    lists0, _ = ctx.search((3, 3, 3), 10)
    assert (lists0["score"] == 0).all()
    for _ in range(2):  # and again after a frame that did search
        ctx.voxelize(big, 0.02)
        sb, _ = ctx.extract(117, THR, 6)
        f, ex = ctx.features(), ctx.exist()
        ctx.set_rank(1)
        lists, _ = ctx.search((3, 3, 3), 10)
        L, _, scd = po.search(sb, f, ex, synth.whiten(axis_t, var), axis_q, (3, 3, 3), 1, 10, dbl=True,
                              want_scores=True)
        for m in range(3):
            want = L.records()[m][0][0]
            assert want > 0 and abs(float(lists[m, 0]["score"]) - want) <= SCORE_RTOL_F64 * want, (m, want)
        ctx.voxelize(small, 0.02)
        ctx.extract(117, THR, 6)
        ctx.set_rank(1)
        assert (ctx.search((3, 3, 3), 10)[0]["score"] == 0).all()


def test_search_without_rotation_and_feature_max(ctx):
    pts = synth.kinect_scene(200_000, grid=64, leaf=0.02, seed=5)
    ctx.voxelize(pts, 0.02)
    sb, hn = ctx.extract(117, THR, 5)
    f = ctx.features()
    ex = ctx.exist()
    fmax = f.max(0) * np.float32(0.75)
    fmax[3] = 0
    axis_t, var, axis_q = synth.random_bases(117, 30, 2, 6, seed=3)
    ctx.search_setup(axis_t, var, axis_q, feature_max=fmax)
    ctx.set_rank(2)
    lists, nm = ctx.search((1, 2, 3), 30, rotate=False)
    assert nm == 1
    Ld, _, scd = po.search(sb, f, ex, synth.whiten(axis_t, var), axis_q, (1, 2, 3), 2, 30, rotate=False,
                           dbl=True, fmax=fmax, want_scores=True)
    sc = ctx.scores()
    ok = scd > 0
    np.testing.assert_allclose(sc[ok], scd[ok], rtol=SCORE_RTOL_F64)
    _assert_replay_matches(ctx, (1, 2, 3), 2, lists, rotate=False)
    # D = 30 runs on 32 internal axes (two zero axes appended): the readback holds the
    # caller's 30, equal to the float64 compress of the normalised features
    G = ctx.compressed()
    assert G.shape == (hn, 30)
    fn = f.astype(np.float64)
    fn = np.where(fmax > 0, fn / np.where(fmax > 0, fmax, 1), 0.0)  # setData's normalisation (oracle)
    Gd = fn @ synth.whiten(axis_t, var).astype(np.float64).T
    live = ex > 0
    np.testing.assert_allclose(G[live], Gd[live], rtol=1e-4, atol=1e-4 * np.abs(Gd[live]).max())


def test_no_compression_path(ctx):
    pts = synth.kinect_scene(100_000, grid=48, leaf=0.02, seed=6)
    ctx.voxelize(pts, 0.02)
    sb, hn = ctx.extract(117, THR, 6)
    f = ctx.features()
    ex = ctx.exist()
    rng = np.random.default_rng(0)
    axis_q = rng.standard_normal((2, 5, 117)).astype(np.float32)
    ctx.search_setup(None, None, axis_q)
    ctx.set_rank(1)
    lists, nm = ctx.search((2, 2, 2), 20)
    Ld, _, scd = po.search(sb, f, ex, None, axis_q, (2, 2, 2), 1, 20, dbl=True, want_scores=True)
    sc = ctx.scores()
    ok = scd > 0
    np.testing.assert_allclose(sc[ok], scd[ok], rtol=SCORE_RTOL_F64)


def test_dense_grid_512_style_small(ctx):
    """Config-5 style dense occupancy (100 %) on a small grid: exact vs numpy."""
    words = synth.dense_words(40, seed=8)
    ctx.set_grid(words.reshape(-1), (40, 40, 40))
    for variant in (981, 117):
        ctx.extract(variant, THR, 10)
        fn, ex, _ = npr.c3hlac(words, variant, THR, 10)
        assert np.array_equal(ctx.features(), fn)
        assert np.array_equal(ctx.exist(), ex)


@pytest.mark.parametrize("G,S", [(36, 3), (37, 6), (39, 13), (34, 16), (33, 7)])
def test_dense_grid_tile_pitches(ctx, G, S):
    """The dense matrix-core tile body at every plane pitch it specialises (row pitch
    lx + 2 rounded up to 4 = 4, 8, 12, 16, 20 bytes; ragged edge tiles): exact vs numpy."""
    words = synth.dense_words(G, seed=8 + S)
    ctx.set_grid(words.reshape(-1), (G, G, G))
    for variant in (981, 117):
        ctx.extract(variant, THR, S)
        fn, ex, _ = npr.c3hlac(words, variant, THR, S)
        assert np.array_equal(ctx.features(), fn)
        assert np.array_equal(ctx.exist(), ex)


def test_dense_256_bin_block_linearity(ctx):
    """Size-independent property at full size: the binary-count bins (normalised by 1)
    are exact integers, and summing them over subdivisions must give the whole-grid
    (subdivision_size 0) histogram; checked on a dense 256^3 grid the oracle would take
    minutes on."""
    words = synth.dense_words(256, seed=12)
    ctx.set_grid(words.reshape(-1), (256, 256, 256))
    ctx.extract(981, THR, 16)
    parts = ctx.features()[:, 495:].astype(np.float64).sum(0)
    ctx.extract(981, THR, 0)
    whole = ctx.features()[0, 495:].astype(np.float64)
    # per-subdivision counts are exact in float32; the whole-grid ones are float(exact int)
    np.testing.assert_array_equal(parts.astype(np.float32), whole.astype(np.float32))
    assert whole[:6].sum() == 3 * 256 ** 3  # each voxel adds beta_c + (1-beta_c) per colour


@pytest.mark.parametrize("lanes,batch,rank,pipe", [(1, 1, 1, 0), (1, 4, 1, 0), (3, 1, 1, 0), (3, 4, 1, 0),
                                                   (2, 3, 2, 0), (4, 8, 1, 0), (1, 1, 1, 1), (1, 2, 1, 1),
                                                   (1, 3, 1, 1), (1, 8, 1, 1), (2, 3, 2, 1), (1, 32, 1, 1),
                                                   (1, 64, 1, 1), (2, 32, 1, 0)])
def test_run_frames_lanes_match_sequential(ctx, lanes, batch, rank, pipe):
    """c3h_run_frames (frames batched per launch; batches in flight on lane contexts, or
    software-pipelined through the tick kernel: 8 frames at batch 1/2 rotate through all
    four buffer sets) == frame-by-frame setRank / extract / search on one context; the
    context ends with the last frame's state."""
    import torch
    G, S, rng_box = 64, 8, (2, 2, 1)
    frames = [synth.kinect_scene(60_000, grid=G, leaf=0.01, seed=synth.BASE_SEED + 40 + i) for i in range(7)]
    words = []
    for pts in frames:
        gi = ctx.voxelize(pts, 0.01)
        assert list(gi.div_b) == [G] * 3
        words.append(ctx.grid().reshape(-1).astype(np.uint32))
    words.append(np.zeros_like(words[0]))  # an empty frame: no position passes the gate
    axis_t, var, axis_q = synth.random_bases(117, 24, 4, 6, seed=3)
    ctx.search_setup(axis_t, var, axis_q)
    ref = []
    for w in words:
        ctx.set_grid(w, (G, G, G))
        ctx.set_rank(rank)  # run_frames: every frame starts from fresh lists
        ctx.extract(117, THR, S)
        det, _ = ctx.search(rng_box, 20)
        ref.append(det.copy())
    last_feat = ctx.features()
    last_exist = ctx.exist()
    dev = torch.device("cuda", 0)
    d_grids = [torch.from_numpy(w.view(np.int32)).to(dev) for w in words]
    d_out = torch.zeros((len(words), 4 * rank * 3), dtype=torch.int64, device=dev)
    ctx.set_lanes(lanes)
    ctx.set_batch(batch)
    ctx.set_pipeline(pipe)
    torch.cuda.synchronize()  # d_out / grids were written on torch's stream, the library runs on its own
    ctx.run_frames(np.array([g.data_ptr() for g in d_grids], np.uint64), (G, G, G), (0, 0, 0), 0.01, 117,
                   THR, S, rng_box, 20, True, d_out.data_ptr())
    ctx.synchronize()
    got = d_out.cpu().numpy().view(c3hlac.DET_DTYPE).reshape(len(words), 4, rank)
    for i in range(len(words)):
        np.testing.assert_array_equal(got[i], ref[i])
    np.testing.assert_array_equal(ctx.features(), last_feat)
    np.testing.assert_array_equal(ctx.exist(), last_exist)
    ctx.set_lanes(3)
    ctx.set_batch(4)
    ctx.set_pipeline(1)


def test_config5_dense_512_periodic(ctx):
    """Config 5 at full size (512^3, 100 % occupancy, C3-HLAC-981, compress 981->100,
    10 models x r=20): size-independent property checks.  The grid is periodic with the
    subdivision side (10), so every subdivision whose half-neighbourhood lies inside the
    grid (indices 1..50 per axis) must hold exactly the features of the centre
    subdivision of a 30^3 periodic grid from the numpy oracle; every box position over
    those subdivisions must score bit-identically (fixed-order box sums) and match the
    float64 score of that feature row within SCORE_RTOL_F64."""
    G, S, n = 512, 10, 52
    base = synth.dense_words(S, seed=51)
    small = np.tile(base, (3, 3, 3))
    fr, exr, _ = npr.c3hlac(small, 981, THR, S)
    ref, ref_ex = fr[13], exr[13]  # subdivision (1, 1, 1) of 3^3
    words = np.tile(base, (n, n, n))[:G, :G, :G]
    ctx.set_grid(np.ascontiguousarray(words).reshape(-1), (G, G, G))
    del words
    sb, hn = ctx.extract(981, THR, S)
    assert sb == (n, n, n) and hn == n ** 3
    f = ctx.features().reshape(n, n, n, 981)
    for z in range(1, n - 1):  # per slab: bounded host temporaries
        assert (f[z, 1:n - 1, 1:n - 1] == ref).all(), "interior subdivision differs (z=%d)" % z
    ex = ctx.exist().reshape(n, n, n)
    assert (ex[1:n - 1, 1:n - 1, 1:n - 1] == ref_ex).all()
    del f
    M, D, R = 10, 100, 20
    axis_t, var, axis_q = synth.random_bases(981, D, M, R, seed=52)
    ctx.search_setup(axis_t, var, axis_q)
    ctx.set_rank(1)
    lists, nm = ctx.search((2, 2, 2), 100)
    P = (n - 1) ** 3
    sc = ctx.scores().reshape(M, n - 1, n - 1, n - 1)
    assert sc.size == M * P and (sc > 0).all()  # dense: every position passes the gate
    inner = sc[:, 1:n - 2, 1:n - 2, 1:n - 2].reshape(M, -1)
    assert (inner == inner[:, :1]).all(), "interior positions must score bit-identically"
    g = synth.whiten(axis_t, var).astype(np.float64) @ ref.astype(np.float64)
    q = axis_q.astype(np.float64) @ g
    s64 = np.sqrt((q * q).sum(1)) / np.sqrt(g @ g)
    np.testing.assert_allclose(inner[:, 0], s64, rtol=SCORE_RTOL_F64)
    # rank 1 = first maximum in scan order over all positions (boundary ones included)
    flat = sc.reshape(M, -1)
    for m in range(M):
        p = int(np.argmax(flat[m]))
        assert float(lists[m, 0]["score"]) == flat[m, p]
        assert (int(lists[m, 0]["z"]), int(lists[m, 0]["y"]), int(lists[m, 0]["x"])) == \
            np.unravel_index(p, (n - 1,) * 3)
    # fp16 matrix-core compress (c3h_set_search_precision): stated tolerance 2e-3 relative
    ctx.set_search_precision(True)
    try:
        ctx.set_rank(1)
        lists16, _ = ctx.search((2, 2, 2), 100)
        sc16 = ctx.scores().reshape(M, n - 1, n - 1, n - 1)
        assert (sc16 > 0).all()
        inner16 = sc16[:, 1:n - 2, 1:n - 2, 1:n - 2].reshape(M, -1)
        assert (inner16 == inner16[:, :1]).all()
        np.testing.assert_allclose(inner16[:, 0], s64, rtol=2e-3)
        assert not np.array_equal(inner16[:, 0], inner[:, 0])  # the f16 path really ran
        flat16 = sc16.reshape(M, -1)
        for m in range(M):
            assert float(lists16[m, 0]["score"]) == flat16[m].max()
    finally:
        ctx.set_search_precision(False)


REF_CLOUDS = ["noisy_torus_blue.pcd", "bowl1_0000.pcd", "tmp_normal.pcd", "obj_torus_black.pcd",
              "noiseless_cone_red.pcd", "noisy_sphere_green.pcd", "noiseless_cylinder_yellow.pcd",
              "noisy_plane_purple.pcd", "noiseless_torus_black.pcd", "plastic-cup1_0000.pcd",
              "assam_blend_tea_0000.pcd", "messmer_tea_0000.pcd", "bouillon_0000.pcd", "marker_red_0000.pcd",
              "bowl1_0015.pcd"]


def _pcd(name):
    from pathlib import Path
    return c3hlac.read_pcd(Path(__file__).resolve().parent / "golden" / "ref_fixtures" / "pcd" / name)


def _check_cloud(ctx, pts, leaf, cases):
    """voxelise + C3-HLAC on the GPU vs the oracle on the same points: voxel indices, leaf
    layout, packed colours and the downsampled centroids bit-exact; exact-integer features
    bit-exact, including voxels whose float centroid rounds across a cell boundary (the
    reference takes their subdivision, c3_hlac.cpp:349-354, and neighbour base, PCL
    getNeighborCentroidIndices, from the centroid)."""
    gi = ctx.voxelize(pts, leaf)
    g, layout, cloud = po.voxelize(pts, leaf)
    assert list(gi.div_b) == list(g.div_b) and gi.n_occ == g.n_occ
    assert np.array_equal(ctx.leaf_layout(), layout)
    assert np.array_equal(ctx.downsampled().view(np.uint32), cloud.view(np.uint32))
    checked = 0
    for variant, S, off in cases:
        fe, sbo, hn = po.c3hlac(g, layout, cloud, variant, THR, leaf, S, off, exact=True)
        if hn < 0:  # a centroid past the last subdivision: out of bounds in the reference
            continue
        sb, hn2 = ctx.extract(variant, THR, S, off)
        assert tuple(sb) == tuple(sbo) and hn2 == hn
        assert np.array_equal(ctx.features(), fe), (variant, S, off)
        fa, _, _ = po.c3hlac(g, layout, cloud, 981, THR, leaf, S, off, exact=False)
        assert np.array_equal(ctx.exist(), po.exist(fa))
        checked += 1
    return checked


@pytest.mark.parametrize("leaf", [0.004, 0.005, 0.01])
@pytest.mark.parametrize("name", REF_CLOUDS)
def test_reference_clouds_end_to_end(ctx, name, leaf):
    """The reference's own demo clouds (tests/golden/ref_fixtures/pcd: synthetic shapes and
    real Kinect object views) read with c3h_pcd_read_xyzrgb, at three leaf sizes."""
    cases = [(981, 5, (0, 0, 0)), (117, 5, (0, 0, 0)), (981, 0, (0, 0, 0)), (117, 4, (1, 0, 2))]
    assert _check_cloud(ctx, _pcd(name), leaf, cases) >= 2


def test_points_on_cell_boundaries(ctx):
    """Every point on (or one ulp beside) a cell boundary, several points per voxel: the
    centroids of most voxels round across a boundary in some direction, so the exact
    centroid pass and the off-cell correction of the C3-HLAC sums carry the whole result."""
    rng = np.random.default_rng(11)
    leaf = np.float32(0.005)
    n = 30000
    cells = rng.integers(0, 24, (n, 3)).astype(np.float32)
    xyz = cells * leaf
    ulp = rng.integers(-1, 2, (n, 3))
    xyz = np.nextafter(xyz, np.where(ulp < 0, -np.inf, np.inf).astype(np.float32)) * (ulp != 0) + xyz * (ulp == 0)
    col = rng.integers(0, 256, (n, 3))
    pts = np.concatenate([xyz.astype(np.float32), synth.pack_rgb(col[:, 0], col[:, 1], col[:, 2])[:, None]], 1)
    pts = np.ascontiguousarray(pts, np.float32)
    g, layout, cloud = po.voxelize(pts, leaf)
    occ = np.flatnonzero(layout >= 0)
    d = np.array(g.div_b)
    own = np.stack([occ % d[0], (occ // d[0]) % d[1], occ // (d[0] * d[1])], 1) + np.array(g.min_b)
    c = cloud[layout[occ], :3]
    moved = ((np.floor(c * (np.float32(1) / leaf)) != own) | (np.floor(c / leaf) != own)).any(1)
    assert moved.sum() > 100  # the case under test is there
    cases = [(981, 6, (0, 0, 0)), (117, 6, (0, 0, 0)), (981, 0, (0, 0, 0)), (117, 5, (2, 1, 0)),
             (981, 20, (0, 0, 0))]
    assert _check_cloud(ctx, pts, float(leaf), cases) >= 3


@pytest.mark.parametrize("batch", [32, 64])
def test_run_frames_pipelined_many_batches(ctx, batch):
    """The production configuration: the pipelined tick at 32 / 64 frames per tick over 150
    distinct resident grids (several full batches, a ragged last one, the fill/drain ticks,
    all four buffer sets) == frame-by-frame extract + search."""
    import torch
    G, S, rng_box = 64, 8, (2, 2, 2)
    base = []
    for i in range(5):
        ctx.voxelize(synth.kinect_scene(60_000, grid=G, leaf=0.01, seed=synth.BASE_SEED + 70 + i), 0.01)
        base.append(ctx.grid().reshape(G, G, G).astype(np.uint32))
    words = [np.roll(base[i % 5], 3 * (i // 5), axis=2).reshape(-1) for i in range(150)]
    axis_t, var, axis_q = synth.random_bases(117, 24, 4, 6, seed=5)
    ctx.search_setup(axis_t, var, axis_q)
    ref = []
    for w in words:
        ctx.set_grid(w, (G, G, G))
        ctx.set_rank(1)
        ctx.extract(117, THR, S)
        det, _ = ctx.search(rng_box, 20)
        ref.append(det.copy())
    dev = torch.device("cuda", 0)
    d_grids = [torch.from_numpy(w.view(np.int32)).to(dev) for w in words]
    d_out = torch.zeros((len(words), 4 * 3), dtype=torch.int64, device=dev)
    ctx.set_batch(batch)
    ctx.set_pipeline(1)
    torch.cuda.synchronize()  # d_out / grids were written on torch's stream, the library runs on its own
    ctx.run_frames(np.array([g.data_ptr() for g in d_grids], np.uint64), (G, G, G), (0, 0, 0), 0.01, 117,
                   THR, S, rng_box, 20, True, d_out.data_ptr())
    ctx.synchronize()
    got = d_out.cpu().numpy().view(c3hlac.DET_DTYPE).reshape(len(words), 4, 1)
    for i in range(len(words)):
        np.testing.assert_array_equal(got[i], ref[i], err_msg="frame %d" % i)
    ctx.set_batch(4)


def test_voxelize_range_error_leaves_no_sums(ctx):
    """A frame with cells beyond +-2^20 (C3H_ERR_RANGE; its valid points span more than the
    accumulator dims too) fails, and the next frame's grid is the oracle's: the failed
    frame's sums do not leak into it."""
    rng = np.random.default_rng(17)
    xyz = (rng.random((5000, 3)) * 2.0).astype(np.float32)
    xyz[0] = (30.0, 0.5, 0.5)  # 3e6 cells at leaf 1e-5: beyond +-2^20
    col = rng.integers(0, 256, (5000, 3))
    bad = np.concatenate([xyz, synth.pack_rgb(col[:, 0], col[:, 1], col[:, 2])[:, None]], 1).astype(np.float32)
    with pytest.raises(c3hlac._capi.C3HError):
        ctx.voxelize(bad, 1e-5)
    pts = synth.parity_cloud(3000, grid=16, leaf=0.01, seed=19)
    ctx.voxelize(pts, 0.01)
    g, layout, cl = po.voxelize(pts, 0.01)
    occ = layout >= 0
    words = ctx.grid()
    assert np.array_equal(ctx.leaf_layout(), layout)
    assert np.array_equal(words[occ], (1 << 24) | cl[layout[occ], 3].view(np.uint32)) and not words[~occ].any()
