"""CPU tests of the oracle (the checker): pinned against the reference's own tables and
fixtures, cross-checked against the independent numpy restatement."""
import json

import numpy as np
import pytest

import np_ref as npr
import pyoracle as po
from c3hlac import synth
from conftest import GOLDEN, GOLDEN_CASES, THR, load_golden

PAIRS = [(0, 2), (0, 3), (0, 4), (0, 5), (1, 2), (1, 3), (1, 4), (1, 5), (2, 4), (2, 5), (3, 4), (3, 5)]


def bin981(k, c, n):
    return 6 + 78 * c + 9 * n + k if k <= 8 else 60 + 78 * c + 4 * n + (k - 9)


def tri(c, n):
    return 6 * c - c * (c - 1) // 2 + (n - c)


def test_binmap_closed_form_matches_reference_tables():
    """The closed form used by the oracle and the HIP kernel equals the bin table
    extracted from color_chlac.hpp (oracle/gen_binmap.py); every bin appears once."""
    m = json.loads((GOLDEN / "binmap_981.json").read_text())
    assert all(b == bin981(k, c, n) for k, c, n, b in m["first"])
    assert all(b == 495 + bin981(k, c, n) for k, c, n, b in m["bin_first"])
    assert all(b == 474 + tri(c, n) for c, n, b in m["auto"])
    assert all(b == c for c, b in m["zero"])
    assert all(b == 495 + c for c, b in m["bin_zero"])
    assert all(b == 969 + PAIRS.index((c, n)) for c, n, b in m["bin_pairs"])
    bins = [e[-1] for key in ("zero", "bin_zero", "auto", "bin_pairs", "first", "bin_first") for e in m[key]]
    assert sorted(bins) == list(range(981))
    m117 = json.loads((GOLDEN / "binmap_117.json").read_text())
    assert all(b == 6 + 6 * c + n for _, c, n, b in m117["first"])
    assert all(b == 69 + 6 * c + n for _, c, n, b in m117["bin_first"])
    assert all(b == 42 + tri(c, n) for c, n, b in m117["auto"])
    bins = [e[-1] for key in ("zero", "bin_zero", "auto", "bin_pairs", "first", "bin_first") for e in m117[key]]
    assert sorted(bins) == list(range(117))


def test_lut_float_double_differ_only_at_255():
    d, f = po.lut(True), po.lut(False)
    assert np.array_equal(d, npr.lut(True)) and np.array_equal(f, npr.lut(False))
    diff = np.nonzero((d != f).any(1))[0]
    assert list(diff) == [255]
    assert tuple(d[255]) == (254, 0) and tuple(f[255]) == (255, 0)
    assert tuple(d[0]) == (0, 255)


@pytest.mark.parametrize("variant", [981, 117])
@pytest.mark.parametrize("subdiv,offset", [(10, (0, 0, 0)), (7, (2, 1, 3)), (0, (0, 0, 0)),
                                           (40, (1, 1, 1)), (3, (0, 0, 0)), (25, (0, 0, 0))])
def test_oracle_exact_equals_numpy_restatement(variant, subdiv, offset):
    pts = synth.parity_cloud(9000, grid=30, leaf=0.01, seed=7)
    g, layout, cloud = po.voxelize(pts, 0.01)
    div, mb, words, lay = npr.voxelize(pts, 0.01)
    assert np.array_equal(layout, lay)
    fe, sb, hn = po.c3hlac(g, layout, cloud, variant, THR, 0.01, subdiv, offset, exact=True)
    fn, exn, sbn = npr.c3hlac(words, variant, THR, subdiv, offset)
    assert tuple(sb) == tuple(sbn)
    assert np.array_equal(fe, fn)
    ff, _, _ = po.c3hlac(g, layout, cloud, variant, THR, 0.01, subdiv, offset, exact=False)
    # the reference's fp32 running sums round only once they pass 2^24
    np.testing.assert_allclose(ff, fe, rtol=1e-4, atol=0)
    if variant == 981:
        assert np.array_equal(po.exist(ff), exn)


def test_oracle_kinect_scene_exact_equals_numpy():
    pts = synth.kinect_scene(80_000, grid=48, leaf=0.02, seed=9)
    g, layout, cloud = po.voxelize(pts, 0.02)
    div, mb, words, lay = npr.voxelize(pts, 0.02)
    assert div == (48, 48, 48) and np.array_equal(layout, lay)
    for variant in (981, 117):
        fe, sb, _ = po.c3hlac(g, layout, cloud, variant, THR, 0.02, 10, (0, 0, 0), exact=True)
        fn, _, _ = npr.c3hlac(words, variant, THR, 10, (0, 0, 0))
        assert np.array_equal(fe, fn)


@pytest.mark.parametrize("name", GOLDEN_CASES)
def test_golden_fixtures_reproduce(name):
    z = load_golden(name)
    g, layout, cloud = po.voxelize(z["pts"], float(z["leaf"]), float(z["z_limit"]))
    assert np.array_equal(layout, z["leaf_layout"])
    np.testing.assert_array_equal(cloud, z["cloud"])
    for variant in (981, 117):
        fe, sb, _ = po.c3hlac(g, layout, cloud, variant, tuple(z["thr"]), float(z["leaf"]), int(z["subdiv"]),
                              tuple(z["offset"]), exact=True)
        assert np.array_equal(fe, z["feat%d_exact" % variant])
    assert np.array_equal(po.exist(z["feat981_faithful"]), z["exist"])


def _kat_expect(c1, c2, k, thr=THR):
    """Hand-derived 981 integer histogram (Appendix A) of a centre voxel of colour c1
    whose half-neighbour k has colour c2 (the neighbour sees no half-neighbour)."""
    L = npr.lut(True)
    def chans(c):
        r, g, b = c
        a = [L[r, 0], L[r, 1], L[g, 0], L[g, 1], L[b, 0], L[b, 1]]
        br, bg, bb = int(r > thr[0]), int(g > thr[1]), int(b > thr[2])
        return a, [br, 1 - br, bg, 1 - bg, bb, 1 - bb]
    a1, b1 = chans(c1)
    a2, b2 = chans(c2)
    h = np.zeros(981, np.int64)
    for a, b in ((a1, b1), (a2, b2)):
        for c in range(6):
            h[c] += a[c]
            h[495 + c] += b[c]
            for n in range(c, 6):
                h[474 + tri(c, n)] += a[c] * a[n]
        for q, (c, n) in enumerate(PAIRS):
            h[969 + q] += b[c] * b[n]
    for c in range(6):
        for n in range(6):
            h[bin981(k, c, n)] += a1[c] * a2[n]
            h[495 + bin981(k, c, n)] += b1[c] * b2[n]
    return h


@pytest.mark.parametrize("k", range(13))
def test_kat_voxel_pair_per_offset(k):
    rel = npr.REL[k]
    words = np.zeros((3, 3, 3), np.uint32)
    c1, c2 = (200, 30, 149), (10, 250, 147)
    words[1, 1, 1] = (1 << 24) | (c1[0] << 16) | (c1[1] << 8) | c1[2]
    words[1 + rel[2], 1 + rel[1], 1 + rel[0]] = (1 << 24) | (c2[0] << 16) | (c2[1] << 8) | c2[2]
    fn, ex, _ = npr.c3hlac(words, 981, THR, 0)
    h = _kat_expect(c1, c2, k)
    norm = np.ones(981, np.float32)
    norm[:6] = np.float32(1 / 255.0)
    norm[6:495] = np.float32(1 / 65025.0)
    np.testing.assert_array_equal(fn[0], h.astype(np.float32) * norm)
    # same pair through the C oracle (point cloud path)
    pts = []
    for (z, y, x), w in np.ndenumerate(words):
        if w:
            pts.append([x + 0.5, y + 0.5, z + 0.5, np.uint32(w & 0xFFFFFF).view(np.float32)])
    pts = np.array(pts, np.float32) * np.array([0.01, 0.01, 0.01, 1], np.float32)
    g, layout, cloud = po.voxelize(pts, 0.01)
    # the grid spans only the occupied bounding box: the result must not depend on it
    fe, _, _ = po.c3hlac(g, layout, cloud, 981, THR, 0.01, 0, (0, 0, 0), exact=True)
    np.testing.assert_array_equal(fe[0], fn[0])


def test_voxelize_semantics():
    leaf = np.float32(0.01)
    rgb = synth.pack_rgb
    pts = np.array([
        [0.005, 0.005, 0.005, rgb(10, 20, 30)],
        [0.006, 0.004, 0.007, rgb(11, 21, 32)],     # same voxel: canonical mean (10.5, 20.5, 31)
        [-0.015, 0.025, 0.015, rgb(255, 0, 255)],   # negative coordinates -> min_b < 0
        [np.nan, 0.0, 0.0, rgb(1, 1, 1)],           # dropped (non-finite)
        [0.0, np.inf, 0.0, rgb(1, 1, 1)],           # dropped
        [0.0, 0.0, 5.0, rgb(1, 1, 1)],              # dropped by z_limit
    ], np.float32)
    g, layout, cloud = po.voxelize(pts, leaf, z_limit=1.0)
    assert g.n_valid == 3 and g.n_occ == 2
    assert list(g.min_b) == [-2, 0, 0] and list(g.div_b) == [3, 3, 2]
    rgbs = cloud[:, 3].view(np.uint32)
    assert (rgbs[0] >> 16) == 10 and ((rgbs[0] >> 8) & 255) == 20 and (rgbs[0] & 255) == 31
    div, mb, words, lay = npr.voxelize(pts, leaf, 1.0)
    assert np.array_equal(lay, layout)


@pytest.mark.parametrize("ranges,rank", [((2, 2, 2), 1), ((1, 2, 1), 1), ((2, 2, 2), 4), ((1, 2, 3), 3),
                                         ((3, 1, 1), 2)])
def test_search_oracle_vs_numpy(ranges, rank):
    pts = synth.kinect_scene(150_000, grid=64, leaf=0.02, seed=21)
    g, layout, cloud = po.voxelize(pts, 0.02)
    feat, sb, _ = po.c3hlac(g, layout, cloud, 981, THR, 0.02, 5, (0, 0, 0))
    ex = po.exist(feat)
    axis_t, var, axis_q = synth.random_bases(981, 24, 3, 6, seed=4)
    ap = synth.whiten(axis_t, var)
    Ld, nm, scd = po.search(sb, feat, ex, ap, axis_q, ranges, rank, 60, dbl=True, want_scores=True)
    L32, _, sc32 = po.search(sb, feat, ex, ap, axis_q, ranges, rank, 60, dbl=False, want_scores=True)
    ms = npr.scores(sb, feat, ex, ap, axis_q, ranges, 60)
    flat = np.concatenate([s.reshape(-1) for (_, _, _, s) in ms])
    np.testing.assert_allclose(scd, flat, rtol=1e-10, atol=1e-12)
    ok = scd > 0
    np.testing.assert_allclose(sc32[ok], scd[ok], rtol=1e-4)  # fp32 summed-volume error (A12)
    # replay logic: numpy's restatement fed the oracle's own scores gives the same lists
    # (comparing across restatements would let exact ties in the true score flip on
    # 1e-16 noise: two boxes with identical content)
    off, ms_c = 0, []
    for mode, xe, ye, s in ms:
        n = s.size
        ms_c.append((mode, xe, ye, scd[off:off + n].reshape(s.shape)))
        off += n
    nl = npr.replay(ms_c, ranges, rank)
    assert [[tuple(e[1:]) for e in m] for m in nl] == [[e[1:] for e in m] for m in Ld.records()]
    nl2 = npr.replay(ms, ranges, rank)
    np.testing.assert_allclose([[e[0] for e in m] for m in nl2], [[e[0] for e in m] for m in Ld.records()],
                               rtol=1e-12)


def test_replay_rank_update_quirks():
    """checkOverlap / shift semantics on a hand-made score sequence (rank 3)."""
    r = (2, 2, 2)
    sc = np.array([[0.5, 0.6, 0.55, 0.9, 0.1, 0.7, 0.65, 0.95]])
    lists = npr.replay([(0, 8, 1, sc)], r, 3)
    # positions are x = 0..7 on one row: boxes of width 2 touch when |dx| <= 2
    assert [e[1] for e in lists[0]] == [7, 3, 0]
    assert lists[0][0][0] == 0.95


def test_remove_overlap_oracle_matches_python():
    rng = np.random.default_rng(3)
    M, rank, r = 4, 3, (2, 1, 2)
    L = po.Lists(M, rank)
    L.score[:] = np.sort(rng.random(M * rank).reshape(M, rank), 1)[:, ::-1].ravel()
    L.x[:] = rng.integers(0, 6, M * rank)
    L.y[:] = rng.integers(0, 6, M * rank)
    L.z[:] = rng.integers(0, 6, M * rank)
    L.mode[:] = rng.integers(0, 6, M * rank)
    ref = [[list(e) for e in m] for m in L.records()]
    po.remove_overlap(L, r)

    def rng_(mode):
        return npr._ranges(mode, r)

    def overlap(lst, x, y, z, mode):
        xr, yr, zr = rng_(mode)
        num = 0
        while num < rank - 1:
            e = lst[num]
            oxr, oyr, ozr = rng_(e[4])
            v1 = e[1] - x; v1 = -v1 - oxr if v1 < 0 else v1 - xr
            v2 = e[2] - y; v2 = -v2 - oyr if v2 < 0 else v2 - yr
            v3 = e[3] - z; v3 = -v3 - ozr if v3 < 0 else v3 - zr
            if v1 <= 0 and v2 <= 0 and v3 <= 0:
                return num
            num += 1
        return num

    for m in range(M):
        for m2 in range(M):
            if m2 == m:
                continue
            ov = overlap(ref[m2], *ref[m][0][1:])
            if ref[m][0][0] > ref[m2][ov][0]:
                for j in range(ov, rank - 1):
                    ref[m2][j] = list(ref[m2][j + 1])
            else:
                for j in range(0, rank - 1):
                    ref[m][j] = list(ref[m][j + 1])
    assert [[tuple(e) for e in m] for m in ref] == L.records()


def test_pca_reader_on_reference_fixtures():
    base = GOLDEN / "ref_fixtures" / "models_offline_r"
    axis, var, mean = po.pca_read(base / "compress_axis")
    assert axis.shape == (137, 137) and mean is None
    np.testing.assert_allclose(np.linalg.norm(axis, axis=0), 1.0, atol=1e-4)
    assert np.all(np.diff(var[var > 1e-6]) <= 1e-6)
    for m in ("000", "001", "002"):
        a, v, mu = po.pca_read(base / m / "pca_result")
        assert a.shape == (100, 100)
        np.testing.assert_allclose(np.linalg.norm(a, axis=0), 1.0, atol=1e-4)
        assert v[0] >= v[1] >= v[2]


def test_exist_gate_formula():
    f = np.zeros((3, 981), np.float32)
    f[0, :2] = [np.float32(1020 * np.float32(1 / 255.0)), np.float32(1275 * np.float32(1 / 255.0))]
    f[1, :2] = [np.float32(254 / 255.0), 0]
    assert list(po.exist(f)) == [int(np.float64((f[0, 0] + f[0, 1]) * np.float32(2)) + 0.001), 1, 0]


@pytest.mark.parametrize("G,S", [(22, 10), (37, 6)])
def test_crop_oracle_matches_whole_grid(G, S):
    """The per-subdivision crop oracle of test_gpu_config5_nonperiodic (a subdivision's
    centres plus its half neighbourhood, x padded to two subdivisions) equals the
    whole-grid oracle at every subdivision, ragged edges and corners included."""
    from test_gpu_config5_nonperiodic import _crop_row
    rng = np.random.default_rng(G)
    w = (rng.integers(0, 1 << 24, size=G ** 3, dtype=np.uint32) | np.uint32(1 << 24)).reshape(G, G, G)
    for variant in (981, 117):
        g, layout, cloud = po.grid_inputs(w.reshape(-1), (G,) * 3, 0.01)
        fe, sb, _ = po.c3hlac(g, layout, cloud, variant, THR, 0.01, S, exact=True)
        n = sb[0]
        fe = fe.reshape(n, n, n, variant)
        for z in range(n):
            for y in range(n):
                for x in range(n):
                    assert np.array_equal(_crop_row(w, (x, y, z), S, variant), fe[z, y, x]), (x, y, z)
