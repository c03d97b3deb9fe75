"""The large-grid search engines and the dense matrix-core C3 body on data whose rows all
differ (VERDICT r2 "next" item 1).

The engines below switch on at >= 65,536 subdivisions (c3h_internal.h kBoxsumRows,
search.hip kCompressMfmaRows) -- BASELINE config 5's regime:
- compress_f32c_kernel (f32 matrix cores; the same k-ordered fma
  chain as the VALU compress_kernel, so G must be bit-identical to it),
- compress_f16_kernel + score_mfma_f16_kernel (fp16 search precision, 2e-3),
- boxsum_kernel, score_mfma_kernel (f32 matrix cores; bit-identical to the VALU engine),
- scores_argmax_kernel + argmax_finalize_kernel (the parallel rank-1 argmax).
Earlier tests ran them only on grids periodic with the subdivision side, where every
interior row is the same and an interior indexing error is invisible.  Here:
- 256^3 Kinect scenes at S = 6 (43^3 = 79,507 subdivisions, distinct rows), C3-HLAC-117
  and -981, M = 10 x r = 20 and M = 5 x r = 70: every score against the float64 oracle
  (SearchObjMulti::searchPart, search.cpp:915-968, 1e-5), every rank-1 record against the
  oracle's position, G of the matrix-core compress == G of the VALU compress;
- a random dense 512^3 grid (not tiled): >= 200 sampled subdivisions of the MFMA C3 body
  (c3hlac_mfma_kernel) against the exact-integer oracle run on the (S+2)^2 x (S+1) crop
  each depends on (c3_hlac.cpp:344-393: the half neighbourhood reaches x +-1, y +-1,
  z - 1), then the whole search against the float64 oracle on those features."""
import concurrent.futures as cf

import numpy as np
import pytest

import pyoracle as po
from c3hlac import synth
from conftest import THR

from test_gpu_parity import SCORE_RTOL_F64

pytestmark = pytest.mark.gpu

F16_RTOL = 2e-3


def _check_records(lists, scd, P, rtol, tag):
    """lists (M, 1) DET records; scd = modes x M x P oracle scores (single mode here).
    Rank 1 = the first maximum in scan order (search.cpp:464-474, strict '>'); a record
    may name another position only if it ties the maximum within rtol."""
    M = lists.shape[0]
    ref = scd.reshape(M, P)
    for m in range(M):
        e = lists[m, 0]
        best = int(np.argmax(ref[m]))
        assert float(e["score"]) > 0, (tag, m)
        p = int(e["x"]) + P_dims[0] * (int(e["y"]) + P_dims[1] * int(e["z"]))
        assert int(e["mode"]) == 0, (tag, m)
        assert abs(float(e["score"]) - ref[m, p]) <= rtol * ref[m, p], (tag, m, float(e["score"]), ref[m, p])
        if p != best:
            assert ref[m, p] >= ref[m, best] * (1 - 2 * rtol), (tag, m, p, best)


P_dims = [0, 0, 0]


def _set_pdims(sb, box):
    for a in range(3):
        P_dims[a] = sb[a] - box[a] + 1
    return P_dims[0] * P_dims[1] * P_dims[2]


@pytest.fixture(scope="module")
def kinect256(ctx):
    pts = synth.kinect_scene(1_000_000, grid=256, leaf=0.01, seed=synth.BASE_SEED + 256)
    gi = ctx.voxelize(pts, 0.01)
    assert list(gi.div_b) == [256] * 3
    words = ctx.grid().copy()
    g, layout, cloud = po.grid_inputs(words, (256,) * 3, 0.01)
    return words, g, layout, cloud


@pytest.mark.parametrize("variant,M,r,use_fmax", [(117, 10, 20, True), (981, 10, 20, False), (981, 5, 70, False)])
def test_kinect256_s6_large_grid_engines(ctx, kinect256, variant, M, r, use_fmax):
    """use_fmax: setNormalizeVal maxima (search.cpp:563-570), applied on the LDS store of
    the matrix-core compress."""
    words, g, layout, cloud = kinect256
    S, D, BOX, THRX = 6, 100, (2, 2, 2), 100
    ctx.set_grid(words, (256,) * 3, leaf=0.01)
    sb, H = ctx.extract(variant, THR, S)
    assert sb == (43, 43, 43) and H == 79507 >= 65536
    fe, sbo, _ = po.c3hlac(g, layout, cloud, variant, THR, 0.01, S, exact=True)
    f = ctx.features()
    ex = ctx.exist()
    assert tuple(sbo) == sb
    bad = np.flatnonzero((f != fe).any(1))
    assert bad.size == 0, ("feature rows", bad.size, bad[:8].tolist())
    ex_ref = po.exist(fe)
    assert np.array_equal(ex, ex_ref)
    assert len(np.unique(fe[ex > 0], axis=0)) > 0.9 * int((ex > 0).sum())  # rows differ
    axis_t, var, axis_q = synth.random_bases(variant, D, M, r, seed=600 + variant + r)
    ap = synth.whiten(axis_t, var)
    fmax = (fe.max(0) * np.float32(0.8)).astype(np.float32) if use_fmax else None
    ctx.search_setup(axis_t, var, axis_q, feature_max=fmax)
    ctx.set_rank(1)
    lists, _ = ctx.search(BOX, THRX)  # auto: matrix-core compress, box sums, score_mfma, argmax
    sc = ctx.scores().copy()
    G_mf = ctx.compressed().copy()
    _, _, scd = po.search(sb, fe, ex_ref, ap, axis_q, BOX, 1, THRX, dbl=True, fmax=fmax, want_scores=True)
    P = _set_pdims(sb, BOX)
    ok = scd > 0
    assert ok.sum() > 100 and np.array_equal(sc > 0, ok)
    np.testing.assert_allclose(sc[ok], scd[ok], rtol=SCORE_RTOL_F64)
    _check_records(lists, scd, P, SCORE_RTOL_F64, "mfma %d r%d" % (variant, r))
    # the VALU compress (dense compress_kernel via c3h_set_features) gives the same G bits
    ctx.set_features(f, sb, exist=ex)
    ctx.set_rank(1)
    lists_v, _ = ctx.search(BOX, THRX)
    G_valu = ctx.compressed()
    rows = ex > 0
    assert np.array_equal(G_mf[rows], G_valu[rows]), "matrix-core compress != VALU compress"
    assert np.array_equal(ctx.scores(), sc)
    assert np.array_equal(lists_v, lists)
    # the VALU projection engine (score_list over the box sums; the generic kernel at r > 64)
    ctx.set_score_engine(1)
    try:
        ctx.set_rank(1)
        lists_1, _ = ctx.search(BOX, THRX)
        assert np.array_equal(ctx.scores(), sc), "VALU engine scores differ from the matrix cores'"
        assert np.array_equal(lists_1, lists)
    finally:
        ctx.set_score_engine(0)
    # fp16 search precision: f16 compress + f16 projection, stated tolerance 2e-3
    ctx.extract(variant, THR, S)  # sparse rows again (the fp16 compress runs on the row list)
    ctx.set_search_precision(True)
    try:
        ctx.set_rank(1)
        lists16, _ = ctx.search(BOX, THRX)
        s16 = ctx.scores()
        assert np.array_equal(s16 > 0, ok)
        np.testing.assert_allclose(s16[ok], scd[ok], rtol=F16_RTOL)
        assert not np.array_equal(s16[ok], sc[ok])  # the f16 path really ran
        _check_records(lists16, scd, P, F16_RTOL, "f16 %d r%d" % (variant, r))
    finally:
        ctx.set_search_precision(False)


def _crop_row(words, sub, S, variant):
    """Exact-integer oracle features of subdivision sub = (sx, sy, sz) of the packed grid
    words[z, y, x], computed on the crop its centres and half neighbourhood span."""
    gz, gy, gx = words.shape
    x0, y0, z0 = (s * S for s in sub)
    lx, ly, lz = max(x0 - 1, 0), max(y0 - 1, 0), max(z0 - 1, 0)
    hx, hy, hz = min(x0 + S + 1, gx), min(y0 + S + 1, gy), min(z0 + S, gz)
    crop = words[lz:hz, ly:hy, lx:hx]
    # pad x with empty cells to S + 2 (+ offset): the crop then always holds two subdivisions.
    # With a single one (hist_num == 1) computeC3HLAC puts every voxel, offset halo included,
    # into histogram 0 (c3_hlac.cpp:348).  Empty cells past the grid's edge are what an
    # out-of-grid neighbour lookup sees anyway.
    pad = (x0 - lx) + S + 2 - crop.shape[2]
    if pad > 0:
        crop = np.concatenate([crop, np.zeros(crop.shape[:2] + (pad,), crop.dtype)], 2)
    crop = np.ascontiguousarray(crop)
    g, layout, cloud = po.grid_inputs(crop, (crop.shape[2], hy - ly, hz - lz), 0.01)
    fe, _, _ = po.c3hlac(g, layout, cloud, variant, THR, 0.01, S, (x0 - lx, y0 - ly, z0 - lz), exact=True)
    return fe[0]


@pytest.fixture(scope="module")
def dense512():
    rng = np.random.default_rng(512)
    w = rng.integers(0, 1 << 24, size=512 ** 3, dtype=np.uint32) | np.uint32(1 << 24)
    return w.reshape(512, 512, 512)


def _sample_subdivisions(n, count, seed):
    rng = np.random.default_rng(seed)
    s = [(0, 0, 0), (n - 1, n - 1, n - 1), (n - 1, 0, n - 1), (0, n - 1, 0)]  # corners (ragged last tile)
    while len(s) < count:
        s.append(tuple(int(v) for v in rng.integers(0, n, 3)))
    return s


@pytest.mark.parametrize("variant", [981, 117])
def test_dense512_random_mfma_c3_sampled(ctx, dense512, variant):
    G, S = 512, 10
    n = -(-G // S)
    ctx.set_grid(dense512.reshape(-1), (G,) * 3, leaf=0.01)
    sb, H = ctx.extract(variant, THR, S)
    assert sb == (n, n, n)
    f = ctx.features().reshape(n, n, n, variant)
    ex = ctx.exist().reshape(n, n, n)
    subs = _sample_subdivisions(n, 220, 7 + variant)
    with cf.ThreadPoolExecutor(8) as pool:  # the C oracle releases the GIL
        refs = list(pool.map(lambda s: _crop_row(dense512, s, S, variant), subs))
    for s, ref in zip(subs, refs):
        sx, sy, sz = s
        bad = np.flatnonzero(f[sz, sy, sx] != ref)
        assert bad.size == 0, ("subdivision", s, bad[:8].tolist())
        assert ex[sz, sy, sx] == po.exist(ref[None, :])[0], s
    # neighbouring rows differ (not a periodic grid)
    assert not np.array_equal(f[5, 5, 5], f[5, 5, 6])


def test_dense512_random_search_vs_oracle(ctx, dense512):
    """Config 5 search (132,651 positions x 10 models x r = 20) on the random dense grid:
    every score against the float64 oracle on the GPU's features (the features themselves
    are pinned by test_dense512_random_mfma_c3_sampled), rank-1 records, the VALU engine
    bit-identical, the fp16 precision within 2e-3."""
    G, S, M, D, R, BOX = 512, 10, 10, 100, 20, (2, 2, 2)
    ctx.set_grid(dense512.reshape(-1), (G,) * 3, leaf=0.01)
    sb, H = ctx.extract(981, THR, S)
    fe = ctx.features()
    ex = ctx.exist()
    axis_t, var, axis_q = synth.random_bases(981, D, M, R, seed=5120)
    ctx.search_setup(axis_t, var, axis_q)
    ctx.set_rank(1)
    lists, _ = ctx.search(BOX, 100)
    sc = ctx.scores().copy()
    _, _, scd = po.search(sb, fe, ex, synth.whiten(axis_t, var), axis_q, BOX, 1, 100, dbl=True, want_scores=True)
    P = _set_pdims(sb, BOX)
    assert (scd > 0).all() and (sc > 0).all()
    np.testing.assert_allclose(sc, scd, rtol=SCORE_RTOL_F64)
    assert len(np.unique(sc[:P])) > P // 2  # scores differ across positions
    _check_records(lists, scd, P, SCORE_RTOL_F64, "dense512")
    ctx.set_score_engine(1)
    try:
        ctx.set_rank(1)
        l1, _ = ctx.search(BOX, 100)
        assert np.array_equal(ctx.scores(), sc)
        assert np.array_equal(l1, lists)
    finally:
        ctx.set_score_engine(0)
    ctx.extract(981, THR, S)
    ctx.set_search_precision(True)
    try:
        ctx.set_rank(1)
        l16, _ = ctx.search(BOX, 100)
        s16 = ctx.scores()
        np.testing.assert_allclose(s16, scd, rtol=F16_RTOL)
        _check_records(l16, scd, P, F16_RTOL, "dense512 f16")
    finally:
        ctx.set_search_precision(False)


def test_dense512_fp16_feature_rows(ctx, dense512):
    """fp16 search precision set before the extract (BASELINE configs[4]: "fp16 features";
    VERDICT r4 item 4): the dense MFMA body writes the 981-feature rows as f16 (half the
    bytes; the f16 compress reads them).  The rows are the f32 rows rounded to nearest f16,
    bit for bit (features() converts them); scores within the fp16 tolerance of the float64
    oracle; a search at f32 precision on the same extract converts the rows first."""
    G, S, M, D, R, BOX = 512, 10, 10, 100, 20, (2, 2, 2)
    ctx.set_grid(dense512.reshape(-1), (G,) * 3, leaf=0.01)
    sb, H = ctx.extract(981, THR, S)
    fe = ctx.features()
    ex = ctx.exist()
    axis_t, var, axis_q = synth.random_bases(981, D, M, R, seed=5120)
    ctx.search_setup(axis_t, var, axis_q)
    _, _, scd = po.search(sb, fe, ex, synth.whiten(axis_t, var), axis_q, BOX, 1, 100, dbl=True, want_scores=True)
    P = _set_pdims(sb, BOX)
    ctx.set_search_precision(True)
    try:
        ctx.extract(981, THR, S)
        ctx.set_rank(1)
        l16, _ = ctx.search(BOX, 100)
        s16 = ctx.scores()
        np.testing.assert_allclose(s16, scd, rtol=F16_RTOL)
        _check_records(l16, scd, P, F16_RTOL, "dense512 f16 rows")
        f16 = ctx.features()
        assert np.array_equal(f16, fe.astype(np.float16).astype(np.float32))
        assert np.array_equal(ctx.exist(), ex)
        ctx.extract(981, THR, S)
        ctx.set_search_precision(False)  # f32 search on f16 rows: converted on the device
        ctx.set_rank(1)
        ctx.search(BOX, 100)
        np.testing.assert_allclose(ctx.scores(), scd, rtol=F16_RTOL)
    finally:
        ctx.set_search_precision(False)
