"""The matrix-core projection (score_mfma_kernel, c3h_set_score_engine(ctx, 2)) against
the VALU kernels and the float64 oracle.  Both engines form every projection as the same
k-ordered fp32 fma chain (v_mfma_f32_32x32x2_f32 is bit-for-bit that chain), so scores
and rank lists must be bit-identical between them; against the oracle the stated
tolerance is SCORE_RTOL_F64 (SearchObjMulti::searchPart, search.cpp:915-968)."""
import numpy as np
import pytest

import pyoracle as po
from c3hlac import synth
from conftest import THR

from test_gpu_parity import SCORE_RTOL_F64, _assert_replay_matches

pytestmark = pytest.mark.gpu


def _search(ctx, engine, ranges, rank, thr, rotate=True):
    ctx.set_score_engine(engine)
    try:
        ctx.set_rank(rank)
        lists, nm = ctx.search(ranges, thr, rotate=rotate)
        return lists.copy(), nm, ctx.scores().copy()
    finally:
        ctx.set_score_engine(0)


@pytest.mark.parametrize("D,M,r", [(40, 3, 8), (100, 10, 20), (100, 4, 64), (12, 2, 5)])
@pytest.mark.parametrize("ranges,rank", [((2, 2, 2), 1), ((1, 2, 3), 4), ((3, 3, 1), 1)])
def test_engines_bit_identical(ctx, D, M, r, ranges, rank):
    pts = synth.kinect_scene(300_000, grid=96, leaf=0.02, seed=77)
    ctx.voxelize(pts, 0.02)
    sb, hn = ctx.extract(981, THR, 8)
    axis_t, var, axis_q = synth.random_bases(981, D, M, r, seed=9)
    ctx.search_setup(axis_t, var, axis_q)
    l1, n1, s1 = _search(ctx, 1, ranges, rank, 50)
    l2, n2, s2 = _search(ctx, 2, ranges, rank, 50)
    assert n1 == n2
    assert (s1 > 0).any()
    assert np.array_equal(s1, s2)
    assert np.array_equal(l1, l2)
    _assert_replay_matches(ctx, ranges, rank, l2)
    f, ex = ctx.features(), ctx.exist()
    _, _, scd = po.search(sb, f, ex, synth.whiten(axis_t, var), axis_q, ranges, rank, 50, dbl=True,
                          want_scores=True)
    ok = scd > 0
    assert np.array_equal(s2 > 0, ok)
    np.testing.assert_allclose(s2[ok], scd[ok], rtol=SCORE_RTOL_F64)


@pytest.mark.parametrize("M", [1, 5])
def test_r70_models_matrix_cores_vs_generic(ctx, M):
    """r = 70 (color_voxel_recognition_2's model dimension) is beyond the VALU list
    kernel: engine 1 runs the generic kernel, engine 0/2 the matrix cores."""
    pts = synth.kinect_scene(1_000_000, grid=128, leaf=0.02, seed=synth.BASE_SEED + 3)
    ctx.voxelize(pts, 0.02)
    sb, hn = ctx.extract(981, THR, 10)
    axis_t, var, axis_q = synth.random_bases(981, 100, M, 70, seed=70)
    ctx.search_setup(axis_t, var, axis_q)
    lg, _, sg = _search(ctx, 1, (2, 2, 2), M, 100)
    la, _, sa = _search(ctx, 0, (2, 2, 2), M, 100)  # automatic: r > 64 -> matrix cores
    assert (sg > 0).any()
    assert np.array_equal(sg, sa)
    assert np.array_equal(lg, la)
    f, ex = ctx.features(), ctx.exist()
    Ld, _, scd = po.search(sb, f, ex, synth.whiten(axis_t, var), axis_q, (2, 2, 2), M, 100, dbl=True,
                           want_scores=True)
    ok = scd > 0
    assert np.array_equal(sa > 0, ok)
    np.testing.assert_allclose(sa[ok], scd[ok], rtol=SCORE_RTOL_F64)
    _assert_replay_matches(ctx, (2, 2, 2), M, la)
    # fp16 search precision: f16 operands on v_mfma_f32_32x32x16_f16, stated tolerance 2e-3
    ctx.set_search_precision(True)
    try:
        lh, _, sh = _search(ctx, 2, (2, 2, 2), M, 100)
    finally:
        ctx.set_search_precision(False)
    assert np.array_equal(sh > 0, ok)
    np.testing.assert_allclose(sh[ok], scd[ok], rtol=2e-3)
    assert not np.array_equal(sh, sa)  # the f16 path really ran


def test_config5_stress_63_models_r70(ctx):
    """Config 5's stress case: 512^3 dense, C3-HLAC-981, compress 981->100,
    63 models x r=70 (118 GF of projections) on the matrix cores.  The grid is periodic
    with the subdivision side, so every interior position must score bit-identically and
    match the float64 score of the periodic feature row."""
    import numpy.testing as npt
    import np_ref as npr
    G, S, n = 512, 10, 52
    base = synth.dense_words(S, seed=51)
    fr, _, _ = npr.c3hlac(np.tile(base, (3, 3, 3)), 981, THR, S)
    ref = fr[13]
    words = np.tile(base, (n, n, n))[:G, :G, :G]
    ctx.set_grid(np.ascontiguousarray(words).reshape(-1), (G, G, G))
    del words
    sb, hn = ctx.extract(981, THR, S)
    M, D, R = 63, 100, 70
    axis_t, var, axis_q = synth.random_bases(981, D, M, R, seed=53)
    ctx.search_setup(axis_t, var, axis_q)
    ctx.set_rank(1)
    lists, _ = ctx.search((2, 2, 2), 100)
    sc = ctx.scores().reshape(M, n - 1, n - 1, n - 1)
    assert (sc > 0).all()
    inner = sc[:, 1:n - 2, 1:n - 2, 1:n - 2].reshape(M, -1)
    assert (inner == inner[:, :1]).all(), "interior positions must score bit-identically"
    g = synth.whiten(axis_t, var).astype(np.float64) @ (8.0 * ref.astype(np.float64))
    q = np.einsum("mrd,d->mr", axis_q.astype(np.float64), g)
    s64 = np.sqrt((q * q).sum(1)) / np.sqrt(g @ g)
    npt.assert_allclose(inner[:, 0], s64, rtol=SCORE_RTOL_F64)
    flat = sc.reshape(M, -1)
    for m in range(M):
        p = int(np.argmax(flat[m]))
        assert float(lists[m, 0]["score"]) == flat[m, p]
        assert (int(lists[m, 0]["z"]), int(lists[m, 0]["y"]), int(lists[m, 0]["x"])) == \
            np.unravel_index(p, (n - 1,) * 3)
    # fp16 search precision (f16 compress + f16 projection): stated tolerance 2e-3
    ctx.set_search_precision(True)
    try:
        ctx.set_rank(1)
        lists16, _ = ctx.search((2, 2, 2), 100)
        sc16 = ctx.scores().reshape(M, n - 1, n - 1, n - 1)
    finally:
        ctx.set_search_precision(False)
    assert (sc16 > 0).all()
    inner16 = sc16[:, 1:n - 2, 1:n - 2, 1:n - 2].reshape(M, -1)
    assert (inner16 == inner16[:, :1]).all()
    npt.assert_allclose(inner16[:, 0], s64, rtol=2e-3)
    assert not np.array_equal(inner16[:, 0], inner[:, 0])
    flat16 = sc16.reshape(M, -1)
    for m in range(M):
        assert float(lists16[m, 0]["score"]) == flat16[m].max()
