"""The single-frame voxeliser's state between calls (round 6).

- VERDICT r5 item 1: the round-5 fault (an illegal memory access raised from c3h_voxelize
  on a fresh context whose first frame had many points per voxel).  Cause, DESIGN.md
  section 8: the run-merge bug of that build moved one point's count to the voxel at
  toroidal index 0, so that voxel's bucket in the exact-centroid pass had one slot no point
  filled, and on a fresh context the slot's uninitialised point index was read.  The exact
  sequence runs here on a fresh context against the oracle.
- ADVICE r5 (medium): error exits after the accumulate pass leave no sums behind; frames
  wider than the toroidal accumulator budget (2^26 cells) take the sorted path instead of
  failing, with the oracle's grid, leaf layout and centroids.

Voxel semantics: PCL VoxelGrid as the reference built it (c3_hlac/include/c3_hlac/
c3_hlac_tools.hpp:124-130; the oracle's orc_voxel_fill)."""
import numpy as np
import pytest

import c3hlac
import pyoracle as po
from c3hlac import synth
from conftest import THR

pytestmark = pytest.mark.gpu


def _fresh():
    """A context of its own (the session fixture's buffers are not fresh)."""
    import os
    try:
        return c3hlac.Context(0)
    except c3hlac._capi.C3HError as e:
        if os.environ.get("C3H_REQUIRE_GPU"):
            raise
        pytest.skip("no HIP device: %s" % e)


def _cloud(rng, n, span, lo=0.0):
    xyz = (lo + rng.random((n, 3)) * np.asarray(span, np.float64)).astype(np.float32)
    col = rng.integers(0, 256, (n, 3))
    return np.concatenate([xyz, synth.pack_rgb(col[:, 0], col[:, 1], col[:, 2])[:, None]], 1).astype(np.float32)


def _check_voxels(ctx, pts, leaf, grid=True):
    gi = ctx.voxelize(pts, leaf)
    g, layout, cl = po.voxelize(pts, leaf)
    assert list(gi.div_b) == list(g.div_b) and list(gi.min_b) == list(g.min_b)
    assert gi.n_valid == g.n_valid and gi.n_occ == (layout >= 0).sum()
    if grid:
        assert np.array_equal(ctx.leaf_layout(), layout)
        occ = layout >= 0
        words = ctx.grid()
        assert np.array_equal(words[occ], (1 << 24) | cl[layout[occ], 3].view(np.uint32)) and not words[~occ].any()
    assert np.array_equal(ctx.downsampled().view(np.uint32), cl.view(np.uint32))
    return g, layout, cl


def test_fresh_context_multipoint_first_frame():
    """a fresh context whose first frame is tools/vox_bad.py's
    dense_multi cloud (20,000 points in 6^3 voxels at leaf 0.01: ~93 points per voxel, so
    near-face points flag voxels and the exact-centroid pass runs), then a sparse
    400k-point frame (the accumulators regrow), then the dense frame again.  Grid, leaf
    layout and centroids are the oracle's each time; so are the exact C3-HLAC features of
    the dense frame."""
    rng = np.random.default_rng(11)
    _ = _cloud(rng, 3000, 0.08)  # vox_bad.py's draw order: the same dense_multi cloud
    dense = _cloud(rng, 20000, 0.06)
    sparse = _cloud(np.random.default_rng(12), 400_000, 1.0)
    with _fresh() as ctx:
        for pts in (dense, sparse, dense):
            g, layout, cl = _check_voxels(ctx, pts, 0.01)
        fe, sbo, hn = po.c3hlac(g, layout, cl, 981, THR, 0.01, 2, (0, 0, 0), exact=True)
        sb, hn2 = ctx.extract(981, THR, 2, (0, 0, 0))
        assert tuple(sb) == tuple(sbo) and hn2 == hn
        assert np.array_equal(ctx.features(), fe)


def test_wide_frame_sorted_path_then_toroidal():
    """a frame whose extent needs 2^27 accumulator cells (2,000 x 250 x 200 cells
    at leaf 0.01) goes to the sorted path: its grid, layout, centroids (exact, input-order
    fp32 sums, with many points per voxel near cell faces) and C3-HLAC features are the
    oracle's.  The toroidal path's next frames on the same context are exact too (the wide
    frame's first-pass sums were returned to zero)."""
    rng = np.random.default_rng(21)
    far = _cloud(rng, 60_000, (20.0, 2.5, 2.0))
    # clusters of points around cell faces: multi-point voxels whose centroids round across
    cells = rng.integers(0, 40, (3000, 3)).astype(np.float64) * 0.01
    jit = (rng.random((3000, 3)) - 0.5) * 1e-6
    col = rng.integers(0, 256, (3000, 3))
    near = np.concatenate([(cells + jit).astype(np.float32),
                           synth.pack_rgb(col[:, 0], col[:, 1], col[:, 2])[:, None]], 1).astype(np.float32)
    pts = np.ascontiguousarray(np.concatenate([far, near, near[::-1]]), np.float32)
    small = _cloud(np.random.default_rng(22), 20000, 0.06)
    with _fresh() as ctx:
        _check_voxels(ctx, small, 0.01)
        g, layout, cl = _check_voxels(ctx, pts, 0.01)
        fe, sbo, hn = po.c3hlac(g, layout, cl, 117, THR, 0.01, 0, (0, 0, 0), exact=True)
        sb, hn2 = ctx.extract(117, THR, 0, (0, 0, 0))
        assert tuple(sb) == tuple(sbo) and hn2 == hn
        assert np.array_equal(ctx.features(), fe)
        for p in (small, _cloud(np.random.default_rng(23), 300_000, 1.0), small):
            _check_voxels(ctx, p, 0.01)


def test_int32_extent_beyond_old_accumulators():
    """1,700 x 1,300 x 900 cells (1.99e9 voxels: within PCL's int32 check, beyond
    2^31 rounded accumulator cells) -- round 5 failed with C3H_ERR_RANGE, now the sorted
    path: the oracle's valid and occupied counts and centroids (the 8 GB grid stays on the
    device).  A 4e9-voxel extent still fails (int32 voxel indices) and leaves no sums: the
    next frame is the oracle's."""
    rng = np.random.default_rng(31)
    pts = _cloud(rng, 50_000, (17.0, 13.0, 9.0))
    pts[0, :3] = (0.0, 0.0, 0.0)
    pts[1, :3] = (16.995, 12.995, 8.995)
    small = _cloud(np.random.default_rng(32), 20000, 0.06)
    with _fresh() as ctx:
        gi = ctx.voxelize(pts, 0.01)
        g, layout, cl = po.voxelize(pts, 0.01)
        del layout
        assert list(gi.div_b) == list(g.div_b) == [1700, 1300, 900]
        assert gi.n_valid == g.n_valid and gi.n_occ == g.n_occ
        assert np.array_equal(ctx.downsampled().view(np.uint32), cl.view(np.uint32))
        _check_voxels(ctx, small, 0.01)
        too_wide = pts.copy()
        too_wide[1, :3] = (19.995, 19.995, 9.995)  # 2,000 x 2,000 x 1,000 voxels
        with pytest.raises(c3hlac._capi.C3HError):
            ctx.voxelize(too_wide, 0.01)
        _check_voxels(ctx, small, 0.01)


@pytest.mark.parametrize("variant,S,off", [(117, 10, (0, 0, 0)), (981, 10, (0, 0, 0)), (981, 7, (1, 2, 3)),
                                            (117, 0, (0, 0, 0)), (981, 3, (0, 0, 0)), (117, 40, (5, 0, 0))])
def test_extract_tiles_from_voxeliser_list(ctx, variant, S, off):
    """Round 6: c3h_extract right after c3h_voxelize stamps its tiles
    from the voxeliser's list of occupied voxels instead of streaming the grid.  Exact
    features and exist equal the oracle's on the same points (subdivisions with offsets,
    the whole-cloud histogram, sizes whose tiles split subdivisions), and the stream path
    (c3h_set_grid of the same words, no list) gives the same exist."""
    pts = synth.kinect_scene(400_000, grid=96, leaf=0.01, seed=synth.BASE_SEED + 611)
    gi = ctx.voxelize(pts, 0.01)
    g, layout, cl = po.voxelize(pts, 0.01)
    fe, sbo, hn = po.c3hlac(g, layout, cl, variant, THR, 0.01, S, off, exact=True)
    sb, hn2 = ctx.extract(variant, THR, S, off)
    assert tuple(sb) == tuple(sbo) and hn2 == hn
    assert np.array_equal(ctx.features(), fe)
    e_list = ctx.exist().copy()
    ctx.set_grid(ctx.grid(), tuple(gi.div_b), tuple(gi.min_b), 0.01)
    ctx.extract(variant, THR, S, off)
    assert np.array_equal(ctx.exist() > 0, e_list > 0)
