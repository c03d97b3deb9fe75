"""Automatic colour threshold (calc_scene_auto_threshold.cpp): the C-ABI
threshold arithmetic against the numpy restatement (CPU), and the GPU histograms of the
occupied voxels against numpy (exact counts).  The reference ships no scene clouds for
this tool (demos/param/color_threshold.txt holds only its output), so the restatement is
"parity unpinned" beyond the tool's own source."""
import numpy as np
import pytest

import c3hlac
from c3hlac import _capi
import np_ref as npr
from c3hlac import synth
from conftest import THR  # noqa: F401  (shared constants module)


def _cases():
    rng = np.random.default_rng(7)
    yield "random", rng.integers(0, 1000, (3, 256))
    bi = np.zeros((3, 256), np.int64)
    bi[:, 40:60] = 500
    bi[:, 180:220] = 300
    yield "bimodal", bi
    one = np.zeros((3, 256), np.int64)
    one[:, 77] = 1234  # every voxel in one bin: the loop breaks at once, threshold 0
    yield "single_bin", one
    two = np.zeros((3, 256), np.int64)
    two[:, 0] = 5
    two[:, 255] = 7
    yield "two_extremes", two
    big = rng.integers(0, 10 ** 9, (3, 256))
    big[:, :30] = 0
    yield "large_counts", big
    skew = np.zeros((3, 256), np.int64)
    skew[0, 10] = 1
    skew[0, 200] = 10 ** 6
    skew[1, 3] = 10 ** 6
    skew[1, 250] = 1
    skew[2, 100:110] = 1
    skew[2, 100] += 10 ** 6 - 10
    yield "skewed", skew


@pytest.mark.parametrize("name,hist", list(_cases()), ids=[c[0] for c in _cases()])
def test_auto_threshold_matches_restatement(name, hist):
    hist = np.asarray(hist, np.int64)
    # every channel must hold the same total (one count per voxel per channel)
    tot = hist.sum(1)
    hist[1:] = (hist[1:] * (tot[0] / np.maximum(tot[1:], 1))[:, None]).astype(np.int64)
    hist[1:, 0] += tot[0] - hist[1:].sum(1)
    assert (hist >= 0).all() and (hist.sum(1) == hist[0].sum()).all()
    thr, ave = c3hlac.auto_threshold(hist)
    t_ref, a_ref = npr.auto_threshold(hist)
    assert list(thr) == list(t_ref)
    np.testing.assert_array_equal(ave, a_ref)


def test_auto_threshold_errors():
    with pytest.raises(_capi.C3HError):
        c3hlac.auto_threshold(np.zeros((3, 256), np.int64))
    bad = np.ones((3, 256), np.int64)
    bad[2, 5] = -1
    with pytest.raises(_capi.C3HError):
        c3hlac.auto_threshold(bad)


def test_histogram_restatement_counts_voxels():
    w = synth.random_words(16, 0.3, seed=4).reshape(-1)
    h = npr.color_histogram(w)
    assert (h.sum(1) == np.count_nonzero(w)).all()


@pytest.mark.gpu
def test_gpu_color_histogram_and_threshold(ctx):
    """Exact histograms on a Kinect frame, a dense grid and an odd-sized grid (nvox % 4 != 0,
    the scalar tail), accumulated over frames like the tool's file loop."""
    pts = synth.kinect_scene(300_000, grid=128, leaf=0.02, seed=synth.BASE_SEED + 9)
    ctx.voxelize(pts, 0.02)
    w1 = ctx.grid().reshape(-1).astype(np.uint32)
    h1 = ctx.color_histogram()
    np.testing.assert_array_equal(h1, npr.color_histogram(w1))
    w2 = synth.dense_words(64, seed=21).reshape(-1)
    ctx.set_grid(w2, (64, 64, 64))
    acc = ctx.color_histogram(h1.copy())
    np.testing.assert_array_equal(acc, npr.color_histogram(w1) + npr.color_histogram(w2))
    thr, ave = c3hlac.auto_threshold(acc)
    t_ref, a_ref = npr.auto_threshold(acc)
    assert list(thr) == list(t_ref)
    np.testing.assert_array_equal(ave, a_ref)
    w3 = synth.random_words((37, 23, 19), 0.4, seed=22).reshape(-1)
    ctx.set_grid(w3, (37, 23, 19))
    np.testing.assert_array_equal(ctx.color_histogram(), npr.color_histogram(w3))
    ctx.set_grid(np.zeros(8 * 8 * 8, np.uint32), (8, 8, 8))
    assert ctx.color_histogram().sum() == 0
