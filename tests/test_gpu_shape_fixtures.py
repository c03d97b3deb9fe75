"""The HIP path against the reference's own feature vectors (GPU).

c3h_voxelize + c3h_extract (ColorCHLAC-RI: variant 117, C3H_COLOR_CHLAC, thresholds 127,
leaf 0.01, one histogram for the whole cloud) on the 47 noiseless shape clouds whose
<name>_GRSD_CCHLAC.pcd rows the oracle reproduces (tests/test_shape_fixtures.py; the
other 51 files have stated causes there).  Chain of evidence, per file:
  - the GPU's grid, leaf layout and centroids == the oracle's (bit-exact, PCL 1.0 /
    Eigen 3.0 arithmetic: centroid = sum * (1/n), neighbour base floor(c / leaf));
  - the GPU's exact-integer histogram == the oracle's exact-integer mode (bit-exact);
  - both within 5e-5 of max(|v|, 1) of the reference's vector (zero-order bins in the
    current normalisation, x2): the reference accumulates in fp32 in voxel order, which
    rounds the >2^24 auto-product sums (e.g. 324.999 for 325 voxels x 65025 / 65025).
Also on the same clouds: C3 variants (981 / 117, both C3 colour tables) and subdivided
extraction, bit-exact against the oracle.
"""
import numpy as np
import pytest

import c3hlac
import pyoracle as po
from test_shape_fixtures import FIXTURES, LEAF, MATCHED, THR, c3_part

pytestmark = pytest.mark.gpu


def _voxelize_both(ctx, pts):
    po.set_voxel_semantics(True)
    gi = ctx.voxelize(pts, LEAF)
    g, layout, cloud = po.voxelize(pts, LEAF)
    assert list(gi.div_b) == list(g.div_b) and list(gi.min_b) == list(g.min_b) and gi.n_occ == g.n_occ
    assert np.array_equal(ctx.leaf_layout(), layout)
    assert np.array_equal(ctx.downsampled().view(np.uint32), cloud.view(np.uint32))
    return g, layout, cloud


@pytest.mark.parametrize("fx", MATCHED, ids=[f[0] for f in MATCHED])
def test_gpu_reproduces_reference_vectors(ctx, fx):
    nm, _, _, _, pts, ref = fx
    g, layout, cloud = _voxelize_both(ctx, pts)
    sb, hn = ctx.extract(117, THR, 0, color_mode=c3hlac.COLOR_CHLAC)
    assert hn == 1 and tuple(sb) == (0, 0, 0)
    f = ctx.features()[0]
    fe, _, _ = po.c3hlac(g, layout, cloud, 117, THR, LEAF, 0, color_mode=po.COLOR_CHLAC, exact=True)
    assert np.array_equal(f, fe[0]), nm
    r = c3_part(ref)
    err = np.abs(f - r) / np.maximum(np.abs(r), 1)
    assert err.max() <= 5e-5, (nm, np.flatnonzero(err > 5e-5))


@pytest.mark.parametrize("shape", ["noiseless_cone", "noiseless_cube", "noisy_sphere", "noisy_dice"])
def test_gpu_shape_clouds_other_estimators(ctx, shape):
    """The same clouds through the C3 estimators and subdivisions, bit-exact vs the oracle
    (the cube's and dice's faces lie on cell faces: their centroids exercise the off-cell
    correction under the reciprocal mean)."""
    fxs = [f for f in FIXTURES if f[0].startswith(shape + "_") and f[3] in ("orange", "purple")]
    assert fxs
    for nm, _, _, _, pts, _ in fxs:
        g, layout, cloud = _voxelize_both(ctx, pts)
        for variant, S, off, mode in ((981, 0, (0, 0, 0), c3hlac.COLOR_C3_DOUBLE),
                                      (117, 3, (0, 0, 0), c3hlac.COLOR_C3_FLOAT),
                                      (981, 4, (1, 0, 2), c3hlac.COLOR_CHLAC),
                                      (117, 5, (0, 1, 0), c3hlac.COLOR_CHLAC)):
            fe, sbo, hn = po.c3hlac(g, layout, cloud, variant, (127, 127, 127), LEAF, S, off, color_mode=mode,
                                    exact=True)
            if hn < 0:
                continue
            sb, hn2 = ctx.extract(variant, (127, 127, 127), S, off, color_mode=mode)
            assert tuple(sb) == tuple(sbo) and hn2 == hn
            assert np.array_equal(ctx.features(), fe), (nm, variant, S, off, mode)
