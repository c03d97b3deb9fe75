"""CPU checks of the PCA training boundary that need no device:
rotateFeature90 maps and the PCA file format.

- The rotation maps of the product (c3h_rotate_map) and of the oracle
  (pca_oracle.rotate_map) equal the ones oracle/gen_rotmap.py extracted mechanically from
  the reference source (tests/golden/rotate90_map.json, c3_hlac.cpp:49-172).
- c3h_pca_write reproduces the reference's own PCA files byte for byte after
  c3h_pca_read (models_offline_r: the compress axis and three model subspaces), and the
  ASCII form round-trips through the reader."""
import json

import numpy as np
import pytest

import c3hlac
import pca_oracle as pco
from conftest import GOLDEN

MODES = ["R_MODE_1", "R_MODE_2", "R_MODE_3", "R_MODE_4"]
REF_PCA = ["compress_axis", "000/pca_result", "001/pca_result", "002/pca_result"]


@pytest.fixture(scope="module")
def golden_maps():
    return json.loads((GOLDEN / "rotate90_map.json").read_text())


@pytest.mark.parametrize("dim", [981, 495, 486])
def test_rotate_maps_match_reference_extraction(golden_maps, dim):
    for k, name in enumerate(MODES):
        half = np.asarray(golden_maps[name])
        exp = np.arange(dim)
        exp[6:474] = half[6:474]
        if dim == 981:
            exp[495 + 6:495 + 474] = 495 + half[6:474]
        assert np.array_equal(c3hlac.rotate_map(dim, k), exp), (dim, name)
        assert np.array_equal(pco.rotate_map(dim, k), exp), (dim, name)
        assert np.array_equal(np.sort(exp), np.arange(dim))  # a permutation


def test_rotate_bad_dimension_is_an_error():
    with pytest.raises(c3hlac._capi.C3HError):
        c3hlac.rotate_map(117, 0)


def test_rotations24_distinct():
    f = np.random.default_rng(1).random(981).astype(np.float32)
    assert len({v.tobytes() for v in pco.rotations24(f)}) == 24


@pytest.mark.parametrize("rel", REF_PCA)
def test_pca_write_reproduces_reference_files(tmp_path, rel):
    path = GOLDEN / "ref_fixtures" / "models_offline_r" / rel
    axis, var, mean = c3hlac.pca_read(path)
    out = tmp_path / "pca"
    c3hlac.pca_write(out, axis, var, mean)
    assert out.read_bytes() == path.read_bytes()
    assert pco.write_binary(axis, var, mean) == path.read_bytes()
    # the reference's files are sortVecAndVal output: variances non-increasing
    assert (np.diff(var) <= 0).all()


def test_pca_ascii_round_trip(tmp_path):
    rng = np.random.default_rng(3)
    d = 17
    axis = rng.standard_normal((d, d)).astype(np.float32)
    var = np.sort(rng.random(d).astype(np.float32))[::-1].copy()
    mean = rng.random(d).astype(np.float32)
    for m in (mean, None):
        out = tmp_path / "a.txt"
        c3hlac.pca_write(out, axis, var, m, ascii=True)
        a2, v2, m2 = c3hlac.pca_read(out, ascii=True)
        np.testing.assert_allclose(a2, axis, atol=5e-7)  # "%f": 6 decimals
        np.testing.assert_allclose(v2, var, atol=5e-7)
        assert (m2 is None) == (m is None)
        if m is not None:
            np.testing.assert_allclose(m2, m, atol=5e-7)
        lines = out.read_text().splitlines()
        assert lines[0] == str(d) and len(lines) == 1 + d + d + (d if m is not None else 0)
