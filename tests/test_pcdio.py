"""Wire formats: PCD point clouds and the ASCII feature PCD of
readFeature / writeFeature (c3_hlac_tools.hpp:46-113), pinned on the reference's own data
files (tests/golden/ref_fixtures/pcd/SOURCES.txt)."""
from pathlib import Path

import numpy as np
import pytest

import c3hlac
from c3hlac import _capi

PCD = Path(__file__).resolve().parent / "golden" / "ref_fixtures" / "pcd"
CLOUDS = ["noisy_torus_blue.pcd", "bowl1_0000.pcd", "tmp_normal.pcd", "obj_torus_black.pcd"]
FEATURES = ["noisy_cube_black_GRSD_CCHLAC.pcd", "noiseless_torus_red_GRSD_CCHLAC.pcd"]


def _header(path):
    h, raw = {}, open(path, "rb").read()
    pos = 0
    while True:
        end = raw.index(b"\n", pos)
        line = raw[pos:end].decode()
        pos = end + 1
        t = line.split()
        if not t or t[0].startswith("#"):
            continue
        h[t[0]] = t[1:]
        if t[0] == "DATA":
            return h, raw, pos


def _numpy_cloud(path):
    """Independent restatement: numpy parse of the same file (x, y, z, rgb bits)."""
    h, raw, end = _header(path)
    fields, n = h["FIELDS"], int(h["POINTS"][0])
    idx = [fields.index(k) for k in ("x", "y", "z", "rgb")]
    if h["DATA"][0] == "ascii":
        vals = np.loadtxt(path, skiprows=len(raw[:end].decode().splitlines()), dtype=np.float64, ndmin=2)
        return vals[:, idx].astype(np.float32)
    stride = 4 * len(fields)
    start = len(raw) - n * stride  # the data ends the file (header end or the next page)
    assert start in (end, (end + 4095) // 4096 * 4096)
    a = np.frombuffer(raw[start:], np.float32).reshape(n, len(fields))
    return np.ascontiguousarray(a[:, idx])


@pytest.mark.parametrize("name", CLOUDS)
def test_read_cloud_matches_numpy(name):
    got = c3hlac.read_pcd(PCD / name)
    ref = _numpy_cloud(PCD / name)
    assert got.shape == ref.shape and got.shape[0] == int(_header(PCD / name)[0]["POINTS"][0])
    np.testing.assert_array_equal(got.view(np.uint32), ref.view(np.uint32))
    assert np.isfinite(got[:, :3]).all() and np.abs(got[:, :3]).max() < 100


def test_cloud_colours_follow_the_file_names():
    """A size-independent pin on the page-aligned binary layout: the blue torus is blue."""
    c = c3hlac.read_pcd(PCD / "noisy_torus_blue.pcd").view(np.uint32)[:, 3]
    r, g, b = (c >> 16) & 255, (c >> 8) & 255, c & 255
    assert b.mean() > r.mean() + 50 and b.mean() > g.mean() + 50


@pytest.mark.parametrize("name", FEATURES)
def test_feature_pcd_round_trip_is_byte_identical(name, tmp_path):
    """readFeature then writeFeature (FIELDS vfh, as grsd_colorCHLAC_tools.hpp writes them)
    reproduces the reference-written file byte for byte."""
    f = c3hlac.read_feature(PCD / name)
    assert f.shape == (1, 137)
    out = tmp_path / "f.pcd"
    c3hlac.write_feature(out, f, remove_zero=False, fields="vfh")
    assert out.read_bytes() == (PCD / name).read_bytes()


def test_write_feature_drops_zero_rows(tmp_path):
    rng = np.random.default_rng(3)
    f = rng.random((6, 117), dtype=np.float32)
    f[[1, 4]] = 0
    out = tmp_path / "w.pcd"
    c3hlac.write_feature(out, f)  # c3_hlac_tools.hpp default: remove_0_flg, FIELDS descriptor
    lines = out.read_text().splitlines()
    assert lines[:9] == ["# .PCD v.7 - Point Cloud Data file format", "FIELDS descriptor", "SIZE 4", "TYPE F",
                         "COUNT 117", "WIDTH 4", "HEIGHT 1", "POINTS 4", "DATA ascii"]
    assert lines[9] == "".join("%f " % v for v in f[0])
    back = c3hlac.read_feature(out)
    np.testing.assert_allclose(back, f[[0, 2, 3, 5]], atol=5e-7)


def test_pcd_errors(tmp_path):
    with pytest.raises(_capi.C3HError):
        c3hlac.read_pcd(tmp_path / "missing.pcd")
    bad = tmp_path / "bad.pcd"
    bad.write_text("# .PCD v.7\nFIELDS x y z\nSIZE 4 4 4\nTYPE F F F\nCOUNT 1 1 1\nPOINTS 1\nDATA ascii\n1 2 3\n")
    with pytest.raises(_capi.C3HError):  # no rgb field
        c3hlac.read_pcd(bad)
    with pytest.raises(_capi.C3HError):
        c3hlac.read_feature(tmp_path / "missing.pcd")
