"""Generate tests/golden/shape_data.npz from the reference's shape clouds (run HERE only).

Inputs (read-only, /root/reference; absent on the GPU box, which only sees the .npz):
  color_chlac/demos/shape_data/<kind>_<shape>_<colour>.pcd            (98 binary XYZRGB clouds)
  color_chlac/demos/shape_data/<kind>_<shape>_<colour>_GRSD_CCHLAC.pcd (98 ASCII 137-dim rows,
      [GRSD 20 | ColorCHLAC-RI 117], written by color_chlac/test/example_GRSD_CCHLAC.cpp:13-85:
      thresholds 127, leaf 0.01, the whole cloud as one histogram)

Data only: the seven colour variants of one (kind, shape) share their coordinates bit for
bit and each cloud has one colour, so the fixture stores each shape's xyz once plus one
packed rgb per file, and the reference's 137 floats per file.  Reading goes through the
product's own readers (c3h_pcd_read_xyzrgb, c3h_feature_pcd_read), which are pinned
byte-for-byte on these files elsewhere (tests/test_pcdio.py).

    python tests/golden/gen_shape_fixture.py [reference_root]
"""
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT / "mapping-private_amd"))
import c3hlac  # noqa: E402


def main(ref_root="/root/reference"):
    d = Path(ref_root) / "color_chlac" / "demos" / "shape_data"
    names = sorted(p.stem for p in d.glob("*.pcd") if not p.stem.endswith("_GRSD_CCHLAC"))
    out = {}
    rgb, ref = [], []
    for nm in names:
        kind, shape, _colour = nm.split("_")
        pts = c3hlac.read_pcd(d / (nm + ".pcd"))
        key = "xyz_%s_%s" % (kind, shape)
        if key in out:
            assert np.array_equal(out[key].view(np.uint32), pts[:, :3].view(np.uint32)), nm
        else:
            out[key] = np.ascontiguousarray(pts[:, :3])
        col = np.unique(pts[:, 3].view(np.uint32))
        assert col.size == 1, nm
        rgb.append(col[0])
        f = c3hlac.read_feature(d / (nm + "_GRSD_CCHLAC.pcd"))
        assert f.shape == (1, 137), (nm, f.shape)
        ref.append(f[0])
    out["names"] = np.array(names)
    out["rgb"] = np.array(rgb, np.uint32)
    out["ref"] = np.array(ref, np.float32)
    dst = Path(__file__).resolve().parent / "shape_data.npz"
    np.savez_compressed(dst, **out)
    print("wrote %s: %d files, %d shapes" % (dst, len(names), sum(k.startswith("xyz_") for k in out)))


if __name__ == "__main__":
    main(*sys.argv[1:])
