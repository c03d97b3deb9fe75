"""Real Kinect object views from the reference (run HERE only; /root/reference is absent on
the GPU box).

color_feature_classification/demos/data/obj000..062/<name>_<angle>.pcd are 1,512 captured
views (63 objects x 24 angles, 258..19,005 XYZRGB points each): the reference's own sensor
data, with the voxel-boundary statistics of a real depth camera (quantised depth puts many
points on cell faces).  Data only, read with the product's c3h_pcd_read_xyzrgb.

    python tests/golden/gen_kinect_views.py            # the committed sample
    python tests/golden/gen_kinect_views.py --all DST  # all 1,512 views (not committed: a
                                                       # measurement run copies it in-tree)

Sample: every 12th view in sorted order (126 views, two angles of each object),
tests/golden/kinect_views_126.npz: pts (concatenated n x 4 float32: x, y, z, rgb bits),
starts (n_views + 1 offsets), names.
"""
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT / "mapping-private_amd"))
import c3hlac  # noqa: E402

SRC = Path("/root/reference/color_feature_classification/demos/data")


def collect(files):
    pts = [c3hlac.read_pcd(f) for f in files]
    starts = np.zeros(len(pts) + 1, np.int64)
    starts[1:] = np.cumsum([len(p) for p in pts])
    names = np.array(["%s/%s" % (f.parent.name, f.stem) for f in files])
    return dict(pts=np.concatenate(pts).astype(np.float32), starts=starts, names=names)


def main(argv):
    files = sorted(SRC.glob("obj*/*.pcd"))
    assert len(files) == 1512, len(files)
    if len(argv) >= 2 and argv[0] == "--all":
        dst = Path(argv[1])
        dst.parent.mkdir(parents=True, exist_ok=True)
        np.savez(dst, **collect(files))
        print("wrote", dst)
        return
    dst = Path(__file__).resolve().parent / "kinect_views_126.npz"
    np.savez_compressed(dst, **collect(files[::12]))
    print("wrote", dst, dst.stat().st_size)


if __name__ == "__main__":
    main(sys.argv[1:])
