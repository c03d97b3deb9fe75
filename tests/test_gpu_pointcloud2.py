"""sensor_msgs/PointCloud2 ingestion (pcl::fromROSMsg, detect_object.cpp:142) through
c3h_voxelize_pointcloud2: an organised 640 x 480 Kinect-style message (NaN holes, padded
point_step 32 with rgb at byte 16, row padding), little- and big-endian, host and device
bytes -> the same grid, leaf layout and downsampled cloud as c3h_voxelize on the
equivalent x, y, z, rgb array (bit-exact)."""
import numpy as np
import pytest

from c3hlac import synth

pytestmark = pytest.mark.gpu


def _message(pts, big=False, row_pad=16):
    W, Hh = 640, 480
    n = W * Hh
    xyz = np.full((n, 4), np.nan, np.float32)
    xyz[:, 3] = 0
    xyz[:len(pts)] = pts[:n]
    rng = np.random.default_rng(0)
    xyz[rng.random(n) < 0.1, :3] = np.nan  # holes of an organised cloud
    ps = 32
    rs = W * ps + row_pad
    buf = np.zeros((Hh, rs), np.uint8)
    dt = ">u4" if big else "<u4"
    words = xyz.view(np.uint32).astype(dt)
    rows = np.zeros((Hh, W, ps), np.uint8)
    for k, off in enumerate((0, 4, 8, 16)):  # x y z (pad) rgb
        rows[:, :, off:off + 4] = np.ascontiguousarray(words[:, k]).view(np.uint8).reshape(Hh, W, 4)
    rows[:, :, 12:16] = 0xAB  # padding bytes must be ignored
    buf[:, :W * ps] = rows.reshape(Hh, W * ps)
    msg = dict(height=Hh, width=W, point_step=ps, row_step=rs, is_bigendian=int(big),
               fields={"x": 0, "y": 4, "z": 8, "rgb": 16}, data=buf.reshape(-1))
    return msg, xyz


@pytest.mark.parametrize("big,on_dev", [(False, False), (True, False), (False, True)])
def test_pointcloud2_equals_xyzrgb(ctx, big, on_dev):
    import torch
    pts = synth.kinect_scene(640 * 480, grid=64, leaf=0.02, seed=31)
    msg, xyz = _message(pts, big)
    ctx.voxelize(xyz, 0.02, z_limit=1.5)
    g0, lay0, down0 = ctx.grid().copy(), ctx.leaf_layout().copy(), ctx.downsampled().copy()
    if on_dev:
        msg = dict(msg, data=torch.from_numpy(msg["data"]).cuda())
    ctx.voxelize_pointcloud2(msg, 0.02, z_limit=1.5)
    assert np.array_equal(ctx.grid(), g0)
    assert np.array_equal(ctx.leaf_layout(), lay0)
    assert np.array_equal(ctx.downsampled().view(np.uint32), down0.view(np.uint32))


def test_pointcloud2_bad_fields(ctx):
    msg, _ = _message(synth.kinect_scene(1000, grid=16, leaf=0.05, seed=1))
    with pytest.raises(Exception, match="outside point_step"):
        ctx.voxelize_pointcloud2(dict(msg, fields={"x": 0, "y": 4, "z": 30}), 0.05)
