"""Host-side logic of the points-in binding (no GPU): Context.prepare_point_frames's checks
and pointer arrays for host clouds, PointFrames, and Context.point_batch's batch choice."""
import numpy as np
import pytest

import c3hlac


class _Dev:  # prepare_point_frames reads only the context's device index
    device = 0


def _prep(frames):
    return c3hlac.Context.prepare_point_frames(_Dev(), frames)


def test_prepare_host_frames_pointer_and_count_arrays():
    a = np.zeros((5, 4), np.float32)
    b = np.arange(12, dtype=np.float64).reshape(3, 4)  # converted to float32, kept alive
    pf = _prep([a, b])
    assert isinstance(pf, c3hlac.PointFrames) and len(pf) == 2 and not pf.on_device
    assert pf.ns.tolist() == [5, 3]
    assert pf.ptrs[0] == a.ctypes.data
    kept = pf._keep[1]
    assert kept.dtype == np.float32 and pf.ptrs[1] == kept.ctypes.data
    np.testing.assert_array_equal(kept, b.astype(np.float32))


def test_prepare_rejects_wrong_shape():
    with pytest.raises(ValueError, match="frame 1 must be"):
        _prep([np.zeros((2, 4), np.float32), np.zeros((2, 3), np.float32)])


def test_prepare_empty_list():
    pf = _prep([])
    assert len(pf) == 0 and pf.ptrs.size == 0


def test_point_batch_choice():
    # 32 frames per batch from 256 frames up (profiles/r6/shard/), 64 below
    assert c3hlac.Context.point_batch(512) == 32
    assert c3hlac.Context.point_batch(256) == 32
    assert c3hlac.Context.point_batch(255) == 64
    assert c3hlac.Context.point_batch(64) == 64
    assert c3hlac.Context.point_batch(1) == 64
