"""c3h_allgather_detections: the RCCL gather of the frame-sharded multi-GPU path
 on a single-rank communicator the test creates through librccl itself
(ncclGetUniqueId + ncclCommInitRank, as a C++ caller would): the records of a pipelined
c3h_stream_frames batch arrive unchanged after the stream is flushed.  The N-rank data
flow is covered by tests/test_dist.py (gloo, world size 2)."""
import ctypes as C

import numpy as np
import pytest

from c3hlac import synth
from conftest import THR

pytestmark = pytest.mark.gpu


def test_allgather_detections_single_rank(ctx):
    import torch
    class NcclId(C.Structure):  # ncclUniqueId, passed by value
        _fields_ = [("internal", C.c_char * 128)]

    rccl = C.CDLL("librccl.so.1")
    rccl.ncclGetUniqueId.argtypes = [C.POINTER(NcclId)]
    rccl.ncclCommInitRank.argtypes = [C.POINTER(C.c_void_p), C.c_int, NcclId, C.c_int]
    rccl.ncclCommDestroy.argtypes = [C.c_void_p]
    uid = NcclId()
    assert rccl.ncclGetUniqueId(C.byref(uid)) == 0
    comm = C.c_void_p()
    assert rccl.ncclCommInitRank(C.byref(comm), 1, uid, 0) == 0
    try:
        G, LEAF, S = 64, 0.02, 8
        grids = []
        for s in range(4):
            ctx.voxelize(synth.kinect_scene(100_000, grid=G, leaf=LEAF, seed=synth.BASE_SEED + 700 + s), LEAF)
            grids.append(torch.from_numpy(ctx.grid().view(np.int32).copy()).cuda())
        axis_t, var, axis_q = synth.random_bases(117, 24, 3, 6, seed=9)
        ctx.search_setup(axis_t, var, axis_q)
        ctx.set_rank(1)
        ctx.set_batch(4)
        ptrs = np.array([g.data_ptr() for g in grids], np.uint64)
        d_out = torch.zeros((4, 3 * 3), dtype=torch.int64, device="cuda:0")
        torch.cuda.synchronize()
        ctx.run_frames(ptrs, (G,) * 3, (0, 0, 0), LEAF, 117, THR, S, (2, 2, 2), 10, True, d_out.data_ptr(),
                       stream=True)
        d_all = torch.full_like(d_out, -1)
        rc = ctx.lib.c3h_allgather_detections(ctx.h, comm, C.c_void_p(d_out.data_ptr()), 4 * 3,
                                              C.c_void_p(d_all.data_ptr()))
        assert rc == 0, ctx.lib.c3h_last_error(ctx.h)
        ctx.synchronize()
        got, ref = d_all.cpu().numpy(), d_out.cpu().numpy()
        assert np.array_equal(got, ref)
        assert (ref.reshape(4, 3, 3)[:, :, 0].view(np.float64) > 0).all()
    finally:
        rccl.ncclCommDestroy(comm)
