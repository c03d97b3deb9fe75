"""GPU parity of the production path at the shapes the bench and the multi-GPU configs use.

- The pipelined tick (c3h_run_frames and the streaming c3h_stream_frames) at the bench's
  exact shape -- BASELINE configs[2]: 256^3, C3-HLAC-117, S=10, compress 117->100,
  10 models x r=20, box 2x2x2, rank 1, exist threshold 100 -- at 8, 32 and 64 frames per
  batch over several full batches: every frame's detections against the float64 oracle
  run on the same grid (not against the HIP single-frame path), and the last frame's
  feature rows (exact-integer oracle) and position scores (float64 oracle).
- BASELINE configs[3]-shaped single-GPU run: 64 independent 1M-point frames voxelised
  on the GPU at 128^3 and pushed through c3h_run_frames (C3-HLAC-981 + 1-model search,
  the configs[1] pipeline), sampled frames checked end to end against the oracle.

Scores: within 1e-5 relative of the float64 oracle.  Detections: the oracle's (x, y, z,
mode) unless two positions score within that tolerance of each other (then the GPU's pick
must be one of the tied maxima)."""
import concurrent.futures as cf

import numpy as np
import pytest

import c3hlac
import pyoracle as po
from c3hlac import synth
from conftest import THR

pytestmark = pytest.mark.gpu

RTOL = 1e-5
G, LEAF, S, F, D, M, R, BOX, EXIST = 256, 0.01, 10, 117, 100, 10, 20, (2, 2, 2), 100
N_DISTINCT = 40


def _check_det(rec, scores_f64, shape, tag):
    """rec: (M, 3) int64 c3h_det words of one frame; scores_f64: (M, P) oracle scores of
    the single mode (box 2x2x2), P in (z, y, x) scan order."""
    ze, ye, xe = shape
    for m in range(rec.shape[0]):
        s = float(rec[m, 0:1].view(np.float64)[0])
        x, y, z, mode = (int(v) for v in rec[m, 1:3].view(np.int32))
        ref = scores_f64[m]
        best = int(np.argmax(ref))  # first maximum in scan order = searchPart's strict '>'
        assert mode == 0, (tag, m, mode)
        p = (z * ye + y) * xe + x
        assert abs(s - ref[p]) <= RTOL * ref[p], (tag, m, s, ref[p])
        if p != best:  # only a tie within tolerance may pick another position
            assert ref[p] >= ref[best] * (1 - 2 * RTOL), (tag, m, (x, y, z), np.unravel_index(best, shape))


@pytest.fixture(scope="module")
def prod(ctx):
    """40 distinct resident 256^3 grids (10 ray-cast scenes voxelised on the GPU, each
    with 3 x-shifted copies) and the oracle's results on every one of them."""
    import torch
    dev = torch.device("cuda", 0)
    grids = []
    for s in range(N_DISTINCT // 4):
        ctx.voxelize(synth.kinect_scene(1_000_000, grid=G, leaf=LEAF, seed=synth.BASE_SEED + 500 + s), LEAF)
        w = ctx.grid().reshape(G, G, G)
        for k in range(4):
            grids.append(np.ascontiguousarray(np.roll(w, 37 * k, axis=2)).reshape(-1))
    d_grids = [torch.from_numpy(w.view(np.int32)).to(dev) for w in grids]
    torch.cuda.synchronize()
    axis_t, var, axis_q = synth.random_bases(F, D, M, R, seed=synth.BASE_SEED)
    ap = synth.whiten(axis_t, var)

    def oracle(i):
        g, layout, cloud = po.grid_inputs(grids[i], (G,) * 3, LEAF)
        fe, sb, _ = po.c3hlac(g, layout, cloud, F, THR, LEAF, S, exact=True)
        ex = po.exist(fe)
        _, _, sc = po.search(sb, fe, ex, ap, axis_q, BOX, 1, EXIST, dbl=True, want_scores=True)
        return fe, ex, sc

    with cf.ThreadPoolExecutor(8) as pool:  # the C oracle releases the GIL
        ref = list(pool.map(oracle, range(N_DISTINCT)))
    ctx.search_setup(axis_t, var, axis_q)
    ctx.set_rank(1)
    return dict(grids=grids, d_grids=d_grids, ref=ref)


def _frame_grid(i):
    return (7 * i) % N_DISTINCT  # neighbouring frames of a batch read different grids


P1 = -(-G // S) - BOX[0] + 1  # 26 subdivisions per axis -> 25 box positions


@pytest.mark.parametrize("batch,nbatches", [(8, 3), (32, 3), (64, 2)])
def test_pipeline_at_bench_shape_vs_oracle(ctx, prod, batch, nbatches):
    import torch
    nfr = batch * nbatches + batch // 2  # full batches + a ragged last one
    ptrs = np.array([prod["d_grids"][_frame_grid(i)].data_ptr() for i in range(nfr)], np.uint64)
    d_out = torch.zeros((nfr, M * 3), dtype=torch.int64, device="cuda:0")
    torch.cuda.synchronize()
    ctx.set_batch(batch)
    ctx.set_pipeline(True)
    ctx.run_frames(ptrs, (G,) * 3, (0, 0, 0), LEAF, F, THR, S, BOX, EXIST, True, d_out.data_ptr())
    ctx.synchronize()
    got = d_out.cpu().numpy().reshape(nfr, M, 3)
    for i in range(nfr):
        _check_det(got[i], prod["ref"][_frame_grid(i)][2].reshape(M, -1), (P1, P1, P1), "frame %d" % i)
    # the context holds the last frame's state: exact feature rows, exist, scores
    fe, ex, sc = prod["ref"][_frame_grid(nfr - 1)]
    gex = ctx.exist()
    bad = np.flatnonzero(gex != ex)
    assert bad.size == 0, ("exist", bad.size, bad[:8].tolist(), gex[bad[:8]].tolist(), ex[bad[:8]].tolist())
    gf = ctx.features()
    bad = np.flatnonzero((gf != fe).any(1))
    assert bad.size == 0, ("features", bad.size, bad[:8].tolist())
    gs = ctx.scores()
    assert np.array_equal(gs < 0, sc < 0)
    ok = sc > 0
    np.testing.assert_allclose(gs[ok], sc[ok], rtol=RTOL)


def test_stream_frames_at_bench_shape_vs_oracle(ctx, prod):
    """c3h_stream_frames: uneven pushes (the pipeline stays filled between calls), a
    detection read mid-stream once three later batches were pushed, then flush."""
    import torch
    B = 32
    sizes = [B, 3 * B, 5, B + 7, 2 * B]  # ragged pushes: every call's tail is its own batch
    nfr = sum(sizes)
    ptrs = np.array([prod["d_grids"][_frame_grid(i)].data_ptr() for i in range(nfr)], np.uint64)
    d_out = torch.zeros((nfr, M * 3), dtype=torch.int64, device="cuda:0")
    torch.cuda.synchronize()
    ctx.set_batch(B)
    ctx.set_pipeline(True)
    f0 = 0
    rec = M * 3 * 8
    for k, n in enumerate(sizes):
        ctx.run_frames(ptrs[f0:f0 + n], (G,) * 3, (0, 0, 0), LEAF, F, THR, S, BOX, EXIST, True,
                       d_out.data_ptr() + f0 * rec, stream=True)
        f0 += n
        if k == 1:  # batches 0 (call 0) and 1..3 (call 1) pushed: batch 0 is complete
            ctx.synchronize()
            got = d_out[:B].cpu().numpy().reshape(B, M, 3)
            for i in range(B):
                _check_det(got[i], prod["ref"][_frame_grid(i)][2].reshape(M, -1), (P1, P1, P1), "mid %d" % i)
    ctx.stream_flush()
    ctx.synchronize()
    got = d_out.cpu().numpy().reshape(nfr, M, 3)
    for i in range(nfr):
        _check_det(got[i], prod["ref"][_frame_grid(i)][2].reshape(M, -1), (P1, P1, P1), "frame %d" % i)
    # any entry point that touches the context's buffers drains an open stream first
    ctx.run_frames(ptrs[:B + 3], (G,) * 3, (0, 0, 0), LEAF, F, THR, S, BOX, EXIST, True, d_out.data_ptr(),
                   stream=True)
    ctx.set_rank(1)  # drains
    ctx.synchronize()
    got = d_out[:B + 3].cpu().numpy().reshape(B + 3, M, 3)
    for i in range(B + 3):
        _check_det(got[i], prod["ref"][_frame_grid(i)][2].reshape(M, -1), (P1, P1, P1), "drain %d" % i)


def test_stream_switched_mid_stream(ctx, prod):
    """c3h_set_stream while a frame stream is open (no host sync): the open batches finish
    on the old stream before anything the new stream runs, and the detections of both
    pushes equal c3h_run_frames' (set_stream drains and joins the streams)."""
    import torch
    B, n1, n2 = 8, 27, 21
    nfr = n1 + n2
    ptrs = np.array([prod["d_grids"][_frame_grid(i)].data_ptr() for i in range(nfr)], np.uint64)
    d_out = torch.zeros((nfr, M * 3), dtype=torch.int64, device="cuda:0")
    d_ref = torch.zeros((nfr, M * 3), dtype=torch.int64, device="cuda:0")
    torch.cuda.synchronize()
    ctx.set_batch(B)
    ctx.set_pipeline(True)
    side = torch.cuda.Stream()
    rec = M * 3 * 8
    try:
        ctx.run_frames(ptrs[:n1], (G,) * 3, (0, 0, 0), LEAF, F, THR, S, BOX, EXIST, True, d_out.data_ptr(),
                       stream=True)
        ctx.set_stream(side.cuda_stream)
        ctx.run_frames(ptrs[n1:], (G,) * 3, (0, 0, 0), LEAF, F, THR, S, BOX, EXIST, True,
                       d_out.data_ptr() + n1 * rec, stream=True)
        ctx.stream_flush()
        ctx.synchronize()
    finally:
        ctx.set_stream(None)
    ctx.run_frames(ptrs, (G,) * 3, (0, 0, 0), LEAF, F, THR, S, BOX, EXIST, True, d_ref.data_ptr())
    ctx.synchronize()
    got, ref = d_out.cpu().numpy(), d_ref.cpu().numpy()
    assert np.array_equal(got, ref)
    got = got.reshape(nfr, M, 3)
    for i in range(0, nfr, 5):
        _check_det(got[i], prod["ref"][_frame_grid(i)][2].reshape(M, -1), (P1, P1, P1), "switch %d" % i)


def test_bases_swapped_between_unsynchronised_runs(ctx, prod):
    """c3h_search_setup while a streamed run is still queued (no host sync): the queued
    frames must finish on the old bases, the next run must use the new ones."""
    import torch
    B, nfr = 8, 19
    ptrs = np.array([prod["d_grids"][_frame_grid(i)].data_ptr() for i in range(nfr)], np.uint64)
    d_old = torch.zeros((nfr, M * 3), dtype=torch.int64, device="cuda:0")
    d_new = torch.zeros((nfr, M * 3), dtype=torch.int64, device="cuda:0")
    torch.cuda.synchronize()
    ctx.set_batch(B)
    ctx.set_pipeline(True)
    ctx.run_frames(ptrs, (G,) * 3, (0, 0, 0), LEAF, F, THR, S, BOX, EXIST, True, d_old.data_ptr(), stream=True)
    axis_t2, var2, axis_q2 = synth.random_bases(F, D, M, R, seed=synth.BASE_SEED + 77)
    try:
        ctx.search_setup(axis_t2, var2, axis_q2)  # same sizes: the buffers are overwritten in place
        ctx.set_rank(1)
        ctx.run_frames(ptrs, (G,) * 3, (0, 0, 0), LEAF, F, THR, S, BOX, EXIST, True, d_new.data_ptr())
        ctx.synchronize()
        old = d_old.cpu().numpy().reshape(nfr, M, 3)
        new = d_new.cpu().numpy().reshape(nfr, M, 3)
        ap2 = synth.whiten(axis_t2, var2)
        for i in range(nfr):
            fe, ex, sc = prod["ref"][_frame_grid(i)]
            _check_det(old[i], sc.reshape(M, -1), (P1, P1, P1), "old bases, frame %d" % i)
            if i % 6 == 0:
                _, _, sc2 = po.search((P1 + 1,) * 3, fe, ex, ap2, axis_q2, BOX, 1, EXIST, dbl=True, want_scores=True)
                _check_det(new[i], sc2.reshape(M, -1), (P1, P1, P1), "new bases, frame %d" % i)
    finally:
        axis_t, var, axis_q = synth.random_bases(F, D, M, R, seed=synth.BASE_SEED)
        ctx.search_setup(axis_t, var, axis_q)
        ctx.set_rank(1)


def test_config4_shape_voxelise_and_run_frames(ctx):
    """BASELINE configs[3] on one GPU: 64 independent 1M-point frames (8 ray-cast scenes,
    each under 8 colour masks and x translations by whole cells) voxelised on the GPU at
    128^3, then C3-HLAC-981 + 1-model search for all 64 in one c3h_run_frames (32 frames
    per batch); every 8th frame is re-computed by the oracle from its points (voxel grid
    bit-exact, detection within RTOL)."""
    import torch
    G2, L2, S2, D2, R2 = 128, 0.02, 10, 100, 20
    base = [synth.kinect_scene(1_000_000, grid=G2, leaf=L2, seed=synth.BASE_SEED + 900 + s) for s in range(8)]
    axis_t, var, axis_q = synth.random_bases(981, D2, 1, R2, seed=synth.BASE_SEED + 1)
    ap = synth.whiten(axis_t, var)

    def frame_points(i):
        pts = base[i % 8].copy()
        k = i // 8
        rgb = pts[:, 3].view(np.uint32) ^ np.uint32((k * 0x2F1D37) & 0xFFFFFF)
        pts[:, 3] = rgb.view(np.float32)
        pts[:, 0] = (pts[:, 0].astype(np.float64) + k * L2).astype(np.float32)
        return pts

    d_grids, sampled = [], {}
    for i in range(64):
        pts = frame_points(i)
        gi = ctx.voxelize(pts, L2)
        assert list(gi.div_b) == [G2] * 3
        w = torch.empty(G2 ** 3, dtype=torch.int32, device="cuda:0")
        ctx.lib.c3h_get_grid(ctx.h, c3hlac.ptr(w), 1)
        d_grids.append(w)
        if i % 8 == 3:
            sampled[i] = (pts, ctx.grid().copy())
    ctx.search_setup(axis_t, var, axis_q)
    ctx.set_rank(1)
    ctx.set_batch(32)
    ctx.set_pipeline(True)
    d_out = torch.zeros((64, 3), dtype=torch.int64, device="cuda:0")
    torch.cuda.synchronize()
    ctx.run_frames(np.array([g.data_ptr() for g in d_grids], np.uint64), (G2,) * 3, (0, 0, 0), L2, 981, THR, S2,
                   BOX, EXIST, True, d_out.data_ptr())
    ctx.synchronize()
    got = d_out.cpu().numpy().reshape(64, 1, 3)
    P2 = -(-G2 // S2) - BOX[0] + 1

    def oracle(i):
        pts, words = sampled[i]
        g, layout, cloud = po.voxelize(pts, L2)
        fe, sb, _ = po.c3hlac(g, layout, cloud, 981, THR, L2, S2, exact=True)
        ex = po.exist(fe)
        _, _, sc = po.search(sb, fe, ex, ap, axis_q, BOX, 1, EXIST, dbl=True, want_scores=True)
        return i, layout, cloud, words, sc

    with cf.ThreadPoolExecutor(8) as pool:
        for i, layout, cloud, words, sc in pool.map(oracle, sorted(sampled)):
            occ = layout >= 0  # packed grid bit-exact: occupancy and the voxels' mean colours
            exp = np.zeros_like(words)
            exp[occ] = (1 << 24) | cloud[layout[occ], 3].view(np.uint32)
            assert np.array_equal(words, exp), "frame %d grid" % i
            _check_det(got[i], sc.reshape(1, -1), (P2, P2, P2), "frame %d" % i)
    assert (got[:, 0, 0].view(np.float64) > 0).all()


def test_pipeline_offset_subdivisions_vs_oracle(ctx, prod):
    """The tick with an offset and another subdivision size (S = 7 from (1, 2, 3)): the
    occupancy stream's closed-form (y, z) subdivisions and per-lane subdivision pairs, the
    pooled chunk tails and the dense memsets of a not-fully-covered grid, every frame's
    detections against the float64 oracle on its grid."""
    import torch
    s7, off = 7, (1, 2, 3)
    ngrid = 8
    axis_t, var, axis_q = synth.random_bases(F, D, M, R, seed=synth.BASE_SEED)
    ap = synth.whiten(axis_t, var)

    def oracle(i):
        g, layout, cloud = po.grid_inputs(prod["grids"][i], (G,) * 3, LEAF)
        fe, sb, _ = po.c3hlac(g, layout, cloud, F, THR, LEAF, s7, off, exact=True)
        ex = po.exist(fe)
        _, _, sc = po.search(sb, fe, ex, ap, axis_q, BOX, 1, EXIST, dbl=True, want_scores=True)
        return sb, sc

    with cf.ThreadPoolExecutor(8) as pool:
        ref = list(pool.map(oracle, range(ngrid)))
    ctx.search_setup(axis_t, var, axis_q)  # (other tests of the module set other axes)
    ctx.set_rank(1)
    nfr = 40  # two full batches of 16 and a ragged one
    ptrs = np.array([prod["d_grids"][i % ngrid].data_ptr() for i in range(nfr)], np.uint64)
    d_out = torch.zeros((nfr, M * 3), dtype=torch.int64, device="cuda:0")
    torch.cuda.synchronize()
    ctx.set_batch(16)
    ctx.set_pipeline(True)
    ctx.run_frames(ptrs, (G,) * 3, (0, 0, 0), LEAF, F, THR, s7, BOX, EXIST, True, d_out.data_ptr(), offset=off)
    ctx.synchronize()
    got = d_out.cpu().numpy().reshape(nfr, M, 3)
    for i in range(nfr):
        sb, sc = ref[i % ngrid]
        shape = tuple(int(n) - b + 1 for n, b in zip(sb[::-1], BOX))  # (z, y, x) positions
        _check_det(got[i], sc.reshape(M, -1), shape, "frame %d" % i)
    ctx.set_batch(32)


def test_score_layout_across_pipelined_and_single_searches(ctx, prod):
    """The sparse -1 fill of the score arrays (a position is rewritten only where the last
    search of the same layout had not gated it out) across single-frame searches and
    pipelined batches of one frame on the same context, whose score arrays share that
    layout (the layout is recorded once a search's gate is enqueued, not at
    capture).  After every single search the whole score array equals the float64
    oracle's: -1 exactly where the oracle gates the position out."""
    import torch
    d_out = torch.zeros((4, M * 3), dtype=torch.int64, device="cuda:0")
    ctx.set_batch(1)
    ctx.set_pipeline(True)
    for k, (single, batch) in enumerate([(3, 11), (11, 3), (5, 5), (17, 29)]):
        g = prod["d_grids"][single]
        ctx.set_grid(g, (G,) * 3, leaf=LEAF)
        ctx.extract(F, THR, S)
        ctx.search(BOX, EXIST, rotate=True)
        sc = ctx.scores()
        ref = prod["ref"][single][2]
        assert np.array_equal(sc < 0, ref < 0), k
        ok = ref > 0
        np.testing.assert_allclose(sc[ok], ref[ok], rtol=RTOL)
        ptrs = np.array([prod["d_grids"][batch].data_ptr()], np.uint64)
        ctx.run_frames(ptrs, (G,) * 3, (0, 0, 0), LEAF, F, THR, S, BOX, EXIST, True, d_out[k].data_ptr())
        ctx.synchronize()
        _check_det(d_out[k].cpu().numpy().reshape(M, 3), prod["ref"][batch][2].reshape(M, -1), (P1, P1, P1),
                   "batch %d" % k)
        sc = ctx.scores()  # the context holds the batch's frame
        ref = prod["ref"][batch][2]
        assert np.array_equal(sc < 0, ref < 0), ("batch", k)
