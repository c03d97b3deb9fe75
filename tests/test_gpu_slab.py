"""One scene split into z-slabs of subdivision planes over ranks (BASELINE
config 5 across GPUs; c3hlac.dist.slab_search): every rank's slab runs through the C-ABI
on its own sub-grid (one halo voxel plane below, zr_max - 1 planes after), and the merged
rank-1 records must equal the whole-scene search bit-for-bit (score, x, y, z, mode).  The
ranks run one after another on this process's context (the GPU box has one GPU); the
gather itself is covered with gloo in test_dist.py."""
import numpy as np
import pytest

from c3hlac import synth
from c3hlac.dist import merge_slab_lists, mode_schedule, slab_search
from conftest import THR

pytestmark = pytest.mark.gpu


def _whole(ctx, words, variant, S, ranges, thr):
    gz, gy, gx = words.shape
    ctx.set_grid(np.ascontiguousarray(words).reshape(-1), (gx, gy, gz))
    ctx.extract(variant, THR, S)
    ctx.set_rank(1)
    lists, _ = ctx.search(ranges, thr)
    return np.ascontiguousarray(lists[:, 0])


def _split(ctx, words, variant, S, ranges, thr, world):
    parts = [slab_search(ctx, words, variant, THR, S, ranges, thr, r, world) for r in range(world)]
    return merge_slab_lists([p for p in parts if p is not None], mode_schedule(ranges))


@pytest.mark.parametrize("world", [2, 3, 8])
@pytest.mark.parametrize("ranges", [(2, 2, 2), (1, 2, 3), (3, 1, 1)])
def test_slabs_kinect_256(ctx, world, ranges):
    pts = synth.kinect_scene(1_000_000, grid=256, leaf=0.01, seed=synth.BASE_SEED + 11)
    gi = ctx.voxelize(pts, 0.01)
    d = gi.div_b
    words = ctx.grid().reshape(d[2], d[1], d[0])
    axis_t, var, axis_q = synth.random_bases(117, 100, 10, 20, seed=4)
    ctx.search_setup(axis_t, var, axis_q)
    whole = _whole(ctx, words, 117, 10, ranges, 100)
    assert (whole["score"] > 0).all()
    got = _split(ctx, words, 117, 10, ranges, 100, world)
    assert np.array_equal(got, whole)


def test_slabs_config5_dense_512_eight_ranks(ctx):
    """512^3 dense, C3-HLAC-981, 52 planes over 8 ranks (7,7,7,7,6,6,6,6): every interior
    position ties, so the merge's scan-order tie-break decides the records."""
    G, S, n = 512, 10, 52
    words = np.tile(synth.dense_words(S, seed=51), (n, n, n))[:G, :G, :G]
    axis_t, var, axis_q = synth.random_bases(981, 100, 10, 20, seed=52)
    ctx.search_setup(axis_t, var, axis_q)
    whole = _whole(ctx, words, 981, S, (2, 2, 2), 100)
    got = _split(ctx, words, 981, S, (2, 2, 2), 100, 8)
    assert np.array_equal(got, whole)


@pytest.mark.parametrize("srank", [3, 4])
@pytest.mark.parametrize("world", [2, 3, 8])
@pytest.mark.parametrize("ranges", [(2, 2, 2), (1, 2, 3)])
def test_slabs_rank_above_one_kinect_256(ctx, srank, world, ranges):
    """rank 3 / 4 (SearchObj::setRank) over z-slabs: every slab's owned position scores
    (slab_scores), reassembled and replayed with the sequential checkOverlap update on the
    host (merge_slab_scores -> c3h_replay_scores), equal the whole-scene search's lists
    (the GPU replay kernel) bit for bit, and the score arrays position for position."""
    from c3hlac.dist import merge_slab_scores, slab_scores
    pts = synth.kinect_scene(1_000_000, grid=256, leaf=0.01, seed=synth.BASE_SEED + 11)
    gi = ctx.voxelize(pts, 0.01)
    d = gi.div_b
    words = ctx.grid().reshape(d[2], d[1], d[0])
    axis_t, var, axis_q = synth.random_bases(117, 100, 10, 20, seed=4)
    ctx.search_setup(axis_t, var, axis_q)
    ctx.set_grid(np.ascontiguousarray(words).reshape(-1), (d[0], d[1], d[2]))
    ctx.extract(117, THR, 10)
    ctx.set_rank(srank)
    whole, _ = ctx.search(ranges, 100)
    whole_scores = ctx.scores()
    assert (whole["score"] > 0).all()
    parts = [slab_scores(ctx, words, 117, THR, 10, ranges, 100, r, world) for r in range(world)]
    scores, lists = merge_slab_scores(parts, (d[0], d[1], d[2]), 10, ranges, srank)
    assert np.array_equal(scores, whole_scores)
    assert np.array_equal(lists, np.ascontiguousarray(whole))
    # the candidate merge (what gather_slab_scores sends over the collective) gives the same
    from c3hlac.dist import merge_slab_candidates
    cand, st = merge_slab_candidates(parts, (d[0], d[1], d[2]), 10, ranges, 10, srank)
    assert np.array_equal(cand, np.ascontiguousarray(whole))
    assert sum(st["bytes_per_rank"]) < scores.size * 8


def test_slab_merge_rank4_dense_512_eight_slabs(ctx, record_property):
    """512^3 (random dense words: no ties), C3-HLAC-981, M = 10 x r = 20,
    rank 4, 8 slabs on this GPU one after another.  Dense merge (every owned score) and the
    candidate merge give the whole-scene search's lists bit for bit; the candidate payload
    and both merges' host times are recorded (json in the test's stdout)."""
    import json
    import time
    from c3hlac.dist import merge_slab_candidates, merge_slab_scores, slab_scores
    G, S, world, srank, ranges = 512, 10, 8, 4, (2, 2, 2)
    words = synth.random_words(G, 0.5, seed=61, colour_max=255).reshape(G, G, G)
    axis_t, var, axis_q = synth.random_bases(981, 100, 10, 20, seed=62)
    ctx.search_setup(axis_t, var, axis_q)
    ctx.set_grid(np.ascontiguousarray(words).reshape(-1), (G, G, G))
    ctx.extract(981, THR, S)
    ctx.set_rank(srank)
    whole, _ = ctx.search(ranges, 100)
    whole = np.ascontiguousarray(whole)
    assert (whole["score"] > 0).all()
    parts = [slab_scores(ctx, words, 981, THR, S, ranges, 100, r, world) for r in range(world)]
    t0 = time.perf_counter()
    scores, dense_lists = merge_slab_scores(parts, (G, G, G), S, ranges, srank)
    t1 = time.perf_counter()
    cand, st = merge_slab_candidates(parts, (G, G, G), S, ranges, 10, srank)
    t2 = time.perf_counter()
    assert np.array_equal(dense_lists, whole)
    assert np.array_equal(cand, whole)
    rec = {"dense_bytes_per_rank_max": max(sum(b.size for b in p[1]) * 8 for p in parts),
           "candidate_bytes_per_rank": st["bytes_per_rank"], "row_rounds": st["row_rounds"],
           "dense_merge_s": t1 - t0, "candidate_merge_s": t2 - t1,
           "candidate_sender_s_max_rank": st["sender_s_max"], "candidate_merge_only_s": st["merge_s"]}
    print("slab_merge_512:", json.dumps(rec))
    record_property("slab_merge_512", rec)
    assert max(st["bytes_per_rank"]) * 4 < rec["dense_bytes_per_rank_max"]
