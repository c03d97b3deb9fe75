"""Multi-process path on CPU (gloo, world_size 2): frames sharded round-robin, each rank
runs the detection pipeline on its frames, records gathered with one all_gather and
re-ordered by frame.  The per-frame pipeline here is the oracle (CPU); on the GPU box
bench.py runs the same sharding and gather with the HIP path over RCCL."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import ROOT, THR

import sys
sys.path[:0] = [str(ROOT / "mapping-private_amd"), str(ROOT / "oracle")]

N_FRAMES, G, S, BOX = 5, 24, 8, (2, 2, 1)


def _frame_records(f):
    """Oracle detections of frame f: M x rank records as int64 words (score bits, x|y, z|mode)."""
    import pyoracle as po
    from c3hlac import synth
    pts = synth.kinect_scene(20_000, grid=G, leaf=0.01, seed=synth.BASE_SEED + 100 + f)
    g, layout, cloud = po.voxelize(pts, 0.01)
    feat, sb, _ = po.c3hlac(g, layout, cloud, 117, THR, 0.01, S)
    ex = po.exist(feat)
    axis_t, var, axis_q = synth.random_bases(117, 12, 3, 4, seed=7)
    L, _, _ = po.search(sb, feat, ex, synth.whiten(axis_t, var), axis_q, BOX, 1, 10)
    rec = np.zeros((3, 3), np.int64)
    for m in range(3):
        rec[m, 0] = np.float64(L.score[m]).view(np.int64)
        rec[m, 1] = (np.int64(L.x[m]) & 0xFFFFFFFF) | (np.int64(L.y[m]) << 32)
        rec[m, 2] = (np.int64(L.z[m]) & 0xFFFFFFFF) | (np.int64(L.mode[m]) << 32)
    return rec.reshape(-1)


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from c3hlac.dist import frame_shard, gather_records
    mine = frame_shard(N_FRAMES, rank, world)
    local = torch.from_numpy(np.stack([_frame_records(f) for f in mine]))
    out = gather_records(local, N_FRAMES, rank, world, dist)
    q.put((rank, mine, out.numpy()))
    dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_frame_shard_partition():
    from c3hlac.dist import frame_shard
    for n in (1, 5, 8, 513):
        for w in (1, 2, 3, 8):
            got = sorted(f for r in range(w) for f in frame_shard(n, r, w))
            assert got == list(range(n))


def test_gloo_two_ranks_gather_matches_single_process():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    ref = np.stack([_frame_records(f) for f in range(N_FRAMES)])
    shards = {}
    for rank, mine, out in res:
        shards[rank] = mine
        np.testing.assert_array_equal(out, ref)  # every rank holds all frames in order
    assert sorted(shards[0] + shards[1]) == list(range(N_FRAMES))
    assert any(np.frombuffer(ref[:, 0].tobytes(), np.float64) > 0)


# ---------------------------------------------------------------- one scene in z-slabs
SLAB_G, SLAB_S = 40, 8


def _oracle_records(words, ranges, offset=(0, 0, 0), z0=0):
    """Rank-1 records of the float64 oracle on words[z, y, x] (c3h_det layout, global z)."""
    import np_ref as npr
    import pyoracle as po
    from c3hlac import synth
    from c3hlac._capi import DET_DTYPE
    feat, ex, sb = npr.c3hlac(words, 117, THR, SLAB_S, offset)
    axis_t, var, axis_q = synth.random_bases(117, 12, 3, 4, seed=7)
    L, _, _ = po.search(sb, feat, ex, synth.whiten(axis_t, var), axis_q, ranges, 1, 10, dbl=True)
    rec = np.zeros(3, DET_DTYPE)
    for m in range(3):
        rec[m] = (L.score[m], L.x[m], L.y[m], L.z[m] + (z0 if L.score[m] > 0 else 0), L.mode[m])
    return rec


def _sparse_words():
    rng = np.random.default_rng(33)
    w = rng.integers(0, 1 << 24, size=(SLAB_G,) * 3, dtype=np.uint32) | np.uint32(1 << 24)
    w[rng.random(w.shape) > 0.08] = 0
    return w


def _slab_worker(rank, world, port, ranges, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from c3hlac.dist import gather_slab_lists, mode_ranges, mode_schedule, slab_extent
    words = _sparse_words()
    zr_max = max(mode_ranges(md, ranges)[2] for md in mode_schedule(ranges))
    ext = slab_extent(SLAB_G, SLAB_S, zr_max, rank, world)
    local = None
    if ext is not None:
        p0, p1, vz0, vz1, zoff = ext
        local = _oracle_records(words[vz0:vz1], ranges, (0, 0, zoff), p0)
    out = gather_slab_lists(local, 3, mode_schedule(ranges), dist)
    q.put((rank, out.tobytes()))
    dist.destroy_process_group()


@pytest.mark.parametrize("ranges", [(2, 2, 2), (1, 2, 3)])
def test_gloo_two_ranks_scene_slabs_match_whole_scene(ranges):
    from c3hlac._capi import DET_DTYPE
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_slab_worker, args=(r, 2, port, ranges, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    ref = _oracle_records(_sparse_words(), ranges)
    assert (ref["score"] > 0).all()
    for rank, raw in res:
        got = np.frombuffer(raw, DET_DTYPE)
        for f in ("x", "y", "z", "mode"):
            np.testing.assert_array_equal(got[f], ref[f])
        np.testing.assert_allclose(got["score"], ref["score"], rtol=1e-12)


def test_slab_partition():
    from c3hlac.dist import slab_extent, slab_planes
    assert [b - a for a, b in slab_planes(52, 8)] == [7, 7, 7, 7, 6, 6, 6, 6]
    for n in (1, 5, 52):
        for w in (1, 2, 3, 8):
            sp = slab_planes(n, w)
            assert sp[0][0] == 0 and sp[-1][1] == n and all(sp[i][1] == sp[i + 1][0] for i in range(w - 1))
    # halo plane below every slab but the first, zr_max - 1 planes after, clipped to the grid
    assert slab_extent(512, 10, 2, 0, 8) == (0, 7, 0, 80, 0)
    assert slab_extent(512, 10, 2, 1, 8) == (7, 14, 69, 150, 1)
    assert slab_extent(512, 10, 2, 7, 8) == (46, 52, 459, 512, 1)


def test_slab_search_rejects_rank_above_one():
    """rank > 1 lists cannot be merged from per-slab lists (the checkOverlap update is
    sequential over the whole scene): slab_search fails with C3H_ERR_ARG before touching a
    context; rank > 1 goes through slab_scores + merge_slab_scores (below)."""
    from c3hlac import dist as cdist
    from c3hlac._capi import C3HError
    words = np.zeros((20, 20, 20), np.uint32)
    with pytest.raises(C3HError, match="C3H_ERR_ARG"):
        cdist.slab_search(None, words, 117, THR, 10, (2, 2, 2), 0, 0, 2, search_rank=3)


def _oracle_scene(words, ranges, rank, offset=(0, 0, 0)):
    """float64 oracle: (subdivisions, score arrays, rank-`rank` lists) of words[z, y, x]."""
    import np_ref as npr
    import pyoracle as po
    from c3hlac import synth
    from c3hlac._capi import DET_DTYPE
    feat, ex, sb = npr.c3hlac(words, 117, THR, SLAB_S, offset)
    axis_t, var, axis_q = synth.random_bases(117, 12, 3, 4, seed=7)
    L, _, sc = po.search(sb, feat, ex, synth.whiten(axis_t, var), axis_q, ranges, rank, 10, dbl=True,
                         want_scores=True)
    rec = np.zeros((3, rank), DET_DTYPE)
    for m in range(3):
        for i in range(rank):
            k = m * rank + i
            rec[m, i] = (L.score[k], L.x[k], L.y[k], L.z[k], L.mode[k])
    return sb, sc, rec


def _slab_scores_worker(rank, world, port, ranges, srank, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from c3hlac.dist import gather_slab_scores, mode_ranges, mode_schedule, owned_blocks, slab_extent
    words = _sparse_words()
    zr_max = max(mode_ranges(md, ranges)[2] for md in mode_schedule(ranges))
    ext = slab_extent(SLAB_G, SLAB_S, zr_max, rank, world)
    local = None
    if ext is not None:
        p0, p1, vz0, vz1, zoff = ext
        sbl, sc, _ = _oracle_scene(words[vz0:vz1], ranges, 1, (0, 0, zoff))
        local = owned_blocks(sc, sbl, p0, p1, (SLAB_G,) * 3, SLAB_S, ranges, 3)
    out = gather_slab_scores(local, (SLAB_G,) * 3, SLAB_S, ranges, 3, srank, dist)
    q.put((rank, out.tobytes()))
    dist.destroy_process_group()


@pytest.mark.parametrize("ranges,srank", [((2, 2, 2), 3), ((1, 2, 3), 4)])
def test_gloo_two_ranks_scene_slabs_rank_above_one(ranges, srank):
    """rank 3 / 4 over two z-slabs (gloo, world size 2): every rank's owned position scores
    are gathered and the sequential update replayed over the whole scene; the lists equal
    the whole-scene float64 oracle's (search.cpp:327-356, 464-474)."""
    from c3hlac._capi import DET_DTYPE
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_slab_scores_worker, args=(r, 2, port, ranges, srank, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    _, _, ref = _oracle_scene(_sparse_words(), ranges, srank)
    assert (ref["score"] > 0).sum() >= 2 * 3  # several entries per list: the update is exercised
    for rank, raw in res:
        got = np.frombuffer(raw, DET_DTYPE).reshape(3, srank)
        for f in ("x", "y", "z", "mode"):
            np.testing.assert_array_equal(got[f], ref[f])
        np.testing.assert_allclose(got["score"], ref["score"], rtol=1e-12)


@pytest.mark.parametrize("ranges", [(2, 2, 2), (1, 2, 3), (3, 1, 1)])
@pytest.mark.parametrize("world", [2, 3, 5])
def test_merge_slab_scores_equals_whole_scene_replay(ranges, world):
    """In one process: the slabs' owned blocks reassemble the whole scene's score arrays
    position for position, and c3h_replay_scores over them gives the oracle's rank-4 lists."""
    from c3hlac.dist import merge_slab_scores, mode_ranges, mode_schedule, owned_blocks, slab_extent
    words = _sparse_words()
    sbw, scw, ref = _oracle_scene(words, ranges, 4)
    zr_max = max(mode_ranges(md, ranges)[2] for md in mode_schedule(ranges))
    parts = []
    for r in range(world):
        ext = slab_extent(SLAB_G, SLAB_S, zr_max, r, world)
        if ext is None:
            continue
        p0, p1, vz0, vz1, zoff = ext
        sbl, sc, _ = _oracle_scene(words[vz0:vz1], ranges, 1, (0, 0, zoff))
        parts.append(owned_blocks(sc, sbl, p0, p1, (SLAB_G,) * 3, SLAB_S, ranges, 3))
    scores, lists = merge_slab_scores(parts, (SLAB_G,) * 3, SLAB_S, ranges, 4)
    np.testing.assert_allclose(scores, scw, rtol=1e-12)
    assert np.array_equal(scores < 0, scw < 0)
    for f in ("x", "y", "z", "mode"):
        np.testing.assert_array_equal(lists[f], ref[f])
    np.testing.assert_allclose(lists["score"], ref["score"], rtol=1e-12)


def _random_scene_parts(rng, grid, subdiv, ranges, M, world, rotate=True):
    """Whole-scene score arrays of a random scene (smooth field + noise, gated holes, a few
    sharp peaks next to slab boundaries: a peak of one slab suppresses the other slab's top
    positions through checkOverlap, so low positions of that slab enter the lists) and every
    rank's owned blocks of them."""
    from c3hlac.dist import _mode_geoms, mode_ranges, mode_schedule, owned_blocks, scene_subdivisions, slab_extent
    sbg = scene_subdivisions(grid, subdiv)
    full = []
    for _, xe, ye, ze in _mode_geoms(sbg, ranges, rotate):
        z, y, x = np.meshgrid(np.arange(ze), np.arange(ye), np.arange(xe), indexing="ij")
        a = []
        for m in range(M):
            f = 0.3 + 0.1 * np.sin(x * rng.random() + y * rng.random() + z * rng.random())
            f = f + 0.01 * rng.random(f.shape)
            f[rng.random(f.shape) < 0.2] = -1.0
            for _ in range(3):  # peaks
                f[rng.integers(ze), rng.integers(ye), rng.integers(xe)] = 0.6 + 0.1 * rng.random()
            a.append(f)
        full.append(np.stack(a).reshape(-1))
    scores = np.concatenate(full)
    zr_max = max(mode_ranges(md, ranges)[2] for md in mode_schedule(ranges, rotate))
    locals_ = []
    for r in range(world):
        ext = slab_extent(grid[2], subdiv, zr_max, r, world)
        if ext is None:
            locals_.append(None)
            continue
        p0, p1 = ext[0], ext[1]
        blocks, o = [], 0
        for _, xe, ye, ze in _mode_geoms(sbg, ranges, rotate):
            blk = scores[o:o + M * ze * ye * xe].reshape(M, ze, ye, xe)
            blocks.append(np.ascontiguousarray(blk[:, p0:max(p0, min(p1, ze))]))
            o += M * ze * ye * xe
        locals_.append((p0, blocks))
    return sbg, scores, locals_


@pytest.mark.parametrize("seed", range(12))
def test_candidate_merge_equals_dense_replay(seed):
    """The z-slab candidate merge: slabs send only positions above
    their own local rank-th score plus per-row bounds of the rest, unresolved rows are
    fetched whole; the lists equal the dense replay over every score (c3h_replay_scores),
    on random scenes with peaks that make low positions enter across slab boundaries."""
    from c3hlac import replay_scores
    from c3hlac._capi import DET_DTYPE
    from c3hlac.dist import merge_slab_candidates
    rng = np.random.default_rng(seed)
    ranges = [(2, 2, 2), (1, 2, 3), (3, 1, 1), (2, 3, 2)][seed % 4]
    world = [2, 3, 5, 8][seed % 4]
    M, srank = 3, [2, 4, 6][seed % 3]
    grid = (70, 60, 90)
    sbg, scores, locals_ = _random_scene_parts(rng, grid, 5, ranges, M, world)
    ref = replay_scores(scores, sbg, ranges, np.zeros((M, srank), DET_DTYPE))
    got, st = merge_slab_candidates(locals_, grid, 5, ranges, M, srank)
    assert np.array_equal(got, ref)
    dense = scores.size * 8
    assert sum(st["bytes_per_rank"]) < dense  # less than every score once


def test_candidate_merge_needs_row_rounds():
    """A scene built so the first guess fails: slab 1's own top positions all overlap a peak
    of slab 0 reaching into its planes, so its (unsent) low positions enter the lists; the
    row bounds expose them and the rows are fetched."""
    from c3hlac import replay_scores
    from c3hlac._capi import DET_DTYPE
    from c3hlac.dist import merge_slab_candidates, _mode_geoms, scene_subdivisions
    ranges, M, srank, world, grid, S = (2, 2, 2), 1, 3, 2, (40, 40, 40), 5
    sbg = scene_subdivisions(grid, S)
    (_, xe, ye, ze), = _mode_geoms(sbg, ranges, False)
    a = np.full((ze, ye, xe), 0.05)  # a[z, y, x]
    a[3, 3, 3] = 0.99            # slab 0 (planes 0..3): a peak in its last plane
    # slab 1's four best positions, mutually apart (checkOverlap: more than the box range
    # in x or y) but each overlapping the peak's box: its local lists hold three of them
    # (local rank-3 score 0.9), the whole scene's drops them all
    a[4, 1, 1] = a[4, 1, 4] = a[4, 4, 1] = a[4, 4, 4] = 0.9
    a[6, 6, 6] = 0.2             # below slab 1's local rank-th score, yet enters the lists
    scores = a.reshape(-1).copy()
    locals_ = [(0, [a[None, 0:4].copy()]), (4, [a[None, 4:7].copy()])]
    ref = replay_scores(scores, sbg, ranges, np.zeros((M, srank), DET_DTYPE), rotate=False)
    got, st = merge_slab_candidates(locals_, grid, S, ranges, M, srank, rotate=False)
    assert np.array_equal(got, ref)
    assert st["row_rounds"] >= 1
    assert any(int(e["z"]) == 6 for e in ref[0])  # the low position is in the lists


def _cand_worker(rank, world, port, seed, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from c3hlac.dist import gather_slab_scores
    rng = np.random.default_rng(seed)
    sbg, scores, locals_ = _random_scene_parts(rng, (70, 60, 90), 5, (1, 2, 3), 3, world)
    st = {}
    out = gather_slab_scores(locals_[rank], (70, 60, 90), 5, (1, 2, 3), 3, 4, dist, stats=st)
    q.put((rank, out.tobytes(), st["row_rounds"]))
    dist.destroy_process_group()


def test_gloo_candidate_merge_world_three():
    """The candidate merge over gloo at world size 3 (size exchange, candidates, row
    rounds): every rank's lists equal the dense replay."""
    from c3hlac import replay_scores
    from c3hlac._capi import DET_DTYPE
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_cand_worker, args=(r, 3, port, 5, q)) for r in range(3)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    sbg, scores, _ = _random_scene_parts(np.random.default_rng(5), (70, 60, 90), 5, (1, 2, 3), 3, 3)
    ref = replay_scores(scores, sbg, (1, 2, 3), np.zeros((3, 4), DET_DTYPE))
    for rank, raw, _ in res:
        assert np.array_equal(np.frombuffer(raw, DET_DTYPE).reshape(3, 4), ref)


def test_slab_scores_restores_rank_on_error():
    """slab_scores sets the context's rank to 1 for its search and gives the
    caller's rank back when the search raises, too."""
    from c3hlac import dist as cd

    class Ctx:
        rank, M = 4, 1
        ranks = []

        def set_grid(self, *a):
            pass

        def extract(self, *a):
            return (6, 6, 6), 216

        def set_rank(self, r):
            self.rank = r
            self.ranks.append(r)

        def search(self, *a, **k):
            raise RuntimeError("search failed")

    c = Ctx()
    words = np.zeros((64, 64, 64), np.uint32)
    with pytest.raises(RuntimeError):
        cd.slab_scores(c, words, 117, THR, 10, (2, 2, 2), 100, 0, 2)
    assert c.rank == 4 and c.ranks == [1, 4]
