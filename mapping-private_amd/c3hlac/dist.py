"""Frame sharding over ranks and the detection gather.

Frames are independent, so rank r of W processes frames r, r+W, r+2W, ... with no
data-path collective.  After a batch, every rank's M x rank detection records (c3h_det:
double score + 4 int32, viewed as 3 int64 words) are gathered with a single all_gather
(RCCL on the GPU, gloo in the CPU tests) and re-ordered by frame index.
"""
import torch


def frame_shard(n_frames, rank, world):
    """Frame indices owned by `rank` (round-robin)."""
    return list(range(rank, n_frames, world))


def gather_records(local, n_frames, rank, world, dist):
    """local: (len(frame_shard(...)), K) int64 tensor of this rank's records, in shard
    order.  Returns the (n_frames, K) tensor of all frames in frame order (every rank)."""
    per = (n_frames + world - 1) // world
    K = local.shape[1]
    buf = torch.zeros((per, K), dtype=local.dtype, device=local.device)
    buf[: local.shape[0]] = local
    parts = [torch.empty_like(buf) for _ in range(world)]
    dist.all_gather(parts, buf)
    out = torch.empty((n_frames, K), dtype=local.dtype, device=local.device)
    for r in range(world):
        idx = frame_shard(n_frames, r, world)
        out[idx] = parts[r][: len(idx)]
    return out


# ---------------------------------------------------------------- one scene over ranks
# A single huge scene (BASELINE config 5 across GPUs) is split into z-slabs of
# whole subdivision planes (52 planes over 8 ranks: 7,7,7,7,6,6,6,6).  The C3 stencil reaches
# one voxel plane down (dz = -1 only, c3_hlac.cpp:183-201), so a slab's sub-grid carries one
# halo voxel plane below its first subdivision plane -- extracted with a z offset of 1, which
# makes those voxels neighbours but not centres (c3_hlac.cpp:349-354).  Boxes that start in
# the slab reach zr_max - 1 planes into the next one: the slab recomputes those planes'
# features itself (integer-exact, so bit-identical to the owner's) instead of receiving
# them.  The search sums boxes directly (no summed-volume table), so no prefix of per-slab
# totals is exchanged either: the only collective is the final gather of the M rank-1
# records, merged by (score desc, scan order asc) -- the reference's strict '>' over
# (mode, z, y, x) (search.cpp:431-480).

def mode_schedule(ranges, rotate=True):
    """SearchObj::search's mode order (search.cpp:384-417): ids 0..5 = S_MODE_1..6."""
    r1, r2, r3 = ranges
    if not rotate:
        return [0]
    if r1 == r2:
        return [0] if r2 == r3 else [0, 1, 4]
    if r2 == r3:
        return [0, 4, 5]
    if r1 == r3:
        return [0, 4, 2]
    return [0, 1, 2, 3, 4, 5]


def mode_ranges(mode, ranges):
    """(xr, yr, zr) of a mode (search.cpp:218-317)."""
    r1, r2, r3 = ranges
    return {0: (r1, r2, r3), 1: (r1, r3, r2), 2: (r2, r1, r3), 3: (r2, r3, r1), 4: (r3, r1, r2),
            5: (r3, r2, r1)}[mode]


def slab_planes(n_planes, world):
    """Subdivision planes [start, stop) of every rank, sizes differing by at most one."""
    base, extra = divmod(n_planes, world)
    out, s = [], 0
    for r in range(world):
        n = base + (1 if r < extra else 0)
        out.append((s, s + n))
        s += n
    return out


def slab_extent(gz, subdiv, zr_max, rank, world):
    """(p0, p1, vz0, vz1, zoff) of `rank`: its subdivision planes [p0, p1), its sub-grid's
    voxel planes [vz0, vz1) (halo below, zr_max - 1 planes after), the extract's z offset;
    None when the rank owns no plane."""
    n_planes = -(-gz // subdiv)
    p0, p1 = slab_planes(n_planes, world)[rank]
    if p0 == p1:
        return None
    vz0 = max(p0 * subdiv - 1, 0)
    vz1 = min((p1 + zr_max - 1) * subdiv, gz)
    return p0, p1, vz0, vz1, p0 * subdiv - vz0


def merge_slab_lists(parts, schedule):
    """parts: per rank (M,) c3h_det records with GLOBAL z (score <= 0: nothing found).
    Per model the highest score; ties go to the earliest (mode, z, y, x) in scan order."""
    import numpy as np

    def key(e):
        return (schedule.index(int(e["mode"])), int(e["z"]), int(e["y"]), int(e["x"]))

    out = parts[0].copy()
    for m in range(out.shape[0]):
        best = None
        for p in parts:
            e = p[m]
            if float(e["score"]) <= 0.0:
                continue
            if best is None or float(e["score"]) > float(best["score"]) or (
                    float(e["score"]) == float(best["score"]) and key(e) < key(best)):
                best = e
        if best is not None:
            out[m] = best
        else:
            out[m]["score"] = 0.0
    return np.ascontiguousarray(out)


def slab_search(ctx, words_zyx, variant, thr, subdiv, ranges, exist_threshold, rank, world, rotate=True,
                search_rank=1):
    """Extract + rank-1 search of rank `rank`'s slab of the packed grid words_zyx[z, y, x]
    (only the slab's planes are read) on this rank's context, whose search bases (and
    engine settings) are already set.  Returns (M,) c3h_det records with global z, or None
    when the slab owns no plane.

    search_rank (SearchObj::setRank) must be 1 here: the rank > 1 update with checkOverlap
    (search.cpp:327-356, 464-474) is sequential over the whole scene's scan order, so
    per-slab lists cannot be merged into it (C3HError(C3H_ERR_ARG) otherwise); rank > 1
    goes through slab_scores + merge_slab_scores, which replay it over the whole scene.

    The slab is loaded from packed grid words (c3h_set_grid), so voxels are placed by their
    cell index.  A scene voxelised from points whose centroids round across a cell boundary
    (c3h_voxelize's off-cell records, c3_hlac.cpp:349-377) is matched only by a whole-scene
    extract of the same words, not of the points."""
    import numpy as np
    from ._capi import C3HError, DET_DTYPE, ERRORS
    if int(search_rank) != 1:
        raise C3HError("slab_search: search_rank %d: %s (rank > 1: slab_scores + merge_slab_scores)"
                       % (search_rank, ERRORS.get(-1, -1)))
    gz, gy, gx = words_zyx.shape
    zr_max = max(mode_ranges(md, ranges)[2] for md in mode_schedule(ranges, rotate))
    ext = slab_extent(gz, subdiv, zr_max, rank, world)
    if ext is None:
        return None
    p0, p1, vz0, vz1, zoff = ext
    ctx.set_grid(np.ascontiguousarray(words_zyx[vz0:vz1]).reshape(-1), (gx, gy, vz1 - vz0))
    ctx.extract(variant, thr, subdiv, (0, 0, zoff))
    ctx.set_rank(1)
    lists, _ = ctx.search(ranges, exist_threshold, rotate=rotate)
    out = np.ascontiguousarray(lists[:, 0], dtype=DET_DTYPE)
    for m in range(out.shape[0]):
        if float(out[m]["score"]) > 0.0:
            out[m]["z"] = int(out[m]["z"]) + p0
    return out


def gather_slab_lists(local, M, schedule, dist, device="cpu"):
    """All-gather every rank's (M,) records (None: no plane) and merge them (every rank)."""
    import numpy as np
    from ._capi import DET_DTYPE
    if local is None:
        local = np.zeros(M, DET_DTYPE)
    buf = torch.from_numpy(np.ascontiguousarray(local).view(np.int64).reshape(M, -1).copy()).to(device)
    parts = [torch.empty_like(buf) for _ in range(dist.get_world_size())]
    dist.all_gather(parts, buf)
    return merge_slab_lists([p.cpu().numpy().reshape(-1).view(DET_DTYPE) for p in parts], schedule)


# ---------------------------------------------------------------- rank > 1 over slabs
# The rank > 1 lists depend on the whole scene's scan order: a candidate enters only above
# the list's current rank-th score, and checkOverlap compares it with every entry ranked
# before it, wherever in the scene that entry came from (search.cpp:327-356, 464-474).  So
# per-slab lists cannot be merged; instead every rank sends the scores of the box positions
# it owns (origins in its subdivision planes [p0, p1); its sub-grid's extra planes only
# complete boxes that start inside the slab), and the sequential update is replayed over
# the assembled whole-scene score arrays (c3h_replay_scores, host).  Scores of a position
# are bit-identical on the slab and on the whole scene (integer-exact features, the same
# box-sum order), so the lists are the whole-scene search's.

def scene_subdivisions(grid_xyz, subdiv):
    """setVoxelFilter's getSubdivNum without offsets (c3_hlac.cpp:210-225, float arithmetic)."""
    import numpy as np
    inv = np.float32(1.0 / subdiv)
    return tuple(int(np.ceil(np.float32(g) * inv)) for g in grid_xyz)


def _mode_geoms(sb, ranges, rotate):
    """(mode, xe, ye, ze) of every scheduled mode with a position (the score layout's order)."""
    out = []
    for md in mode_schedule(ranges, rotate):
        xr, yr, zr = mode_ranges(md, ranges)
        xe, ye, ze = sb[0] - xr + 1, sb[1] - yr + 1, sb[2] - zr + 1
        if xe > 0 and ye > 0 and ze > 0:
            out.append((md, xe, ye, ze))
    return out


def slab_scores(ctx, words_zyx, variant, thr, subdiv, ranges, exist_threshold, rank, world, rotate=True):
    """Extract + search of rank `rank`'s slab (as slab_search) -> (p0, blocks): per mode of
    the whole scene's schedule the (M, nz, ye, xe) float64 scores of the positions whose
    origin plane z is in [p0, min(p1, ze)), -1 where gated out; None when the slab owns no
    plane.  The slab's own lists are not used (rank 1 on the fast path); the context's
    rank is restored afterwards (set_rank: its lists start fresh)."""
    import numpy as np
    gz, gy, gx = words_zyx.shape
    zr_max = max(mode_ranges(md, ranges)[2] for md in mode_schedule(ranges, rotate))
    ext = slab_extent(gz, subdiv, zr_max, rank, world)
    if ext is None:
        return None
    p0, p1, vz0, vz1, zoff = ext
    ctx.set_grid(np.ascontiguousarray(words_zyx[vz0:vz1]).reshape(-1), (gx, gy, vz1 - vz0))
    sbl, _ = ctx.extract(variant, thr, subdiv, (0, 0, zoff))
    prev_rank = getattr(ctx, "rank", None)
    ctx.set_rank(1)  # the fast path: only the scores are used
    try:
        ctx.search(ranges, exist_threshold, rotate=rotate)
        out = owned_blocks(ctx.scores(), sbl, p0, p1, (gx, gy, gz), subdiv, ranges, max(ctx.M, 1), rotate)
    finally:  # restored on errors too
        if prev_rank is not None and prev_rank != 1:
            ctx.set_rank(prev_rank)  # the caller's setRank (fresh lists of that rank)
    return out


def owned_blocks(scores_local, sb_local, p0, p1, grid_xyz, subdiv, ranges, M, rotate=True):
    """A slab's score arrays (c3h_get_scores layout over its sub-grid's subdivisions
    sb_local, plane 0 = the scene's plane p0) -> (p0, per whole-scene mode the (M, nz, ye,
    xe) block of the positions with origin plane in [p0, min(p1, ze)))."""
    import numpy as np
    local, off, o = {}, {}, 0
    for md, xe, ye, ze in _mode_geoms(sb_local, ranges, rotate):
        local[md] = (xe, ye, ze)
        off[md] = o
        o += M * xe * ye * ze
    assert o == scores_local.size or (o == 0 and scores_local.size <= 1), (o, scores_local.size)
    blocks = []
    for md, xe, ye, ze in _mode_geoms(scene_subdivisions(grid_xyz, subdiv), ranges, rotate):
        nz = max(0, min(p1, ze) - p0)
        if nz == 0:
            blocks.append(np.zeros((M, 0, ye, xe)))
            continue
        lx, ly, lz = local[md]
        assert (lx, ly) == (xe, ye) and lz >= nz
        blk = scores_local[off[md]:off[md] + M * lx * ly * lz].reshape(M, lz, ly, lx)
        blocks.append(np.ascontiguousarray(blk[:, :nz], dtype=np.float64))
    return p0, blocks


def merge_slab_scores(parts, grid_xyz, subdiv, ranges, search_rank, rotate=True, lists=None):
    """parts: every rank's slab_scores result (None: no plane) -> (the whole scene's score
    arrays in c3h_get_scores' layout, its (M, search_rank) lists replayed from `lists`
    (default: setRank's state)).  Dense: every owned position's score (the reference for
    the candidate merge below, and its in-process form)."""
    import numpy as np
    from . import replay_scores
    from ._capi import DET_DTYPE
    parts = [p for p in parts if p is not None]
    sbg = scene_subdivisions(grid_xyz, subdiv)
    geoms = _mode_geoms(sbg, ranges, rotate)
    if not parts:  # no rank owns a plane (a scene thinner than one subdivision): nothing searched
        M = 0 if lists is None else lists.shape[0]
        return np.zeros(0), (np.zeros((M, int(search_rank)), DET_DTYPE) if lists is None else lists)
    M = parts[0][1][0].shape[0]
    full = []
    for i, (md, xe, ye, ze) in enumerate(geoms):
        a = np.full((M, ze, ye, xe), np.nan)
        for p0, blocks in parts:
            b = blocks[i]
            a[:, p0:p0 + b.shape[1]] = b
        assert not np.isnan(a).any(), "a position no slab owns"
        full.append(a.reshape(-1))
    scores = np.concatenate(full) if full else np.zeros(0)
    if lists is None:
        lists = np.zeros((M, int(search_rank)), DET_DTYPE)
    return scores, replay_scores(scores, sbg, ranges, lists, rotate=rotate)


# ---------------------------------------------------------------- candidate merge
# Sending every owned score costs M x P x 8 B per rank (10.6 MB over the ranks at 512^3,
# M = 10).  The rank update only ever acts on a position above the model's current rank-th
# score L (search.cpp:464-474: `dot > max_dot[i]` for some i <= rank - 1), and within one
# replay L never decreases: an update writes the new score at index i above the old
# max_dot[i] and shifts entries i..o-1 down over the removed (overlapping or last) entry o,
# so every max_dot[j] is non-decreasing.  Hence a replay over a subset S of the positions
# (the rest treated as gated out) equals the full replay if every unsent position scores
# at or below the S-replay's L at the start of its row (mode, m, z, y) -- its "floor": by
# induction over the scan order, up to such a row both replays hold the same lists, so the
# floor is the true one, and a position at or below it is a no-op in the full replay too.
#
# Protocol (every rank computes the same decisions, so the collectives' sizes are known):
# 1. each slab sends, per model, the positions scoring above its own slab-local replay's
#    rank-th score (a guess of L; any guess is safe), plus per owned row the max of the
#    scores it did not send (-1: none).  The slab owning plane 0 knows the true floors of
#    its rows in the first mode exactly (nothing precedes them in the scan): it sends only
#    the positions above those floors there, and its rows there are resolved at once;
# 2. everyone replays the candidates (c3h_replay_scores_floor) and lists the rows whose
#    unsent max exceeds the row's floor; each owner sends, per listed row, the positions it
#    has not sent that score above that floor, and the row's new unsent max; repeat until
#    no row is unresolved (every round sends at least one position per listed row).

def _geom_offsets(geoms, M):
    """per mode: offset of its M x ze x ye x xe scores, of its M x ze x ye rows."""
    so, ro, s, r = [], [], 0, 0
    for _, xe, ye, ze in geoms:
        so.append(s)
        ro.append(r)
        s += M * ze * ye * xe
        r += M * ze * ye
    return so, ro, s, r


class _SlabSender:
    """One rank's side of the candidate merge: its owned blocks and, per owned row, the
    score above which every position of the row has been sent."""

    def __init__(self, local, grid_xyz, subdiv, ranges, M, search_rank, rotate, lists0):
        import numpy as np
        from . import replay_scores
        self.local = local
        self.sbg = scene_subdivisions(grid_xyz, subdiv)
        self.geoms = _mode_geoms(self.sbg, ranges, rotate)
        self.so, self.ro, self.ns, self.nr = _geom_offsets(self.geoms, M)
        self.M = M
        if local is None:
            return
        p0, blocks = local
        full = np.full(self.ns, -1.0)
        for i, ((_, xe, ye, ze), b) in enumerate(zip(self.geoms, blocks)):
            full[self.so[i]:self.so[i] + M * ze * ye * xe].reshape(M, ze, ye, xe)[:, p0:p0 + b.shape[1]] = b
        guess = replay_scores(full, self.sbg, ranges, lists0.copy(), rotate=rotate)
        thr = guess["score"][:, -1].astype(np.float64)  # the slab-local rank-th score per model
        self.sent = [np.broadcast_to(thr[:, None, None], b.shape[:3]).copy() for b in blocks]
        if p0 == 0 and self.geoms and blocks[0].shape[1] > 0:
            # plane 0's slab, first mode: the exact floors (its rows open the scan)
            (_, xe, ye, ze) = self.geoms[0]
            first = np.full(self.ns, -1.0)
            first[:M * ze * ye * xe].reshape(M, ze, ye, xe)[:, :blocks[0].shape[1]] = blocks[0]
            _, fl = replay_scores(first, self.sbg, ranges, lists0.copy(), rotate=rotate, floors=True)
            self.sent[0] = fl[:M * ze * ye].reshape(M, ze, ye)[:, :blocks[0].shape[1]].copy()

    def phase1(self):
        """[n, flat score index x n, score x n, max unsent score per owned row (mode-major,
        M x nz x ye)]; [0] without planes."""
        import numpy as np
        if self.local is None:
            return np.zeros(1)
        p0, blocks = self.local
        idx, val, bounds = [], [], []
        for i, ((_, xe, ye, ze), b) in enumerate(zip(self.geoms, blocks)):
            send = b > self.sent[i][..., None]
            m_, z_, y_, x_ = np.nonzero(send)
            idx.append(self.so[i] + ((m_ * ze + p0 + z_) * ye + y_) * xe + x_)
            val.append(b[send])
            bounds.append(np.where(send | (b <= 0), -1.0, b).max(axis=3, initial=-1.0).reshape(-1))
        idx = np.concatenate(idx) if idx else np.zeros(0, np.int64)
        val = np.concatenate(val) if val else np.zeros(0)
        return np.concatenate([[float(len(idx))], idx.astype(np.float64), val] + bounds)

    def rows(self, rows, merge):
        """per requested row (canonical order): [n, new unsent max, x x n, score x n] of the
        positions above the row's floor not sent before; the row's sent threshold drops to
        its floor."""
        import numpy as np
        out = []
        if self.local is None or len(rows) == 0:
            return np.zeros(0)
        p0, blocks = self.local
        for row in rows:
            i, m, z, y, xe, ze, ye = merge.row_geom(int(row))
            r = blocks[i][m, z - p0, y]
            fl = merge.floor[row]
            prev = self.sent[i][m, z - p0, y]
            new = (r > fl) & (r <= prev)
            rest = r[(r <= fl) & (r > 0)]
            xs = np.flatnonzero(new)
            out.append(np.concatenate([[float(len(xs)), rest.max() if rest.size else -1.0], xs.astype(np.float64),
                                       r[xs]]))
            self.sent[i][m, z - p0, y] = min(prev, fl)
        return np.concatenate(out)


class _CandMerge:
    """The merge state every rank keeps (deterministic: the same on every rank)."""

    def __init__(self, payloads, grid_xyz, subdiv, ranges, M, search_rank, rotate, lists0):
        import numpy as np
        self.sbg = scene_subdivisions(grid_xyz, subdiv)
        self.geoms = _mode_geoms(self.sbg, ranges, rotate)
        self.so, self.ro, ns, nr = _geom_offsets(self.geoms, M)
        self.M, self.ranges, self.rotate = M, ranges, rotate
        self.world = len(payloads)
        zr_max = max(mode_ranges(md, ranges)[2] for md in mode_schedule(ranges, rotate))
        self.ext = [slab_extent(grid_xyz[2], subdiv, zr_max, r, self.world) for r in range(self.world)]
        self.scores = np.full(ns, -1.0)
        self.bound = np.full(nr, -1.0)
        self.owner = np.full(nr, -1, np.int64)
        self.floor = np.zeros(nr)
        self.lists0 = lists0
        for r, pl in enumerate(payloads):
            n = int(pl[0])
            if self.ext[r] is None:
                continue
            p0, p1 = self.ext[r][0], self.ext[r][1]
            self.scores[pl[1:1 + n].astype(np.int64)] = pl[1 + n:1 + 2 * n]
            o = 1 + 2 * n
            for i, (_, xe, ye, ze) in enumerate(self.geoms):
                nz = max(0, min(p1, ze) - p0)
                rows = self.bound[self.ro[i]:self.ro[i] + M * ze * ye].reshape(M, ze, ye)
                rows[:, p0:p0 + nz] = pl[o:o + M * nz * ye].reshape(M, nz, ye)
                self.owner[self.ro[i]:self.ro[i] + M * ze * ye].reshape(M, ze, ye)[:, p0:p0 + nz] = r
                o += M * nz * ye
        self.sent_bytes = [len(pl) * 8 for pl in payloads]
        self.rounds = 0

    def replay(self):
        """-> (lists, flat indices of the unresolved rows, ascending)."""
        import numpy as np
        from . import replay_scores
        lists, self.floor = replay_scores(self.scores, self.sbg, self.ranges, self.lists0.copy(), rotate=self.rotate,
                                          floors=True)
        return lists, np.flatnonzero(self.bound > self.floor)

    def row_geom(self, row):
        """flat row index -> (mode index, m, z, y, xe, ze, ye)"""
        import bisect
        i = bisect.bisect_right(self.ro, row) - 1
        _, xe, ye, ze = self.geoms[i]
        k = row - self.ro[i]
        return i, k // (ze * ye), (k // ye) % ze, k % ye, xe, ze, ye

    def request(self, rows, r):
        """rows of rank r among `rows` (canonical ascending order)"""
        return rows[self.owner[rows] == r]

    def fill(self, rows, payload):
        o = 0
        for row in rows:
            i, m, z, y, xe, ze, ye = self.row_geom(int(row))
            n = int(payload[o])
            self.bound[row] = payload[o + 1]
            xs = payload[o + 2:o + 2 + n].astype(int)
            a = self.so[i] + ((m * ze + z) * ye + y) * xe
            self.scores[a + xs] = payload[o + 2 + n:o + 2 + 2 * n]
            o += 2 + 2 * n


def _initial_lists(M, search_rank, lists):
    import numpy as np
    from ._capi import DET_DTYPE
    return np.zeros((M, int(search_rank)), DET_DTYPE) if lists is None else np.ascontiguousarray(lists, DET_DTYPE)


def merge_slab_candidates(locals_, grid_xyz, subdiv, ranges, M, search_rank, rotate=True, lists=None):
    """The candidate merge in one process (every rank's local blocks at hand): the same
    payloads and decisions as gather_slab_scores.  Returns (lists, stats); stats times each
    rank's sender side (its slab-local replay and phase-1 payload: in a distributed run the
    ranks do this concurrently, so the max is the critical path) and the merge (the
    candidates' replays and row rounds, done by every rank)."""
    import time
    lists0 = _initial_lists(M, search_rank, lists)
    senders, payloads, t_send = [], [], []
    for lc in locals_:
        t0 = time.perf_counter()
        sd = _SlabSender(lc, grid_xyz, subdiv, ranges, M, search_rank, rotate, lists0)
        payloads.append(sd.phase1())
        t_send.append(time.perf_counter() - t0)
        senders.append(sd)
    t0 = time.perf_counter()
    mg = _CandMerge(payloads, grid_xyz, subdiv, ranges, M, search_rank, rotate, lists0)
    while True:
        lists, rows = mg.replay()
        if len(rows) == 0:
            break
        mg.rounds += 1
        for r, sd in enumerate(senders):
            mine = mg.request(rows, r)
            pl = sd.rows(mine, mg)
            mg.sent_bytes[r] += pl.size * 8
            mg.fill(mine, pl)
    return lists, {"bytes_per_rank": mg.sent_bytes, "row_rounds": mg.rounds, "sender_s_max": max(t_send, default=0.0),
                   "merge_s": time.perf_counter() - t0}


def gather_slab_scores(local, grid_xyz, subdiv, ranges, M, search_rank, dist, rotate=True, device="cpu",
                       stats=None):
    """The whole scene's (M, search_rank) lists on every rank from every rank's slab_scores
    (None: no plane), by the candidate merge above: per round one all_gather of the payload
    sizes and one of the payloads (phase 1, then one round per pass over unresolved rows,
    usually none or one).  Host memory per rank: the scene's score arrays once (M x P x
    8 B) plus the payloads; `stats` (a dict) receives the bytes each rank sent and the rounds."""
    import numpy as np

    def all_gather_f64(arr):
        world = dist.get_world_size()
        n = torch.tensor([float(arr.size)], dtype=torch.float64, device=device)
        sizes = [torch.empty_like(n) for _ in range(world)]
        dist.all_gather(sizes, n)
        sizes = [int(x.item()) for x in sizes]
        buf = torch.zeros(max(max(sizes), 1), dtype=torch.float64, device=device)
        buf[:arr.size] = torch.from_numpy(np.ascontiguousarray(arr, np.float64)).to(device)
        got = [torch.empty_like(buf) for _ in range(world)]
        dist.all_gather(got, buf)
        return [g[:k].cpu().numpy() for g, k in zip(got, sizes)]

    me = dist.get_rank()
    lists0 = _initial_lists(M, search_rank, None)
    sender = _SlabSender(local, grid_xyz, subdiv, ranges, M, search_rank, rotate, lists0)
    mg = _CandMerge(all_gather_f64(sender.phase1()), grid_xyz, subdiv, ranges, M, search_rank, rotate, lists0)
    while True:
        lists, rows = mg.replay()
        if len(rows) == 0:
            break
        mg.rounds += 1
        parts = all_gather_f64(sender.rows(mg.request(rows, me), mg))
        for r, pl in enumerate(parts):
            mg.sent_bytes[r] += pl.size * 8
            mg.fill(mg.request(rows, r), pl)
    if stats is not None:
        stats.update(bytes_per_rank=mg.sent_bytes, row_rounds=mg.rounds)
    return lists
