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

    search_rank (SearchObj::setRank) must be 1: the rank > 1 update with checkOverlap
    (search.cpp:327-356, 464-474) is sequential over the whole scene's scan order, so
    per-slab lists cannot be merged into it; C3HError(C3H_ERR_ARG) otherwise.

    The slab is loaded from packed grid words (c3h_set_grid), so voxels are placed by their
    cell index.  A scene voxelised from points whose centroids round across a cell boundary
    (c3h_voxelize's off-cell records, c3_hlac.cpp:349-377) is matched only by a whole-scene
    extract of the same words, not of the points."""
    import numpy as np
    from ._capi import C3HError, DET_DTYPE, ERRORS
    if int(search_rank) != 1:
        raise C3HError("slab_search: search_rank %d: %s (only rank 1 merges across slabs)"
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
