"""Deterministic synthetic inputs for the C3-HLAC path.

There is no network and no dataset here: scenes are generated, seeded by
splitmix64 (base seed 0xC3A1AC + frame index).

kinect_scene   a virtual depth camera ray-casting a room (back wall, floor, side wall,
               a table and 12 boxes / spheres / cylinders in palette colours with
               per-voxel colour noise), ~15 % NaN rays, points snapped to the interior
               [0.1, 0.9] of their leaf cell on every axis and two sentinel points
               pinning the grid to exactly G^3 cells.
parity_cloud   uniform cloud with at most one point per voxel (config 1 "parity mode").
dense_words    100 %-occupancy packed grid with colour = hash(voxel index) (config 5).
random_bases   orthonormal compress axis (F -> D) with descending variances and M model
               subspaces already transformed as readAxis does (MULTIPLE_SIMILARITY).
"""
import numpy as np

BASE_SEED = 0xC3A1AC
_M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def splitmix64(x):
    x = (np.asarray(x, dtype=np.uint64) + np.uint64(0x9E3779B97F4A7C15)) & _M64
    z = x
    with np.errstate(over="ignore"):
        z = ((z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)) & _M64
        z = ((z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)) & _M64
    return z ^ (z >> np.uint64(31))


def uniform(seed, n, stream=0):
    """n uniforms in [0,1) from splitmix64(seed, stream, i)."""
    base = np.uint64((seed * 0x100000001B3 + stream * 0x9E3779B1) & 0xFFFFFFFFFFFFFFFF)
    with np.errstate(over="ignore"):
        ctr = (np.arange(n, dtype=np.uint64) + base) & _M64
    return (splitmix64(ctr) >> np.uint64(11)).astype(np.float64) * (1.0 / 9007199254740992.0)


def pack_rgb(r, g, b):
    """(r,g,b) uint8-valued arrays -> float32 with the packed bits (PCL PointXYZRGB.rgb)."""
    u = (np.asarray(r, np.uint32) << 16) | (np.asarray(g, np.uint32) << 8) | np.asarray(b, np.uint32)
    return u.astype(np.uint32).view(np.float32)


def snap_to_cells(xyz, leaf, lo=0.1, hi=0.9, u=None):
    """Move every coordinate to the interior of its cell (no point on a boundary)."""
    leaf = np.float32(leaf)
    inv = np.float32(1) / leaf
    cell = np.floor(xyz.astype(np.float32) * inv)
    if u is None:
        u = np.full(xyz.shape, 0.5)
    frac = lo + (hi - lo) * u
    out = ((cell.astype(np.float64) + frac) * np.float64(leaf)).astype(np.float32)
    bad = (np.floor(out * inv) != cell) | (np.floor(out / leaf) != cell)
    if bad.any():
        fix = ((cell.astype(np.float64) + 0.5) * np.float64(leaf)).astype(np.float32)
        out[bad] = fix[bad]
    return out


def parity_cloud(n_points=50000, grid=64, leaf=0.01, seed=BASE_SEED, colour_max=254):
    """Config 1: <= 1 point per voxel, uniform colours in [0, colour_max]."""
    nvox = grid ** 3
    n = min(n_points, nvox)
    keys = splitmix64(np.arange(nvox, dtype=np.uint64) + np.uint64(seed))
    cells = np.argsort(keys, kind="stable")[:n].astype(np.int64)
    cells[0], cells[1 % n] = 0, nvox - 1  # sentinels pin the grid to grid^3
    cells = np.unique(cells)
    x, y, z = cells % grid, (cells // grid) % grid, cells // (grid * grid)
    u = uniform(seed, cells.size * 6, stream=1).reshape(6, -1)
    xyz = np.stack([x + 0.1 + 0.8 * u[0], y + 0.1 + 0.8 * u[1], z + 0.1 + 0.8 * u[2]], 1) * leaf
    xyz = snap_to_cells(xyz.astype(np.float32), leaf, u=np.stack([u[0], u[1], u[2]], 1))
    col = np.minimum((u[3:6] * (colour_max + 1)).astype(np.int64), colour_max)
    pts = np.empty((cells.size, 4), np.float32)
    pts[:, :3] = xyz
    pts[:, 3] = pack_rgb(col[0], col[1], col[2])
    order = np.argsort(splitmix64(cells.astype(np.uint64) + np.uint64(7)), kind="stable")
    return pts[order]


PALETTE = np.array([[200, 60, 50], [40, 160, 70], [50, 80, 200], [220, 200, 40], [160, 60, 170],
                    [40, 190, 190], [230, 130, 40], [120, 120, 120], [250, 250, 250], [20, 20, 20],
                    [150, 100, 60], [240, 160, 200], [90, 200, 120], [60, 60, 130]], np.int64)


def _ray_plane(o, d, axis, val):
    den = d[:, axis]
    with np.errstate(divide="ignore", invalid="ignore"):
        t = (val - o[axis]) / den
    t[~np.isfinite(t) | (t <= 0)] = np.inf
    return t


def _ray_box(o, d, lo, hi):
    with np.errstate(divide="ignore", invalid="ignore"):
        inv = 1.0 / d
        t1 = (lo[None, :] - o[None, :]) * inv
        t2 = (hi[None, :] - o[None, :]) * inv
    tmin = np.nanmax(np.minimum(t1, t2), axis=1)
    tmax = np.nanmin(np.maximum(t1, t2), axis=1)
    hit = (tmax >= tmin) & (tmax > 0)
    t = np.where(tmin > 0, tmin, tmax)
    return np.where(hit, t, np.inf)


def _ray_sphere(o, d, c, r):
    oc = o[None, :] - c[None, :]
    b = (oc * d).sum(1)
    cc = (oc * oc).sum(1) - r * r
    disc = b * b - cc
    with np.errstate(invalid="ignore"):
        s = np.sqrt(disc)
    t = -b - s
    t = np.where(t > 0, t, -b + s)
    return np.where((disc >= 0) & (t > 0), t, np.inf)


def _ray_cylinder(o, d, c, r, y0, y1):
    # vertical (y) axis cylinder
    ox, oz = o[0] - c[0], o[2] - c[2]
    a = d[:, 0] ** 2 + d[:, 2] ** 2
    b = ox * d[:, 0] + oz * d[:, 2]
    cc = ox * ox + oz * oz - r * r
    disc = b * b - a * cc
    with np.errstate(invalid="ignore", divide="ignore"):
        s = np.sqrt(disc)
        t = (-b - s) / a
    y = o[1] + t * d[:, 1]
    ok = (disc >= 0) & (t > 0) & (y >= y0) & (y <= y1)
    return np.where(ok, t, np.inf)


def kinect_scene(n_rays=1_000_000, grid=128, leaf=0.02, seed=BASE_SEED, nan_frac=0.15):
    """Config 2/3 generator: (N,4) float32 XYZRGB, all finite points inside [0, grid*leaf)^3."""
    E = grid * leaf
    u = uniform(seed, 64, stream=2)
    W = int(np.sqrt(n_rays * 4 / 3))
    H = max(1, n_rays // W)
    cam = np.array([E * (0.5 + 0.04 * (u[0] - 0.5)), E * (0.45 + 0.04 * (u[1] - 0.5)), -0.35 * E])
    far = 0.985 * E
    half = (0.5 * E) / (far - cam[2])
    px = (np.arange(W) + 0.5) / W * 2 - 1
    py = (np.arange(H) + 0.5) / H * 2 - 1
    PX, PY = np.meshgrid(px * half, py * half * (H / W) * 1.3, indexing="xy")
    d = np.stack([PX.ravel(), PY.ravel(), np.ones(PX.size)], 1)
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    n = d.shape[0]
    t_best = np.full(n, np.inf)
    col = np.zeros(n, np.int64)

    def take(t, c):
        nonlocal t_best
        better = t < t_best
        t_best = np.where(better, t, t_best)
        col[better] = c

    take(_ray_plane(cam, d, 2, far), 7)          # back wall
    take(_ray_plane(cam, d, 1, 0.975 * E), 10)   # floor (y down)
    take(_ray_plane(cam, d, 0, 0.02 * E), 12)    # side wall
    table_lo = np.array([0.25 * E, 0.62 * E, 0.35 * E])
    table_hi = np.array([0.78 * E, 0.66 * E, 0.80 * E])
    take(_ray_box(cam, d, table_lo, table_hi), 13)
    for i in range(12):
        v = uniform(seed, 8, stream=100 + i)
        kind = i % 3
        cx = (0.3 + 0.45 * v[0]) * E
        cz = (0.4 + 0.35 * v[1]) * E
        size = (0.03 + 0.05 * v[2]) * E
        c = int(i % 7)
        if kind == 0:
            lo = np.array([cx - size, 0.62 * E - 2 * size, cz - size])
            hi = np.array([cx + size, 0.62 * E, cz + size])
            take(_ray_box(cam, d, lo, hi), c)
        elif kind == 1:
            take(_ray_sphere(cam, d, np.array([cx, 0.62 * E - size, cz]), size), c)
        else:
            take(_ray_cylinder(cam, d, np.array([cx, 0.0, cz]), 0.7 * size, 0.62 * E - 2.5 * size, 0.62 * E), c)
    xyz = cam[None, :] + t_best[:, None] * d
    finite = np.isfinite(t_best)
    inside = finite & np.all((xyz >= 0) & (xyz < E), axis=1)
    drop = uniform(seed, n, stream=3) < nan_frac
    valid = inside & ~drop
    xyz32 = np.full((n, 3), np.nan, np.float32)
    xyz32[valid] = snap_to_cells(xyz[valid].astype(np.float32), leaf,
                                 u=uniform(seed, int(valid.sum()) * 3, stream=4).reshape(-1, 3))
    # per-voxel colour noise keeps every voxel single-coloured (exact mean for any rule)
    cell = np.floor(xyz32[valid] * (np.float32(1) / np.float32(leaf))).astype(np.int64)
    cid = (cell[:, 0] + grid * (cell[:, 1] + grid * cell[:, 2])).astype(np.uint64)
    h = splitmix64(cid + np.uint64(seed))
    noise = np.stack([(h >> np.uint64(s)) % np.uint64(21) for s in (0, 8, 16)], 1).astype(np.int64) - 10
    rgb = np.clip(PALETTE[col[valid]] + noise, 0, 254)
    out = np.full((n, 4), np.nan, np.float32)
    out[valid, :3] = xyz32[valid]
    out[:, 3] = pack_rgb(np.zeros(n, np.int64), np.zeros(n, np.int64), np.zeros(n, np.int64))
    out[valid, 3] = pack_rgb(rgb[:, 0], rgb[:, 1], rgb[:, 2])
    # sentinels at the centres of cells (0,0,0) and (G-1,G-1,G-1)
    sent = np.array([[0.5 * leaf] * 3, [(grid - 0.5) * leaf] * 3], np.float32)
    sent_rows = np.concatenate([sent, pack_rgb([128, 128], [128, 128], [128, 128])[:, None]], 1)
    return np.concatenate([sent_rows.astype(np.float32), out], 0)


def dense_words(grid, seed=BASE_SEED):
    """Config 5: every voxel occupied, colour = hash(voxel index); words[z,y,x]."""
    idx = np.arange(grid ** 3, dtype=np.uint64)
    h = splitmix64(idx + np.uint64(seed))
    rgb = (h & np.uint64(0xFFFFFF)).astype(np.uint32)
    return ((np.uint32(1) << np.uint32(24)) | rgb).reshape(grid, grid, grid)


def random_words(grid, occupancy, seed=BASE_SEED, colour_max=255):
    """Random packed grid with the given occupancy fraction (words[z,y,x])."""
    shape = (grid, grid, grid) if np.isscalar(grid) else tuple(grid)[::-1]
    n = int(np.prod(shape))
    u = uniform(seed, n, stream=5)
    h = splitmix64(np.arange(n, dtype=np.uint64) + np.uint64(seed * 3 + 1))
    r = (h & np.uint64(255)).astype(np.uint32) % (colour_max + 1)
    g = ((h >> np.uint64(8)) & np.uint64(255)).astype(np.uint32) % (colour_max + 1)
    b = ((h >> np.uint64(16)) & np.uint64(255)).astype(np.uint32) % (colour_max + 1)
    w = (np.uint32(1) << np.uint32(24)) | (r << 16) | (g << 8) | b
    return np.where(u < occupancy, w, np.uint32(0)).astype(np.uint32).reshape(shape)


def _orthonormal(rng, rows, cols):
    q, r = np.linalg.qr(rng.standard_normal((rows, cols)))
    return q * np.sign(np.diag(r))[None, :]


def random_bases(F, D, M, r, seed=BASE_SEED):
    """-> axis_t (D,F) float32 (setSceneAxis input, not yet whitened), var (D,),
    axis_q (M,r,D) float32 after readAxis' MULTIPLE_SIMILARITY transform."""
    rng = np.random.Generator(np.random.PCG64(seed))
    axis = _orthonormal(rng, F, D)                      # columns = eigenvectors
    var = (10.0 * 0.93 ** np.arange(D)).astype(np.float32)
    qs = []
    for m in range(M):
        A = _orthonormal(rng, D, D)
        v = (5.0 * 0.85 ** np.arange(D)).astype(np.float64)
        q = A[:, :r].T.astype(np.float32)
        for i in range(1, r):
            q[i] = (q[i].astype(np.float64) * np.sqrt(np.float32(v[i])) / np.sqrt(np.float32(v[0]))).astype(np.float32)
        qs.append(q)
    return axis.T.astype(np.float32).copy(), var, np.stack(qs).astype(np.float32)


def whiten(axis_t, var):
    """setSceneAxis(axis, var, dim) whitening (search.cpp:701-712), float."""
    w = (1.0 / np.sqrt(var.astype(np.float64))).astype(np.float32)
    return (axis_t * w[:, None]).astype(np.float32)
